#!/bin/bash
# n32 step with 3 lanes: default NMS vs the multi-workgroup NMS (FCE_NMS_V2=1) vs forward only; 4 lanes x 8 queues
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03u; export TMPDIR=/tmp
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --steps 40 --warmup 10 --cpu-seconds 0 --predict-steps 0 "$@" > gpurun_out/r03u/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc $(tail -1 gpurun_out/r03u/$tag.log | cut -c1-200)"; return $rc; }
for i in 1 2; do
run base$i && FCE_NMS_V2=1 run v2_$i && run nonms$i --no-nms || exit $?
done
GPU_MAX_HW_QUEUES=8 run l4q8 --lanes 4 || exit $?
timeout -k 10 120 python scripts/nms_bench.py > gpurun_out/r03u/nms_bench.txt 2>&1; echo "nms_bench rc=$?"; grep -v amdgpu gpurun_out/r03u/nms_bench.txt | tail -8
