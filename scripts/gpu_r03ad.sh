#!/bin/bash
# RCCL path (one rank, FCE_DIST_FORCE=1): 3 lanes x 4 queues vs 4 lanes x 8 queues vs 4 x 16, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03ad; export TMPDIR=/tmp
run() { local tag=$1 port=$2; shift 2; FCE_DIST_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port $port bench.py --steps 40 --warmup 10 --cpu-seconds 0 --predict-steps 0 --profile-passes 1 "$@" \
  > gpurun_out/r03ad/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc $(tail -1 gpurun_out/r03ad/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["batches_in_flight"], d["config"]["hw_queues"])')"; return $rc; }
for r in 1 2; do
  run l3_$r 2950$r --lanes 3 && run l4_$r 2951$r --lanes 4 && GPU_MAX_HW_QUEUES=16 run l4q16_$r 2952$r --lanes 4 || exit $?
done
