#!/bin/bash
# s-bifpn 640 bs32: 3 lanes x 4 queues vs 4 lanes x 8 queues, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03ak; export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python bench.py --model yolo11s-bifpn.yaml --cpu-seconds 0 --predict-steps 0 --profile-passes 1 --steps 100 > gpurun_out/r03ak/l3_$r.log 2>&1 || exit $?
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --model yolo11s-bifpn.yaml --lanes 4 --cpu-seconds 0 --predict-steps 0 --profile-passes 1 --steps 100 > gpurun_out/r03ak/l4_$r.log 2>&1 || exit $?
  for t in l3 l4; do echo "$t r$r $(tail -1 gpurun_out/r03ak/${t}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["batches_in_flight"], d["config"]["hw_queues"])')"; done
done
