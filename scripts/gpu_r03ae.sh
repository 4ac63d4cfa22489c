#!/bin/bash
# defaults after the process-group rule: one-rank RCCL path (3 lanes x 4 queues expected) and the plain N=1 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03ae; export TMPDIR=/tmp
FCE_DIST_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --steps 40 --warmup 10 --cpu-seconds 0 --predict-steps 0 --profile-passes 1 > gpurun_out/r03ae/rccl1.log 2>&1
rc=$?; echo "rccl1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 40 --warmup 10 --cpu-seconds 0 --predict-steps 0 --profile-passes 1 > gpurun_out/r03ae/n1.log 2>&1
rc=$?; echo "n1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for f in rccl1 n1; do tail -1 gpurun_out/r03ae/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"], d["process_group"])'; done
