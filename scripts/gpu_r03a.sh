#!/bin/bash
# Round-3 pass: GPU parity suite (new: e2e NMS indices vs the reference, 3-lane graph pipeline, batch
# invariance at every config), smoke, bench, and the self-launching `bench.py --gpus 2` rehearsed over gloo
# on the one GPU.  Stops at the first GPU fault / abort / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
bash scripts/gpu_check.sh
rc=$?; ok $rc || exit $rc
FCE_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --cpu-seconds 0 \
  --predict-steps 0 --profile-passes 2 > gpurun_out/bench_gloo2.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; tail -3 gpurun_out/bench_gloo2.log
exit $rc
