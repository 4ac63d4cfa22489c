#!/bin/bash
# n32, 4 lanes x 8 queues: hipGraph replay vs direct launches, interleaved rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03z; export TMPDIR=/tmp
run() { local tag=$1; shift; timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 --predict-steps 0 --profile-passes 1 "$@" > gpurun_out/r03z/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc $(tail -1 gpurun_out/r03z/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["forward_launch"], d["config"]["hw_queues"])')"; return $rc; }
for r in 1 2 3; do
  run g1_$r && run g0_$r --graph 0 || exit $?
done
