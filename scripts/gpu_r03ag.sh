#!/bin/bash
# n32 default line: timed steps 50 vs 200 (pipeline fill / drain amortisation), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03ag; export TMPDIR=/tmp
for r in 1 2 3; do
  for k in 50 200; do
    timeout -k 10 300 python bench.py --steps $k --warmup 10 --cpu-seconds 0 --predict-steps 0 --profile-passes 1 > gpurun_out/r03ag/k${k}_$r.log 2>&1 || exit $?
    echo "k$k r$r $(tail -1 gpurun_out/r03ag/k${k}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
