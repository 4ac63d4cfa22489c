#!/bin/bash
# n32 default line: Pipeline depth (slots; rounded to a multiple of the lanes) 4 vs 8, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03aj; export TMPDIR=/tmp
for r in 1 2 3; do
  for dp in 2 8; do
    FCE_PIPE_DEPTH=$dp timeout -k 10 300 python bench.py --cpu-seconds 0 --predict-steps 0 --profile-passes 1 > gpurun_out/r03aj/d${dp}_$r.log 2>&1 || exit $?
    echo "depth$dp r$r $(tail -1 gpurun_out/r03aj/d${dp}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
