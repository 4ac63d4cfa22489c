#!/bin/bash
# predict leg after releasing the main line's lanes: three default bench runs (value + predict_pcie_inclusive)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03af; export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --profile-passes 1 > gpurun_out/r03af/b$r.log 2>&1 || exit $?
  tail -1 gpurun_out/r03af/b$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["predict_pcie_inclusive"]["images_per_sec"])'
done
