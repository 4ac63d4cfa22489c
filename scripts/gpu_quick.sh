#!/bin/bash
# Quick iteration pass: a pytest -k selection, then the headline bench (no CPU baseline / predict leg).
# usage: gpu_quick.sh "<pytest -k expr>" [tag]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
K=${1:-coord}; TAG=${2:-quick}
timeout -k 10 600 python -u -m pytest tests -q -m gpu -k "$K" --timeout 200 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-seconds 0 --predict-steps 0 --profile-json gpurun_out/${TAG}_profile.json > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"forward_ms_per_batch": [0-9.]*' gpurun_out/${TAG}_bench.log | tr '\n' ' '; echo
exit $rc
