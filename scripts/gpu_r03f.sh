#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_prepost.py -v -m gpu -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_f.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_f.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/predict_diag.py > gpurun_out/predict_diag.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/predict_diag.log | grep Predictor
exit $rc
