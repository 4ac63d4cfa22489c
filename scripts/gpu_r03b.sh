#!/bin/bash
# Targeted pass: e2e NMS indices, predictor tests, bench with the streaming predictor leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_prepost.py -v -m gpu -rf --timeout 120 --timeout-method thread \
  -k "end_to_end_nms or predictor or letterbox" > gpurun_out/pytest_b.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "score err|passed|failed" gpurun_out/pytest_b.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --profile-passes 2 > gpurun_out/bench_b.log 2>&1
rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.loads(open('gpurun_out/bench_b.log').read().strip().splitlines()[-1]); print(d['value'], d['value_1lane'], d['predict_pcie_inclusive'])"
exit $rc
