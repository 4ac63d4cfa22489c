#!/bin/bash
# Multi-workgroup NMS: every NMS test (bitwise vs reference / oracle), v1 vs v2 timing, predictor tests, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_prepost.py -v -m gpu -rf --timeout 120 --timeout-method thread \
  -k "nms or predictor or pipeline or fused_best" > gpurun_out/pytest_c.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "score err|passed|failed|FAILED" gpurun_out/pytest_c.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python scripts/nms_bench.py > gpurun_out/nms_bench.log 2>&1
rc=$?; echo "nms_bench rc=$rc"; cat gpurun_out/nms_bench.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 40 --warmup 10 --cpu-seconds 0 --profile-passes 3 > gpurun_out/bench_c.log 2>&1
rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.loads(open('gpurun_out/bench_c.log').read().strip().splitlines()[-1]); print(d['value'], d['value_1lane'], d['kernels']['nms'], d['predict_pcie_inclusive']['images_per_sec'])"
exit $rc
