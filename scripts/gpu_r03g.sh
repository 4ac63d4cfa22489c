#!/bin/bash
# dense C2f chunk copy (dup store) + predictor: tests, then bench with / without the dup store, predictor diag.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu.py tests/test_prepost.py -v -m gpu -rf --timeout 200 --timeout-method thread \
  -k "dense_chunk or every_op_variant or predictor or end_to_end_parity or batch_invariance" > gpurun_out/pytest_g.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_g.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for mode in 0 1 0 1; do
  FCE_DUP=$mode timeout -k 10 200 python bench.py --steps 40 --warmup 10 --cpu-seconds 0 --profile-passes 3 --predict-steps 30 > gpurun_out/bench_g$mode.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
  python -c "
import json; d=json.loads(open('gpurun_out/bench_g$mode.log').read().strip().splitlines()[-1]); k=d['kernels']
print('FCE_DUP=$mode', d['value'], 'fwd', d['forward_ms_per_batch'], 'c3', k['conv3x3_mfma']['ms'], k['conv3x3_mfma']['GB/s'], 'c1', k['conv1x1_mfma']['ms'], 'pred', d['predict_pcie_inclusive']['images_per_sec'])"
done
timeout -k 10 300 python scripts/predict_diag.py > gpurun_out/predict_diag.log 2>&1
rc=$?; echo "diag rc=$rc"; grep Predictor gpurun_out/predict_diag.log
exit $rc
