#!/bin/bash
# coord projection unrolled by 4: coord GPU tests, then per-kernel times at the l32 / m16 L5 shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -m gpu -k "bicoord or coord or e2e or full_size" --timeout 120 --timeout-method thread > gpurun_out/coord_tests.log 2>&1
rc=$?; tail -3 gpurun_out/coord_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r03m.sh
