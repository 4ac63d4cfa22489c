#!/bin/bash
# XCD-aware gate grid: coord / e2e tests, coord timings, l32 / m16 PMC (bicoord hbm/alg)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03t; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q -m gpu -k "bicoord or coord or e2e or full_size or variant" --timeout 300 --timeout-method thread > gpurun_out/r03t/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03t/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/coord_bench.py > gpurun_out/r03t/coord.txt 2>&1 || exit $?; grep -v amdgpu gpurun_out/r03t/coord.txt
bash scripts/gpu_pmc.sh l32h --model yolo11l-fce.yaml --batch 32 --imgsz 640 &&
bash scripts/gpu_pmc.sh m16h --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 &&
bash scripts/gpu_pmc.sh n32h
