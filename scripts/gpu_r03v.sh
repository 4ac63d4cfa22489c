#!/bin/bash
# 64-cout-per-wave big tiles (0xB80 / 0xC80 ...): variant tests, l32 / m16 tune reports and config benches; then the
# n32 NMS-in-pipeline A/B (scripts/gpu_r03u.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03v; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q -m gpu -k "variant" --timeout 300 --timeout-method thread > gpurun_out/r03v/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03v/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tune_report.py --model yolo11l-fce.yaml --batch 32 --imgsz 640 > gpurun_out/r03v/l32_tune.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/tune_report.py --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 > gpurun_out/r03v/m16_tune.txt 2>&1 || exit $?
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --predict-steps 0 "$@" > gpurun_out/r03v/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc $(tail -1 gpurun_out/r03v/$tag.log | cut -c1-200)"; return $rc; }
run l32 --model yolo11l-fce.yaml --batch 32 --imgsz 640 &&
run m16 --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 &&
run s32 --model yolo11s-bifpn.yaml --batch 32 --imgsz 640 || exit $?
bash scripts/gpu_r03u.sh
