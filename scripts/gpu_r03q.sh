#!/bin/bash
# implicit-GEMM 3x3 in the l32 / m16 models: variant tests, per-op tune reports, config benches with and without
# the 0xC00 candidates on one box (FCE_NO_GEMM3=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03q; export TMPDIR=/tmp
:
:
:
timeout -k 10 300 python -u scripts/tune_report.py --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 > gpurun_out/r03q/m16_tune.txt 2>&1 || exit $?
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 "$@" > gpurun_out/r03q/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc"; tail -1 gpurun_out/r03q/$tag.log | cut -c1-330; echo; return $rc; }
run l32 --model yolo11l-fce.yaml --batch 32 --imgsz 640 &&
FCE_NO_GEMM3=1 run l32_nogemm --model yolo11l-fce.yaml --batch 32 --imgsz 640 &&
run m16 --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 &&
FCE_NO_GEMM3=1 run m16_nogemm --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280
