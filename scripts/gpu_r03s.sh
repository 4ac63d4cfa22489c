#!/bin/bash
# l32 / m16 / n32 benches with the 4-wave big tiles and band pooling, then l32 / m16 PMC passes (hbm/alg, MFMA busy)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03s; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/tune_report.py --model yolo11l-fce.yaml --batch 32 --imgsz 640 > gpurun_out/r03s/l32_tune.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/tune_report.py --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 > gpurun_out/r03s/m16_tune.txt 2>&1 || exit $?
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 "$@" > gpurun_out/r03s/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc"; tail -1 gpurun_out/r03s/$tag.log | cut -c1-240; echo; return $rc; }
run l32 --model yolo11l-fce.yaml --batch 32 --imgsz 640 &&
run m16 --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 &&
run n32 --steps 20 --predict-steps 0 || exit $?
bash scripts/gpu_pmc.sh l32g --model yolo11l-fce.yaml --batch 32 --imgsz 640 &&
bash scripts/gpu_pmc.sh m16g --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280
