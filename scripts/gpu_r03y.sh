#!/bin/bash
# split rings (deep pixel ring, 0xB20 family) for the HBM-bound m/l 1x1s: variant tests, isolated shapes,
# m16 / l32 tune reports and benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03y; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q -m gpu -k "variant" --timeout 300 --timeout-method thread > gpurun_out/r03y/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03y/tests.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; shift; timeout -k 10 180 python scripts/conv_probe.py "$@" > gpurun_out/r03y/$tag.txt 2>&1 || { cat gpurun_out/r03y/$tag.txt; exit 1; }; echo "== $tag $*"; grep -v amdgpu.ids gpurun_out/r03y/$tag.txt | sort -k2 -n | head -6; }
run m10 --cin 192 --cout 256 --k 1 --hw 320 --batch 16
run m2 --cin 128 --cout 128 --k 1 --hw 320 --batch 16
run l17 --cin 256 --cout 256 --k 1 --hw 160 --batch 32
run m20 --cin 384 --cout 256 --k 1 --hw 160 --batch 16
timeout -k 10 300 python -u scripts/tune_report.py --model yolo11l-fce.yaml --batch 32 --imgsz 640 > gpurun_out/r03y/l32_tune.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/tune_report.py --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 > gpurun_out/r03y/m16_tune.txt 2>&1 || exit $?
b() { local tag=$1; shift; timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --predict-steps 0 "$@" > gpurun_out/r03y/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc $(tail -1 gpurun_out/r03y/$tag.log | cut -c1-200)"; return $rc; }
b l32 --model yolo11l-fce.yaml --batch 32 --imgsz 640 --lanes 3 &&
b m16 --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 --lanes 3 &&
b l32_4 --model yolo11l-fce.yaml --batch 32 --imgsz 640 &&
b m16_4 --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280
