#!/bin/bash
# split rings for the 3x3 big tiles (0xC20 family): variant tests, stride-2 shapes, l32 / m16 tune + benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03aa; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q -m gpu -k "variant" --timeout 300 --timeout-method thread > gpurun_out/r03aa/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03aa/tests.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; shift; timeout -k 10 180 python scripts/conv_probe.py "$@" > gpurun_out/r03aa/$tag.txt 2>&1 || { cat gpurun_out/r03aa/$tag.txt; exit 1; }; echo "== $tag $*"; grep -v amdgpu.ids gpurun_out/r03aa/$tag.txt | sort -k2 -n | head -5; }
run l18 --cin 256 --cout 256 --k 3 --stride 2 --hw 160 --batch 32 --codes 0xc10,0xc30,0xc50,0xc70,0xcd0,0xcf0
run l36 --cin 512 --cout 512 --k 3 --stride 2 --hw 80 --batch 32 --codes 0xc10,0xc30,0xc50,0xc70,0xcd0,0xcf0
run m11 --cin 256 --cout 512 --k 3 --stride 2 --hw 320 --batch 16 --codes 0xc10,0xc30,0xc50,0xc70,0xcd0,0xcf0
run s1 --cin 256 --cout 256 --k 3 --stride 1 --hw 80 --batch 32 --codes 0xc10,0xc30,0xc50,0xc70,0xcd0,0xcf0,0x2142
timeout -k 10 300 python -u scripts/tune_report.py --model yolo11l-fce.yaml --batch 32 --imgsz 640 > gpurun_out/r03aa/l32_tune.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/tune_report.py --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280 > gpurun_out/r03aa/m16_tune.txt 2>&1 || exit $?
b() { local tag=$1; shift; timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --predict-steps 0 "$@" > gpurun_out/r03aa/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc $(tail -1 gpurun_out/r03aa/$tag.log | cut -c1-200)"; return $rc; }
b l32 --model yolo11l-fce.yaml --batch 32 --imgsz 640 && b m16 --model yolo11m-fce-h8.yaml --batch 16 --imgsz 1280
