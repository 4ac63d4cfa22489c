#!/bin/bash
# implicit-GEMM big-tile 3x3 (0xC00 / 0xC10) and the raw-barrier big 1x1 (0xB00 / 0xB10): variant tests, then
# per-shape timings against the other candidates on the l32 / m16 downsampling convs and a wide 1x1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03o
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q -m gpu -k "every_variant" --timeout 300 --timeout-method thread > gpurun_out/r03o/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03o/tests.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; shift; timeout -k 10 180 python scripts/conv_probe.py "$@" > gpurun_out/r03o/$tag.txt 2>&1 || { cat gpurun_out/r03o/$tag.txt; exit 1; }; echo "== $tag $*"; grep -v amdgpu.ids gpurun_out/r03o/$tag.txt | sort -k2 -n | head -8; }
run l18 --cin 256 --cout 256 --k 3 --stride 2 --hw 160 --batch 32
run l36 --cin 512 --cout 512 --k 3 --stride 2 --hw 80 --batch 32
run l54 --cin 512 --cout 512 --k 3 --stride 2 --hw 40 --batch 32
run l1 --cin 64 --cout 128 --k 3 --stride 2 --hw 320 --batch 32
run s1 --cin 256 --cout 256 --k 3 --stride 1 --hw 80 --batch 32
run m18 --cin 256 --cout 256 --k 3 --stride 2 --hw 320 --batch 16
run p512 --cin 512 --cout 512 --k 1 --hw 80 --batch 32
run p256 --cin 256 --cout 256 --k 1 --hw 160 --batch 32
