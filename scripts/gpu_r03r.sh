#!/bin/bash
# HBM-bound m/l layers in isolation (1x1 192->256 / 128->128 at 320^2, 3x3 s2 64->128 at 640^2, bs 16; l op 17 / 18)
# with the 4-wave two-blocks-per-CU big tiles (0xB40 / 0xC40 ...), against the box's copy rate; variant tests first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03r; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q -m gpu -k "variant" --timeout 300 --timeout-method thread > gpurun_out/r03r/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03r/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/bw_probe.py > gpurun_out/r03r/bw.txt 2>&1 || exit $?; grep -v amdgpu gpurun_out/r03r/bw.txt
run() { tag=$1; shift; timeout -k 10 180 python scripts/conv_probe.py "$@" > gpurun_out/r03r/$tag.txt 2>&1 || { cat gpurun_out/r03r/$tag.txt; exit 1; }; echo "== $tag $*"; grep -v amdgpu.ids gpurun_out/r03r/$tag.txt | sort -k2 -n | head -8; }
run m10 --cin 192 --cout 256 --k 1 --hw 320 --batch 16
run m2 --cin 128 --cout 128 --k 1 --hw 320 --batch 16
run m1 --cin 64 --cout 128 --k 3 --stride 2 --hw 640 --batch 16
run l17 --cin 256 --cout 256 --k 1 --hw 160 --batch 32
run l18 --cin 256 --cout 256 --k 3 --stride 2 --hw 160 --batch 32
run l36 --cin 512 --cout 512 --k 3 --stride 2 --hw 80 --batch 32
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q -m gpu -k "bicoord or coord or e2e or full_size" --timeout 300 --timeout-method thread > gpurun_out/r03r/coord_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03r/coord_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== coord band pooling"; timeout -k 10 120 python scripts/coord_bench.py > gpurun_out/r03r/coord_band.txt 2>&1 || exit $?; grep -v amdgpu gpurun_out/r03r/coord_band.txt
echo "== coord two-pass pooling"; FCE_COORD_TWO_PASS=1 timeout -k 10 120 python scripts/coord_bench.py > gpurun_out/r03r/coord_2p.txt 2>&1 || exit $?; grep -v amdgpu gpurun_out/r03r/coord_2p.txt
