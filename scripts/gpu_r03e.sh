#!/bin/bash
# Wide-tile 3x3: bitwise variant tests, then per-shape timings of every candidate on the l / m 3x3 shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/probe
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -v -m gpu -rf --timeout 120 --timeout-method thread \
  -k "conv_every_variant or mfma_conv_exact" > gpurun_out/pytest_e.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_e.log | tail -8
[ $rc -eq 0 ] || exit $rc
for shp in "256 256 2 160 32" "512 512 2 80 32" "64 128 2 320 32" "512 512 2 40 32" "256 256 1 80 32" "64 64 1 80 32" "128 128 1 40 32" "256 256 1 20 32" "256 256 1 160 16" "512 512 1 80 16"; do
  set -- $shp
  timeout -k 10 120 python scripts/conv_probe.py --cin $1 --cout $2 --stride $3 --hw $4 --batch $5 --reps 10 > gpurun_out/probe/w_$1_$2_$3_$4_$5.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "probe $shp rc=$rc"; exit $rc; }
  echo "== cin $1 cout $2 s$3 hw $4 bs $5"; grep -v amdgpu.ids gpurun_out/probe/w_$1_$2_$3_$4_$5.txt | sort -k2 -n | head -6
  grep "0xa" gpurun_out/probe/w_$1_$2_$3_$4_$5.txt
done
