#!/bin/bash
# 256-wide-tile 1x1: bitwise variant tests, model-level variant pinning, then per-shape timings on m/l 1x1 shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/probe
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -v -m gpu -rf --timeout 300 --timeout-method thread \
  -k "conv_every_variant or conv1x1_variants or every_op_variant or end_to_end_parity or detect" > gpurun_out/pytest_h.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_h.log | tail -8
[ $rc -eq 0 ] || exit $rc
for shp in "512 512 80 32" "256 512 160 32" "512 256 80 32" "1024 512 40 32" "256 256 160 16" "1024 512 80 16" "768 256 40 32" "384 128 80 32" "128 256 160 32"; do
  set -- $shp
  timeout -k 10 120 python scripts/conv_probe.py --k 1 --cin $1 --cout $2 --hw $3 --batch $4 --reps 10 > gpurun_out/probe/b1_$1_$2_$3_$4.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "probe $shp rc=$rc"; exit $rc; }
  echo "== 1x1 cin $1 cout $2 hw $3 bs $4"; grep -v amdgpu.ids gpurun_out/probe/b1_$1_$2_$3_$4.txt | sort -k2 -n | head -4
  grep "0xb" gpurun_out/probe/b1_$1_$2_$3_$4.txt
done
