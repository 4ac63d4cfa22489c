#!/bin/bash
# BiCoord image chunks sized for the Infinity Cache: per-call time at the l32 / m16 L5 shapes per chunk size
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cc
for mb in 0 32 64 112 160; do
  FCE_COORD_CHUNK_MB=$mb timeout -k 10 120 python scripts/coord_bench.py 100 > gpurun_out/cc/c$mb.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "chunk $mb rc=$rc"; cat gpurun_out/cc/c$mb.txt; exit $rc; }
  echo "CHUNK_MB=$mb"; grep -v amdgpu.ids gpurun_out/cc/c$mb.txt
done
