#!/bin/bash
# big-tile implicit GEMM K-loop schedules (FCE_BIG_PF 0 / 1 / 2) on the l32 / m16 downsampling convs and wide 1x1s
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03p
for pf in 1 0 2; do
  export FCE_BIG_PF=$pf
  run() { tag=$1; shift; timeout -k 10 120 python scripts/conv_probe.py "$@" > gpurun_out/r03p/${tag}_pf$pf.txt 2>&1 || { cat gpurun_out/r03p/${tag}_pf$pf.txt; exit 1; }; echo "== pf$pf $tag $*"; grep -v amdgpu.ids gpurun_out/r03p/${tag}_pf$pf.txt; }
  run l18 --cin 256 --cout 256 --k 3 --stride 2 --hw 160 --batch 32 --codes 0xc00,0xc10,0x2141
  run l36 --cin 512 --cout 512 --k 3 --stride 2 --hw 80 --batch 32 --codes 0xc00,0xc10,0x2141
  run s1 --cin 256 --cout 256 --k 3 --stride 1 --hw 80 --batch 32 --codes 0xc00,0xc10,0x2142
  run m18 --cin 256 --cout 256 --k 3 --stride 2 --hw 320 --batch 16 --codes 0xc00,0xc10,0x2144
  run p512 --cin 512 --cout 512 --k 1 --hw 80 --batch 32 --codes 0xb00,0xb10,0x1700
done
