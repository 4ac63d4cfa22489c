#!/bin/bash
# big-tile implicit GEMM stall breakdown (FCE_BIG1_DIAG: 1 no stores, 2 no copies after the prologue, 3 no MFMAs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03d2
for d in 0 1 2 3; do
  for shp in "l18 --cin 256 --cout 256 --k 3 --stride 2 --hw 160 --batch 32" "l36 --cin 512 --cout 512 --k 3 --stride 2 --hw 80 --batch 32" "p512 --cin 512 --cout 512 --k 1 --hw 80 --batch 32"; do
    set -- $shp; tag=$1; shift
    FCE_BIG1_DIAG=$d timeout -k 10 120 python scripts/conv_probe.py "$@" --codes 0xc10,0xc50,0xb10,0xb50 > gpurun_out/r03d2/${tag}_d$d.txt 2>&1
    echo "== diag $d $tag"; grep -v amdgpu gpurun_out/r03d2/${tag}_d$d.txt | grep -v skipped
  done
done
