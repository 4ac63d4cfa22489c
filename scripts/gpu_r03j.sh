#!/bin/bash
# big 1x1 stall breakdown: no stores / no copies / no MFMAs (FCE_BIG1_DIAG, diagnostics), 512 -> 512 at 80^2 bs 32
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/probe
for d in 0 1 2 3; do
  FCE_BIG1_DIAG=$d timeout -k 10 60 python scripts/conv_probe.py --k 1 --cin 512 --cout 512 --hw 80 --batch 32 --reps 20 --codes 0xb10,0xb00 > gpurun_out/probe/diag$d.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "diag $d rc=$rc"; exit $rc; }
  echo "DIAG=$d"; grep -v amdgpu.ids gpurun_out/probe/diag$d.txt
done
