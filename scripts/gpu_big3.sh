#!/bin/bash
# Big-tile LDS-DMA 3x3 (0x8x0) against the tuned tile variants on the m/l shapes, then the bitwise variant tests.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/big3; export TMPDIR=/tmp
P="timeout -k 10 120 python scripts/conv_probe.py --reps 10"
run() { echo "== $*"; $P "$@" || exit $?; }
{
run --cin 256 --cout 256 --hw 80 --batch 32 --codes 0x2142,0x810,0x820,0x2810,0x2820,0x3820
run --cin 256 --cout 256 --hw 160 --stride 2 --batch 32 --codes 0x2141,0x820,0x1820
run --cin 512 --cout 512 --hw 40 --batch 32 --codes 0x2142,0x810,0x820,0x2810,0x2820,0x3820
run --cin 512 --cout 512 --hw 80 --stride 2 --batch 32 --codes 0x2141,0x820,0x1820
run --cin 128 --cout 128 --hw 160 --batch 32 --codes 0x2142,0x810,0x820,0x2810,0x2820,0x3820
run --cin 256 --cout 256 --hw 160 --batch 16 --codes 0x2142,0x810,0x820,0x2810,0x2820,0x3820
} > gpurun_out/big3/probe.txt 2>&1
rc=$?; cat gpurun_out/big3/probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q -k "conv_every_variant" --timeout 120 --timeout-method thread > gpurun_out/big3/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/big3/pytest.log; exit $rc
