#!/bin/bash
# conv_probe timings + SQ counter passes over a few variants of one conv shape (kernel trace only).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/probe; export TMPDIR=/tmp
TAG=${1:-p}; CODES=${2:-0x2141,0x8122,0x142,0x2144}; shift 2
timeout -k 10 120 python scripts/conv_probe.py "$@" > gpurun_out/probe/${TAG}_all.txt 2>&1 || exit $?
cat gpurun_out/probe/${TAG}_all.txt | sort -k2 -n | head -12
[ -n "$PMC" ] || exit 0
i=0
for set in "$PMC" "$PMC2"; do
  [ -n "$set" ] || continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/probe/${TAG}_pmc$i -o run -- \
    python scripts/conv_probe.py --codes $CODES --reps 3 "$@" > gpurun_out/probe/${TAG}_pmc$i.log 2>&1 || exit $?
done
python scripts/pmc_by_kernel.py gpurun_out/probe/${TAG}_pmc1 gpurun_out/probe/${TAG}_pmc2 > gpurun_out/probe/${TAG}_pmc.txt 2>&1; cat gpurun_out/probe/${TAG}_pmc.txt
