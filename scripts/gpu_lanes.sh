#!/bin/bash
# bench.py at several --lanes values (batches in flight per GPU) for one config.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ln; TAG=$1; LANES=$2; shift 2
for L in $LANES; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --predict-steps 0 --profile-passes 1 --lanes $L "$@" > gpurun_out/ln/${TAG}_l$L.log 2>&1 || exit 1
  echo "$TAG lanes $L $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/ln/${TAG}_l$L.log | tr '\n' ' ')"
done
