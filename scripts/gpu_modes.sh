#!/bin/bash
# Forward-only bench of the executor's launch modes: direct (1 stream), DAG over 2 / 3 streams, hipGraph.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/modes; TAG=${1:-m}; shift
b() { local t=$1; shift; timeout -k 10 200 python bench.py --steps 30 --warmup 5 --cpu-seconds 0 --predict-steps 0 --profile-passes 1 --no-nms "$@" > gpurun_out/modes/${TAG}_$t.log 2>&1 || return $?; echo "$t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/modes/${TAG}_$t.log)"; }
b direct "$@" && FCE_STREAMS=2 b dag2 "$@" && FCE_STREAMS=3 b dag3 "$@" && b graph --graph 1 "$@"
