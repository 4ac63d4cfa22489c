#!/bin/bash
# Headline bench under several environment settings, one process each: gpu_bench_env.sh TAG "ENV..." ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/benv; export TMPDIR=/tmp
TAG=$1; shift
for SET in "$@"; do
  name=$(echo "$SET" | tr ' =' '_-'); [ -z "$name" ] && name=default
  env $SET timeout -k 10 200 python bench.py --steps 40 --warmup 10 --cpu-seconds 0 --predict-steps 0 --profile-passes 1 > gpurun_out/benv/${TAG}_${name}.log 2>&1
  rc=$?; echo "[$SET] rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"forward_ms_per_batch": [0-9.]*' gpurun_out/benv/${TAG}_${name}.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
done
