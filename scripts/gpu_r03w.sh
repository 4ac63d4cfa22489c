#!/bin/bash
# n32 headline: lanes x GPU_MAX_HW_QUEUES, interleaved rounds on one box (value of the default bench step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03w; export TMPDIR=/tmp
run() { local tag=$1 q=$2; shift 2; GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 --predict-steps 0 --profile-passes 1 "$@" > gpurun_out/r03w/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc $(tail -1 gpurun_out/r03w/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; return $rc; }
for r in 1 2 3; do
  run l3q4_$r 4 --lanes 3 && run l4q8_$r 8 --lanes 4 && run l3q8_$r 8 --lanes 3 && run l4q16_$r 16 --lanes 4 && run l5q16_$r 16 --lanes 5 || exit $?
done
