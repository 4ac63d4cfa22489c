#!/bin/bash
# n32 bench at several lanes x GPU_MAX_HW_QUEUES (hardware queues per process; HIP default 4).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/hq
for Q in 4 8 16; do
  for L in 3 4 6; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 200 python bench.py --steps 40 --warmup 5 --cpu-seconds 0 --predict-steps 0 \
      --profile-passes 1 --lanes $L > gpurun_out/hq/q${Q}_l$L.log 2>&1 || exit 1
    echo "queues $Q lanes $L $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/hq/q${Q}_l$L.log | tr '\n' ' ')"
  done
done
