#!/bin/bash
# n32 bench with the fused C3k2 kernel on blocks up to a spatial size (FCE_FUSE_C3K2: 0 off, 1 all, N: h*w <= N)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/fz
for F in 0 400 1600 6400 1 0; do
  FCE_FUSE_C3K2=$F timeout -k 10 200 python bench.py --steps 40 --warmup 5 --cpu-seconds 0 --predict-steps 0 \
    --profile-passes 3 "$@" > gpurun_out/fz/f$F.log 2>&1 || exit 1
  echo "fuse $F $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"forward_ms_per_batch": [0-9.]*' gpurun_out/fz/f$F.log | tr '\n' ' ')"
done
