# Pipeline / launch-mode sweep of the headline bench (one process per setting, each under its own limit).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/exp; export TMPDIR=/tmp
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --steps 30 --warmup 5 --cpu-seconds 0 --predict-steps 0 ${BARGS} > gpurun_out/exp/$tag.log 2>&1; rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"forward_ms_per_batch": [0-9.]*' gpurun_out/exp/$tag.log | tr '\n' ' ')"; return $rc; }
run d2 FCE_PIPE_DEPTH=2 && run d3 FCE_PIPE_DEPTH=3 && run d4 FCE_PIPE_DEPTH=4 && BARGS="--graph 1" run graph FCE_PIPE_DEPTH=2 && run d2b FCE_PIPE_DEPTH=2
