#!/bin/bash
# Graph replay vs direct launches on the headline bench (after the per-(in, out) graph cache), plus the
# BASELINE-size C2PSA parity cases.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/exp; export TMPDIR=/tmp
run() { tag=$1; shift; timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 --predict-steps 0 --profile-passes 1 "$@" > gpurun_out/exp/$tag.log 2>&1; rc=$?; echo "$tag rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"forward_ms_per_batch": [0-9.]*' gpurun_out/exp/$tag.log | tr '\n' ' ')"; return $rc; }
timeout -k 10 300 python -u -m pytest tests -q -m gpu -k "full_size_op_parity or graph_eager" --timeout 200 --timeout-method thread > gpurun_out/exp/pytest.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/exp/pytest.log
run direct && run graph --graph 1 && run direct2 && run graph2 --graph 1 && run direct_nonms --no-nms && run graph_nonms --graph 1 --no-nms
