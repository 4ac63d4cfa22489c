#!/bin/bash
# Forward time of the captured graph with its op DAG spread over 1 / 2 / 4 / 8 streams.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 30 --warmup 5 --cpu-seconds 0 > gpurun_out/sweep/$label.log 2>&1
  local rc=$?
  echo "$label rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"forward_ms_per_batch": [0-9.]*' gpurun_out/sweep/$label.log | tr '\n' ' ')"
  return $rc
}
run graph_s1 FCE_STREAMS=1 &&
run graph_s2 FCE_STREAMS=2 &&
run graph_s4 FCE_STREAMS=4 &&
run graph_s8 FCE_STREAMS=8
