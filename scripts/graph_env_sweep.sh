#!/bin/bash
# Forward time: captured linear hipGraph vs direct launches on 1 / 2 / 4 streams (op DAG).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
run() {  # label, graph, env...
  local label=$1 g=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --steps 30 --warmup 5 --cpu-seconds 0 --graph $g > gpurun_out/sweep/$label.log 2>&1
  local rc=$?
  echo "$label rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"forward_ms_per_batch": [0-9.]*' gpurun_out/sweep/$label.log | tr '\n' ' ')"
  return $rc
}
run graph 1 &&
run direct_s1 0 FCE_STREAMS=1 &&
run direct_s2 0 FCE_STREAMS=2 &&
run direct_s4 0 FCE_STREAMS=4
