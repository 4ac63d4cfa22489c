#!/bin/bash
# rocprofv3 kernel trace of a short bench run under extra environment settings: TAG VAR=VAL ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=$1; shift
for kv in "$@"; do export "$kv"; done
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/$TAG -o run -- \
  python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/prof/${TAG}_bench.log 2>&1
rc=$?; echo "rocprof $TAG rc=$rc"; exit $rc
