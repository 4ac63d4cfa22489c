#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC counters in this pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$TAG -o run -- \
  python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/prof/${TAG}_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof/${TAG}_bench.log
find gpurun_out/prof/$TAG -name "*stats*" | head
exit $rc
