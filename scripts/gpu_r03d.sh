#!/bin/bash
# per-kernel times of the two NMS paths (rocprofv3 kernel trace of scripts/nms_bench.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_nms
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_nms -o run -- python scripts/nms_bench.py --iters 20 > gpurun_out/nms_prof.log 2>&1
rc=$?; echo "rc=$rc"
f=$(find gpurun_out/prof_nms -name "*kernel_stats.csv" | head -1); echo "$f"; grep -i "nms" "$f" | cut -d, -f1-7
exit $rc
