#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC counters in this pass), then the
# per-family summary of the timed region (scripts/trace_summary.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-8}  # the bench default (4 lanes) asks for 8; set before rocprofv3 starts the program
TAG=${1:-r01}
shift
STEPS=20
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$TAG -o run -- \
  python bench.py --steps $STEPS --warmup 5 --cpu-seconds 0 --dist-config-steps 0 "$@" > gpurun_out/prof/${TAG}_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof/${TAG}_bench.log
[ $rc -eq 0 ] || exit $rc
python scripts/trace_summary.py gpurun_out/prof/$TAG $STEPS gpurun_out/prof/${TAG}_bench.log > gpurun_out/prof/${TAG}_trace_summary.json
rc=$?; python -c "import json;d=json.load(open('gpurun_out/prof/${TAG}_trace_summary.json'));print(d.get('agreement'), d['timed_region']['span_ms_per_pass'])"
exit $rc
