#!/bin/bash
# HBM traffic per kernel: two separate rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE cannot
# share a pass on gfx950), kernel trace only, short bench run.  Summary: scripts/pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
TAG=${1:-r01}
shift
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc/${TAG}_$C -o run -- \
    python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --profile-passes 1 --no-nms --profile-json gpurun_out/pmc/${TAG}_profile_$C.json "$@" > gpurun_out/pmc/${TAG}_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python scripts/pmc_summary.py gpurun_out/pmc/${TAG}_FETCH_SIZE gpurun_out/pmc/${TAG}_WRITE_SIZE gpurun_out/pmc/${TAG}_profile_FETCH_SIZE.json > gpurun_out/pmc/${TAG}_summary.json
rc=$?; tail -c 600 gpurun_out/pmc/${TAG}_summary.json
# the raw per-dispatch CSVs of a large model exceed what gpurun copies back: keep the summary only
rm -rf gpurun_out/pmc/${TAG}_FETCH_SIZE gpurun_out/pmc/${TAG}_WRITE_SIZE
exit $rc
