#!/bin/bash
# HBM traffic and MFMA work per kernel: three separate rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE
# cannot share a pass on gfx950; the MFMA counters get their own), kernel trace only, short bench run.
# usage: gpu_pmc.sh TAG [bench args...]   -> gpurun_out/pmc/TAG_summary.json (scripts/pmc_summary.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
TAG=${1:-r02}
shift
pass() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc/${TAG}_$name -o run -- \
    python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --predict-steps 0 --dist-config-steps 0 --profile-passes 1 --no-nms \
    --profile-json gpurun_out/pmc/${TAG}_profile_$name.json $BARGS > gpurun_out/pmc/${TAG}_$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; return $rc
}
BARGS="$*"
pass FETCH FETCH_SIZE && pass WRITE WRITE_SIZE && pass MFMA SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
python scripts/pmc_summary.py gpurun_out/pmc/${TAG}_FETCH gpurun_out/pmc/${TAG}_WRITE gpurun_out/pmc/${TAG}_profile_FETCH.json gpurun_out/pmc/${TAG}_MFMA > gpurun_out/pmc/${TAG}_summary.json
rc=$?; python -c "import json;d=json.load(open('gpurun_out/pmc/${TAG}_summary.json'))['families'];print({k:(round(v['hbm_over_alg'],2),v.get('mfma_frac')) for k,v in d.items()})"
# the raw per-dispatch CSVs of a large model exceed what gpurun copies back: keep the summary only
rm -rf gpurun_out/pmc/${TAG}_FETCH gpurun_out/pmc/${TAG}_WRITE gpurun_out/pmc/${TAG}_MFMA
exit $rc
