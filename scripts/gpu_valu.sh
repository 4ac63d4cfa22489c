#!/bin/bash
# Issue-side counters per kernel of the n32 forward (one rocprofv3 --pmc pass over scripts/pmc_kernel.py):
# how busy the VALU, LDS and memory instruction streams keep the waves, next to their wave cycles.
# usage: gpu_valu.sh TAG "COUNTERS"   -> gpurun_out/TAG/valu_by_kernel.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-valu}
CNT=${2:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"}
mkdir -p gpurun_out/$TAG
timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d gpurun_out/$TAG/valu -o run -- \
  python scripts/pmc_kernel.py > gpurun_out/$TAG/valu.log 2>&1
rc=$?; echo "valu pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
python scripts/pmc_by_kernel.py gpurun_out/$TAG/valu > gpurun_out/$TAG/valu_by_kernel.txt
rc=$?
NL=$(grep -o "launches per forward [0-9]*" gpurun_out/$TAG/valu.log | grep -o "[0-9]*$")
[ $rc -eq 0 ] && python scripts/pmc_last_forward.py gpurun_out/$TAG/valu $NL > gpurun_out/$TAG/valu_last_forward.txt
rc=$?; rm -rf gpurun_out/$TAG/valu; exit $rc
