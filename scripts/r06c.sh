set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06c
timeout -k 10 120 python -u scripts/bneck_probe.py > gpurun_out/r06c/probe.txt 2>&1 || exit $?
FCE_BNECK_DIAG=1 timeout -k 10 120 python -u scripts/bneck_probe.py > gpurun_out/r06c/probe_diag.txt 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/r06c/pmc -o run -- python3 scripts/bneck_probe.py > gpurun_out/r06c/pmc.log 2>&1
echo pmc rc=$?
