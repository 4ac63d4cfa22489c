set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06d
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "bneck" --timeout 120 --timeout-method thread > gpurun_out/r06d/pytest.log 2>&1; echo pytest rc=$? $(tail -1 gpurun_out/r06d/pytest.log)
timeout -k 10 120 python -u scripts/bneck_probe.py > gpurun_out/r06d/probe.txt 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/r06d/pmc -o run -- python3 scripts/bneck_probe.py > gpurun_out/r06d/pmc.log 2>&1
echo pmc rc=$?
