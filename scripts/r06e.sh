set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06e
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "bneck" --timeout 120 --timeout-method thread > gpurun_out/r06e/pytest.log 2>&1; echo pytest rc=$? $(tail -1 gpurun_out/r06e/pytest.log)
for fo in 0 1 0 1; do FCE_BNECK_FO=$fo timeout -k 10 120 python -u scripts/bneck_probe.py >> gpurun_out/r06e/probe.txt 2>&1 || exit $?; done
FCE_BNECK_FO=1 FCE_BNECK_DIAG=1 timeout -k 10 120 python -u scripts/bneck_probe.py 1 > gpurun_out/r06e/diag.txt 2>&1
