set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06i
for th in std alt std alt; do FCE_BNECK_TH=$th timeout -k 10 120 python -u scripts/bneck_probe.py >> gpurun_out/r06i/probe.txt 2>&1 || exit $?; done
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "bneck" --timeout 120 --timeout-method thread > gpurun_out/r06i/pytest.log 2>&1; echo pytest rc=$? $(tail -1 gpurun_out/r06i/pytest.log)
