set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06k
timeout -k 10 600 python -u -m pytest tests -v -m gpu -k "pw2 or bneck" --timeout 120 --timeout-method thread > gpurun_out/r06k/pytest.log 2>&1; rc=$?; echo pytest rc=$rc $(tail -1 gpurun_out/r06k/pytest.log)
