set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06l
timeout -k 10 300 python -u -m pytest tests -v -m gpu -k "pw2_c_abi" --timeout 120 --timeout-method thread > gpurun_out/r06l/pytest.log 2>&1; rc=$?; echo pytest rc=$rc $(tail -1 gpurun_out/r06l/pytest.log)
