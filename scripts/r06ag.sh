set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06ag
timeout -k 10 300 python -u -m pytest tests -v -m gpu -k "channel_slice_views" --timeout 120 --timeout-method thread > gpurun_out/r06ag/pytest.log 2>&1; rc=$?; echo pytest rc=$rc $(tail -1 gpurun_out/r06ag/pytest.log)
