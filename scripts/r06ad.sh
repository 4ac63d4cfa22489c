set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06ad
timeout -k 10 400 python -u -m pytest tests -v -m gpu -k "every_variant" --timeout 120 --timeout-method thread > gpurun_out/r06ad/pytest.log 2>&1; rc=$?; echo pytest rc=$rc $(tail -1 gpurun_out/r06ad/pytest.log); [ $rc -eq 0 ] || exit $rc
bash scripts/gpu.sh configs r06ad
