set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06am
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -v -m gpu -k "every_variant or channel_slice_views" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc $(tail -1 $O/pytest.log); [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/tune_report.py > $O/tune_n32.txt 2>&1; echo tune rc=$?
