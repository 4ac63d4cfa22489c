set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06ak
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -v -m gpu -k "pw2 or c3_concatenated or end_to_end or batch_invariance" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc $(tail -1 $O/pytest.log); [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/tune_report.py > $O/tune_n32.txt 2>&1; echo tune rc=$?
