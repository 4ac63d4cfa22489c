set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06j
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "pw2 or bneck or pipeline" --timeout 120 --timeout-method thread > gpurun_out/r06j/pytest.log 2>&1; rc=$?; echo pytest rc=$rc $(tail -1 gpurun_out/r06j/pytest.log); [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tune_report.py > gpurun_out/r06j/tune.txt 2>&1; echo tune rc=$?
for rep in 1 2; do for v in 0 auto; do echo -n "FCE_FUSE_PW2=$v "; FCE_FUSE_PW2=$v timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 --predict-steps 0 --dist-config-steps 0 --profile-passes 3 > gpurun_out/r06j/b_${v}_$rep.log 2>&1 || exit $?; grep -o '"value": [0-9.]*\|"forward_ms_per_batch": [0-9.]*' gpurun_out/r06j/b_${v}_$rep.log | tr '\n' ' '; echo; done; done
