set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06n
timeout -k 10 300 python -u scripts/pw2_probe.py --time > gpurun_out/r06n/probe.txt 2>&1; rc=$?; echo probe rc=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -v -m gpu -k "pw2 or bneck" --timeout 120 --timeout-method thread > gpurun_out/r06n/pytest.log 2>&1; rc=$?; echo pytest rc=$rc $(tail -1 gpurun_out/r06n/pytest.log); [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in 0 auto; do echo -n "FCE_FUSE_PW2=$v "; FCE_FUSE_PW2=$v timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 --predict-steps 0 --dist-config-steps 0 --profile-passes 3 > gpurun_out/r06n/b_${v}_$rep.log 2>&1 || exit $?; grep -o '"value": [0-9.]*\|"forward_ms_per_batch": [0-9.]*' gpurun_out/r06n/b_${v}_$rep.log | tr '\n' ' '; echo; done; done
