cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -k "variant" --timeout 120 --timeout-method thread > gpurun_out/pt_var.log 2>&1; rc=$?; tail -5 gpurun_out/pt_var.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tune_report.py > gpurun_out/tune_report.txt 2>&1; rc=$?; echo tune rc=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 2 --profile-json gpurun_out/profile.json > gpurun_out/bench.log 2>&1; rc=$?; echo bench rc=$rc; tail -1 gpurun_out/bench.log | cut -c1-400
