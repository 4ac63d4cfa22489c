cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -q -k "sppf or op_parity" --timeout 120 --timeout-method thread > gpurun_out/pt_c.log 2>&1; tail -1 gpurun_out/pt_c.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --profile-json gpurun_out/profile.json > gpurun_out/bench.log 2>&1; echo bench rc=$?; grep -o '"value": [0-9.]*\|"forward_ms_per_batch": [0-9.]*\|"maxpool_chain": {[^}]*}' gpurun_out/bench.log
