cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -q -k "coord or bicoord or op_parity or end_to_end or 640" --timeout 120 --timeout-method thread > gpurun_out/pt_c.log 2>&1; tail -1 gpurun_out/pt_c.log; grep -E "Error|assert" gpurun_out/pt_c.log | head -3
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --profile-json gpurun_out/profile.json > gpurun_out/bench.log 2>&1; echo bench rc=$?; grep -o '"value": [0-9.]*\|"forward_ms_per_batch": [0-9.]*\|"bicoordcrossatt": {[^}]*}' gpurun_out/bench.log
