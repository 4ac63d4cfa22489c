#!/bin/bash
# r02b: full GPU suite + bench + 2-rank gloo rehearsal of the sharded bench + MFMA counter names.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --predict-steps 0 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"forward_ms_per_batch": [0-9.]*' gpurun_out/bench.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
FCE_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --cpu-seconds 0 --predict-steps 0 --profile-passes 1 > gpurun_out/bench_gloo2.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; tail -3 gpurun_out/bench_gloo2.log | cut -c1-400
timeout -k 10 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1; grep -i "mfma\|GRBM_GUI_ACTIVE\|SQ_BUSY_CYCLES" gpurun_out/rocprof_counters.txt | head -20
exit 0
