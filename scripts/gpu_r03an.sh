#!/bin/bash
# final check after the depthwise test: full GPU suite + smoke + the driver's plain `python bench.py`, then rocprof of the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03an; export TMPDIR=/tmp
if [ "$1" != "--bench-only" ]; then
timeout -k 10 900 python -u -m pytest tests -v -m gpu -rf --timeout 120 --timeout-method thread > gpurun_out/r03an/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r03an/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03an/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r03an/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
t0=$(date +%s.%N)
timeout -k 10 400 python bench.py > gpurun_out/r03an/bench_default_cmd.log 2>&1
rc=$?; echo "bench rc=$rc wall $(python -c "import time; print(round(time.time() - $t0, 1))") s"; tail -2 gpurun_out/r03an/bench_default_cmd.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc

