#!/bin/bash
# depthwise column runs of 8 (variant 105): every-variant bitwise test, n32 tune report, bench A/B of the default command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03am; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v -k "variant" --timeout 120 --timeout-method thread > gpurun_out/r03am/pt_var.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r03am/pt_var.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tune_report.py > gpurun_out/r03am/n32_tune.txt 2>&1
rc=$?; echo "tune rc=$rc"; grep dwconv gpurun_out/r03am/n32_tune.txt | cut -c1-160; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/r03am/bench_$i.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/r03am/bench_$i.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
