#!/bin/bash
# per-kernel breakdown of BiCoordCrossAtt at the l32 / m16 L5 shapes (kernel trace + stats)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ct
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ct/p -o run -- python scripts/coord_bench.py 100 > gpurun_out/ct/log.txt 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/ct/log.txt | tail -4
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/ct/p/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:90]:90s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us  total {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
exit $rc
