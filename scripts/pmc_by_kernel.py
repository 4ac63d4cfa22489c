"""Per-kernel-name averages of every PMC counter in rocprofv3 --pmc output directories (+ the average
kernel-trace duration), for conv_probe / gpu_probe.sh passes.

    python scripts/pmc_by_kernel.py DIR [DIR ...]
"""
import csv
import glob
import re
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
durs = defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))


def short(n):
    m = re.search(r"(\w+_kernel)<([^>]*)>", n)
    return f"{m.group(1)}<{m.group(2)}>" if m else n[:80]


for k in sorted(set(vals) | set(durs)):
    if "conv" not in k:
        continue
    d = durs.get(k, [])
    row = {c: sum(v) / len(v) for c, v in vals[k].items()}
    print(short(k), f"dur_us={sum(d) / max(len(d), 1) / 1e3:.1f} n={len(d)}",
          " ".join(f"{c}={v:.4g}" for c, v in sorted(row.items())))
