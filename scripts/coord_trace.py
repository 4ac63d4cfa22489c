"""Per-shape breakdown of scripts/coord_bench.py under rocprofv3 --kernel-trace (3 shapes x 23 calls)."""
import csv
import sys
from collections import defaultdict

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if any(k in n for k in ("pool_", "coord_", "gate_apply")):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
rows.sort()
per_call = len(rows) // 69
for shape in range(3):
    seg = rows[shape * 23 * per_call:(shape + 1) * 23 * per_call]
    d = defaultdict(float)
    for s, e, n in seg:
        key = n.split("(")[0].replace("void fce::", "").replace("fce::", "")[:40]
        d[key] += (e - s) / 1e3 / 23
    print(f"shape {shape}: total {sum(d.values()):.1f} us/call", {k: round(v, 1) for k, v in d.items()})
