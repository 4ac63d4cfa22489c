"""Per-kernel averages of a rocprofv3 --pmc counter CSV (run_counter_collection.csv): python scripts/pmc_kernels.py CSV"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"].split("(")[0][:70]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, v in agg.items():
    n = max(cnt[(k, c)] for c in v)
    print(k, f"({n} dispatches)")
    for c, x in sorted(v.items()):
        print(f"    {c:28s} {x / n:14.0f}")
    if v.get("SQ_LDS_IDX_ACTIVE"):
        print(f"    LDS conflict / active      {v['SQ_LDS_BANK_CONFLICT'] / v['SQ_LDS_IDX_ACTIVE']:.3f}")
