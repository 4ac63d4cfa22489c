"""Per-dispatch issue counters of the LAST forward in a rocprofv3 --pmc pass over scripts/pmc_kernel.py (the
planned net's chosen kernels, not the autotune's candidates): VALU / LDS busy fractions of the SIMDs over each
dispatch's duration, resident waves per SIMD, and the share of the forward's time.

    python scripts/pmc_last_forward.py DIR NDISPATCH [--clock-ghz 2.1]

NDISPATCH = kernel launches per forward (the bench profile's launch count).  SQ_ACTIVE_INST_* and SQ_WAVE_CYCLES
count quad-cycles (MI355X_MICROARCH.md, constants table); 1024 SIMDs.
"""
import argparse
import csv
import glob
import re
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("n", type=int)
ap.add_argument("--clock-ghz", type=float, default=2.1)
a = ap.parse_args()

cnt = defaultdict(dict)  # dispatch id -> counter -> value
name = {}
for f in glob.glob(f"{a.dir}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d = int(r["Dispatch_Id"])
        cnt[d][r["Counter_Name"]] = cnt[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        name[d] = r["Kernel_Name"]
dur = {}
for f in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9


def short(n):
    m = re.search(r"(\w+_kernel)(<[^()]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:60]


ids = sorted(cnt)[-a.n:]
tot = sum(dur.get(d, 0.0) for d in ids)
print(f"{len(ids)} dispatches, {tot * 1e6:.1f} us")
print(f"{'#':>3} {'kernel':58s} {'us':>7} {'share':>6} {'valu':>5} {'lds':>5} {'vmem':>5} {'waves/simd':>10}")
for i, d in enumerate(ids):
    t = dur.get(d, 0.0)
    simd_cyc = max(t, 1e-9) * a.clock_ghz * 1e9 * 1024
    c = cnt[d]
    f = lambda k: 4 * c.get(k, 0.0) / simd_cyc  # noqa: E731
    print(f"{i:3d} {short(name[d])[:58]:58s} {t * 1e6:7.1f} {t / tot:6.3f} {f('SQ_ACTIVE_INST_VALU'):5.2f} "
          f"{f('SQ_ACTIVE_INST_LDS'):5.2f} {f('SQ_ACTIVE_INST_VMEM'):5.2f} {f('SQ_WAVE_CYCLES'):10.1f}")
