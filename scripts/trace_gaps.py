"""Gaps between consecutive kernels of one rocprofv3 kernel trace (csv), inside bench's timed region:
how much of a forward is launch / dependency overhead rather than kernel time.

    python scripts/trace_gaps.py gpurun_out/prof/TAG
"""
import csv
import glob
import statistics
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
# the last 40 % of the trace is inside the timed steps of a short bench run (warm-up and plan excluded)
rows = [r for r in rows if "fce" in r[2]]
tail = rows[int(len(rows) * 0.6):]
gaps = [b[0] - a[1] for a, b in zip(tail, tail[1:])]
busy = sum(e - s for s, e, _ in tail)
span = tail[-1][1] - tail[0][0]
pos = [g for g in gaps if g > 0]
print(f"kernels {len(tail)}  span {span / 1e3:.1f} us  busy {busy / 1e3:.1f} us  idle {100 * (span - busy) / span:.1f} %")
print(f"gap median {statistics.median(gaps) / 1e3:.2f} us  mean {statistics.mean(gaps) / 1e3:.2f} us  "
      f"p90 {sorted(gaps)[int(0.9 * len(gaps))] / 1e3:.2f} us  overlapping pairs {sum(1 for g in gaps if g < 0)}")
