"""Average duration per kernel name in consecutive phases of a rocprofv3 kernel trace, where a phase is a
run of `per_phase` calls of the phase's first (anchor) kernel.  For standalone scripts that time several
shapes one after another (scripts/coord_bench.py): python scripts/trace_by_phase.py <trace.csv> <anchor> <calls>"""
import csv
import sys
from collections import defaultdict

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1])))
anchor, per = sys.argv[2], int(sys.argv[3])
phase, seen, acc = 0, 0, defaultdict(lambda: defaultdict(list))
for st, en, name in rows:
    if anchor in name:
        seen += 1
        phase = (seen - 1) // per
    acc[phase][name[:60]].append((en - st) / 1e3)
for ph in sorted(acc):
    tot = 0.0
    for name, v in acc[ph].items():
        if name.startswith("void at::") or "rocclr" in name:
            continue
        tot += sum(v) / per
        print(f"phase {ph} {name:60s} n={len(v):3d} avg {sum(v)/len(v):7.2f} us")
    print(f"phase {ph} total per call {tot:.1f} us")
