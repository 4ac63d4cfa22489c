"""Per-kernel-family summary of a `rocprofv3 --kernel-trace` run of bench.py, restricted to the timed
region (and, separately, to the per-op HIP-event profile pass), so its average launch durations can be
set beside the `kernels` / `roofline` numbers bench.py printed for the same command.

    python scripts/trace_summary.py <rocprof output dir> <steps> [bench.log] > summary.json

bench.py dispatches a torch spin kernel (`_trace_marker`) after warm-up, after the timed steps, and
before the profile pass: segment 1 = the K timed steps, segment 3 = the profile passes.
"""
import csv
import glob
import json
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import family  # noqa: E402


def segments(d):
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    segs, cur = [], []
    for st, en, name in rows:
        if "spin_kernel" in name:
            segs.append(cur)
            cur = []
        else:
            cur.append((st, en, name))
    segs.append(cur)
    return segs


def summarise(seg, passes):
    fam = defaultdict(lambda: [0, 0.0])
    other = defaultdict(lambda: [0, 0.0])
    for st, en, name in seg:
        f = family(name)
        tgt = fam[f] if f else other[name[:60]]
        tgt[0] += 1
        tgt[1] += (en - st) * 1e-6  # ns -> ms
    span = (seg[-1][1] - seg[0][0]) * 1e-6 if seg else 0.0
    out = {k: {"launches_per_pass": v[0] / passes, "ms_per_pass": round(v[1] / passes, 4),
               "avg_launch_us": round(v[1] / v[0] * 1e3, 3)} for k, v in sorted(fam.items(), key=lambda kv: -kv[1][1])}
    return {"passes": passes, "span_ms_per_pass": round(span / passes, 4),
            "busy_ms_per_pass": round(sum(v[1] for v in fam.values()) / passes, 4), "families": out,
            "unclassified": {k: v[0] for k, v in other.items()}}


def main():
    d, steps = sys.argv[1], int(sys.argv[2])
    bench = None
    if len(sys.argv) > 3:
        for line in open(sys.argv[3]):
            if line.startswith("{"):
                bench = json.loads(line)
    segs = segments(d)
    res = {"source": f"rocprofv3 --kernel-trace of bench.py ({d}); segments split at bench.py trace markers",
           "timed_region": summarise(segs[1], steps) if len(segs) > 1 else None}
    if len(segs) > 3 and bench:
        passes = bench.get("profile_passes", 10)
        res["profile_pass"] = summarise(segs[3], passes)
        dom = bench["roofline"]["kernel"]
        bk = bench["kernels"][dom]
        tr = res["timed_region"]["families"].get(dom, {})
        res["agreement"] = {"kernel": dom,
                            "bench_hip_event_avg_launch_us": round(bk["ms"] / bk["launches"] * 1e3, 3),
                            "rocprof_timed_region_avg_launch_us": tr.get("avg_launch_us"),
                            "rocprof_profile_pass_avg_launch_us":
                                res["profile_pass"]["families"].get(dom, {}).get("avg_launch_us")}
    json.dump(res, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
