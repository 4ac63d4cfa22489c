"""Every plan-time alternative of a planned model (fused C3k2, fused Detect cls branch, fused stem pair): the form
the autotune kept and its timings of both forms, then the fused ops' eager per-op times against the ops they
replace (all alternatives forced fused, then all forced unfused).

    python scripts/alt_probe.py [--model yolo11n-fce.yaml] [--batch 32] [--imgsz 640] [--passes 5]
"""
import argparse
import ctypes as C
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402

fce_pkg.load()
from fce_yolo_amd import _native as N  # noqa: E402
from fce_yolo_amd.engine import Engine  # noqa: E402
from fce_yolo_amd.parser import DetectionModel  # noqa: E402
from fce_yolo_amd.weights import seeded_state_dict  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="yolo11n-fce.yaml")
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--imgsz", type=int, default=640)
ap.add_argument("--passes", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda:0")
model = DetectionModel(a.model)
model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in model.state_dict().items()], 0))
model.eval().to(dev)
x = torch.rand(a.batch, 3, a.imgsz, a.imgsz, generator=torch.Generator().manual_seed(3)).half().to(dev)

ea = Engine(model, a.batch, a.imgsz, dev)
k = 0
op, code, ms = C.c_int(), C.c_int(), C.c_float()
times = {}
while N.lib().fce_net_tune_record(ea.be.net, k, C.byref(op), C.byref(code), C.byref(ms)):
    if code.value & 0xFF0 == 0xF00:
        times.setdefault(op.value, {})[code.value & 1] = ms.value * 1e3
    k += 1
alts = [i for i in range(ea.num_ops()) if ea.alt_form(i) >= 0]
for i in alts:
    t = times.get(i, {})
    print(f"auto op {i:3d} {ea.op_info(i)[0]:18s} keeps {'fused' if ea.alt_form(i) else 'the ops'} "
          f"(plan timing: ops {t.get(0, float('nan')):6.1f} us, fused {t.get(1, float('nan')):6.1f} us)")


def prof(eng):
    tot = None
    for _ in range(a.passes):
        p = eng.profile(x)
        tot = p if tot is None else [(*q[:3], q[3] + r[3]) for q, r in zip(tot, p)]
    return [q[3] / a.passes * 1e3 for q in tot]


y0 = ea(x).clone()
res = {}
for fused in (True, False):
    for i in alts:
        ea.set_alt_form(i, fused)
    res[fused] = prof(ea)
    assert torch.equal(ea(x).clone(), y0)
print("bitwise equal in every form: True")
for i in alts:
    lo = i - {"c3k2_fused": 4, "detect_cls_fused": 5, "stem_fused": 2}[ea.op_info(i)[0]]
    ops = res[False][lo:i]
    print(f"op {i:3d} {ea.op_info(i)[0]:18s} {res[True][i]:7.1f} us  <- ops {lo}-{i - 1}: {sum(ops):7.1f} us "
          f"({', '.join(f'{v:.1f}' for v in ops)})")
print(f"forward kernel time: all fused {sum(res[True]):.1f} us, all unfused {sum(res[False]):.1f} us")
