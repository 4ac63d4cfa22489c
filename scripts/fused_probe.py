"""Fused C3k2 vs its four convs on a planned model: bitwise check of the whole forward, per-op times of
the fused ops against the autotuned convs they replace, and the forward's summed kernel time.

    python scripts/fused_probe.py [--model yolo11n-fce.yaml] [--batch 32] [--imgsz 640] [--passes 5]

FCE_FUSE_C3K2 / FCE_C3K2_TILE select what the 'fused' engine uses (default: every qualifying block).
"""
import argparse
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402

fce_pkg.load()
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


def prof(eng):
    tot = None
    for _ in range(a.passes):
        p = eng.profile(x, launches=True)
        tot = p if tot is None else [(*q[:3], q[3] + r[3], q[4]) for q, r in zip(tot, p)]
    return [(q[0], q[1], q[2], q[3] / a.passes, q[4]) for q in tot]


fuse = os.environ.get("FCE_FUSE_C3K2", "1")
os.environ["FCE_FUSE_C3K2"] = "0"
eu = Engine(model, a.batch, a.imgsz, dev)
yu = eu(x).clone()
pu = prof(eu)
os.environ["FCE_FUSE_C3K2"] = fuse
ef = Engine(model, a.batch, a.imgsz, dev)
yf = ef(x).clone()
pf = prof(ef)
torch.cuda.synchronize()
print(f"bitwise equal: {torch.equal(yu, yf)}  max|d| {(yu - yf).abs().max().item():.3e}")
print(f"ops: unfused {len(pu)}  fused {len(pf)}")
print(f"forward kernel time: unfused {sum(p[3] for p in pu) * 1e3:.1f} us  fused {sum(p[3] for p in pf) * 1e3:.1f} us")
# walk both op lists: every fused op replaces 4 consecutive convs (cv1, m.cv1, m.cv2, cv2)
i = j = 0
while i < len(pu) and j < len(pf):
    if pf[j][0] == "c3k2_fused":
        u = pu[i:i + 4]
        tu = sum(q[3] for q in u) * 1e3
        print(f"op {j:3d} c3k2_fused {pf[j][1] / 1e6:8.1f} MB {pf[j][3] * 1e3:8.1f} us  <- unfused ops {i}-{i + 3}: "
              f"{sum(q[1] for q in u) / 1e6:8.1f} MB {tu:8.1f} us ({', '.join(f'{q[3] * 1e3:.1f}' for q in u)})")
        i += 4
        j += 1
    else:
        i += 1
        j += 1

# the default (auto): both forms recorded, the plan-time autotune's pick per block (tune-log codes 0xF00 / 0xF01)
import ctypes as C  # noqa: E402

from fce_yolo_amd import _native as N  # noqa: E402

os.environ.pop("FCE_FUSE_C3K2", None)
ea = Engine(model, a.batch, a.imgsz, dev)
ya = ea(x).clone()
torch.cuda.synchronize()
print(f"auto: bitwise equal to unfused {torch.equal(ya, yu)}")
k = 0
op, code, ms = C.c_int(), C.c_int(), C.c_float()
times = {}
while N.lib().fce_net_tune_record(ea.be.net, k, C.byref(op), C.byref(code), C.byref(ms)):
    if code.value & 0xFF0 == 0xF00:
        times.setdefault(op.value, {})[code.value & 1] = ms.value * 1e3
    k += 1
for i in range(ea.num_ops()):
    f = ea.c3k2_form(i)
    if f >= 0:
        t = times.get(i, {})
        print(f"  op {i}: {'fused' if f else 'convs'} (plan timing: convs {t.get(0, float('nan')):.1f} us, "
              f"fused {t.get(1, float('nan')):.1f} us)")
pa = prof(ea)
print(f"auto forward kernel time {sum(p[3] for p in pa) * 1e3:.1f} us")
