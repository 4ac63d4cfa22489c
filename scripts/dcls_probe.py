"""Fused Detect cls branch vs its five ops on a planned model: per level, the fused op's time (every tile the
instantiation has) against the autotuned five ops it replaces, and the plan-time timings of both forms.

    python scripts/dcls_probe.py [--model yolo11n-fce.yaml] [--batch 32] [--imgsz 640] [--passes 5]
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
ap.add_argument("--tiles", default="8,16,4/8,8,4 8,8,4/8,8,8 8,16,8/8,8,4",
                help="space-separated FCE_DCLS_TILE_64/FCE_DCLS_TILE_128 pairs")
a = ap.parse_args()
dev = torch.device("cuda:0")
model = DetectionModel(a.model)
model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in model.state_dict().items()], 0))
model.eval().to(dev)
x = torch.rand(a.batch, 3, a.imgsz, a.imgsz, generator=torch.Generator().manual_seed(3)).half().to(dev)


def prof(eng):
    tot = None
    for _ in range(a.passes):
        p = eng.profile(x)
        tot = p if tot is None else [(*q[:3], q[3] + r[3]) for q, r in zip(tot, p)]
    return [(q[0], q[1], q[2], q[3] / a.passes * 1e3) for q in tot]


os.environ["FCE_FUSE_DCLS"] = "0"
eu = Engine(model, a.batch, a.imgsz, dev)
yu = eu(x).clone()
pu = prof(eu)
cls_runs = []  # (first op, five times) of every cls branch: dwconv, 1x1, dwconv, 1x1, detect_cls
for i in range(len(pu) - 4):
    if pu[i][0] == "dwconv3x3" and pu[i + 4][0] == "conv1x1_detect_cls":
        cls_runs.append((i, [q[3] for q in pu[i:i + 5]]))
for i, t in cls_runs:
    print(f"five ops {i}-{i + 4}: {sum(t):7.1f} us ({', '.join(f'{v:.1f}' for v in t)})")
os.environ["FCE_FUSE_DCLS"] = "1"
for t64, t128 in (t.split("/") for t in a.tiles.split()):
    os.environ["FCE_DCLS_TILE_64"], os.environ["FCE_DCLS_TILE_128"] = t64, t128
    ef = Engine(model, a.batch, a.imgsz, dev)
    yf = ef(x).clone()
    pf = prof(ef)
    torch.cuda.synchronize()
    fused = [(q[1], q[3]) for q in pf if q[0] == "detect_cls_fused" and q[3] > 0]
    print(f"tiles {t64} / {t128}: bitwise {torch.equal(yu, yf)}  fused ops "
          + "  ".join(f"{mb / 1e6:.1f} MB {us:.1f} us ({mb / us / 1e6:.2f} TB/s)" for mb, us in fused)
          + f"  forward {sum(q[3] for q in pf):.1f} us (unfused {sum(q[3] for q in pu):.1f})", flush=True)
for k in ("FCE_FUSE_DCLS", "FCE_DCLS_TILE_64", "FCE_DCLS_TILE_128"):
    os.environ.pop(k)
ea = Engine(model, a.batch, a.imgsz, dev)
k = 0
op, code, ms = C.c_int(), C.c_int(), C.c_float()
times = {}
while N.lib().fce_net_tune_record(ea.be.net, k, C.byref(op), C.byref(code), C.byref(ms)):
    if code.value & 0xFF0 == 0xF00:
        times.setdefault(op.value, {})[code.value & 1] = ms.value * 1e3
    k += 1
for i in range(ea.num_ops()):
    if ea.op_info(i)[0] == "detect_cls_fused":
        t = times.get(i, {})
        print(f"auto op {i}: {'fused' if ea.alt_form(i) else 'five ops'} (plan timing: five ops "
              f"{t.get(0, float('nan')):.1f} us, fused {t.get(1, float('nan')):.1f} us)")
