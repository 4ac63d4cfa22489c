"""Find the op whose kernel choice breaks batch invariance: plan a bs-B and a bs-1 engine of one model, then
pin the bs-1 engine's ops one at a time to the variant the bs-B plan chose and report every op whose pin
changes the bs-1 output (and every op whose bs-1 candidates disagree among themselves).

    python scripts/variant_diff.py [--model yolo11m-fce.yaml] [--heads8] [--batch 16] [--imgsz 1280]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
import fce_pkg  # noqa: E402

fce_pkg.load()
import cases  # noqa: E402
from fce_yolo_amd.engine import Engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="yolo11m-fce.yaml")
ap.add_argument("--heads8", action="store_true")
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--imgsz", type=int, default=1280)
ap.add_argument("--all", action="store_true", help="also try every bs-1 candidate of every op")
a = ap.parse_args()
dev = torch.device("cuda:0")
model = cases.seeded_model(a.model, 0, cases.heads8 if a.heads8 else None).to(dev)
xb = torch.rand(a.batch, 3, a.imgsz, a.imgsz, generator=torch.Generator().manual_seed(7)).half().to(dev)
eb = Engine(model, a.batch, a.imgsz, dev)
yb = eb(xb).clone()
picks = [eb.variant(i) for i in range(eb.num_ops())]
names = [eb.op_info(i)[0] for i in range(eb.num_ops())]
eb.close()
e1 = Engine(model, 1, a.imgsz, dev)
x1 = xb[:1].contiguous()
y1 = e1(x1).clone()
print(f"bs1 == bs{a.batch} row 0: {torch.equal(y1[0], yb[0])}  max|d| {(y1[0] - yb[0]).abs().max().item():.3e}")
for i, code in enumerate(picks):
    mine = e1.variant(i)
    if code == mine or code not in e1.variants(i):
        if code != mine:
            print(f"op {i:3d} {names[i]:20s} bs{a.batch} pick {code:#x} is not a bs-1 candidate (bs-1 {mine:#x})")
        continue
    e1.set_variant(i, code)
    y = e1(x1)
    if not torch.equal(y, y1):
        print(f"op {i:3d} {names[i]:20s} bs{a.batch} pick {code:#x} vs bs-1 {mine:#x}: output differs "
              f"max|d| {(y - y1).abs().max().item():.3e}")
    e1.set_variant(i, mine)
    if a.all:
        for c in e1.variants(i):
            e1.set_variant(i, c)
            if not torch.equal(e1(x1), y1):
                print(f"op {i:3d} {names[i]:20s} bs-1 candidate {c:#x} differs from {mine:#x}")
        e1.set_variant(i, mine)
print("done")
