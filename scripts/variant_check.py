"""Every kernel variant of every conv op of a planned model, checked bitwise against the heuristic choice
in the model's own context (views, upsampling, fused epilogues, Detect tails, real batch sizes).

    python scripts/variant_check.py [--model yolo11n-fce.yaml] [--batch 1] [--imgsz 640]
"""
import argparse
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
os.environ["FCE_AUTOTUNE"] = "0"
import fce_pkg  # noqa: E402

fce_pkg.load()
import cases  # noqa: E402
from fce_yolo_amd.engine import Engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="yolo11n-fce.yaml")
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--imgsz", type=int, default=640)
a = ap.parse_args()
dev = torch.device("cuda:0")
model = cases.seeded_model(a.model, 0).to(dev)
x = torch.rand(a.batch, 3, a.imgsz, a.imgsz, generator=torch.Generator().manual_seed(7)).half().to(dev)
eng = Engine(model, a.batch, a.imgsz, dev)
base = eng(x).clone()
bad = 0
for i in range(eng.num_ops()):
    codes = eng.variants(i)
    if not codes:
        continue
    for code in codes:
        eng.set_variant(i, code)
        y = eng(x)
        if not torch.equal(y, base):
            d = (y - base).abs().max().item()
            print(f"op {i} {eng.op_info(i)[0]} variant {code:#x}: max diff {d:.3e}", flush=True)
            bad += 1
    eng.set_variant(i, -1)
print(f"{a.model} b{a.batch} {a.imgsz}: {bad} mismatching (op, variant) pairs")
sys.exit(1 if bad else 0)
