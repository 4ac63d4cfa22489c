"""Per-op autotune report of the bench workload: chosen kernel variant, and every candidate's time.

    python scripts/tune_report.py [--model yolo11n-fce.yaml] [--batch 32] [--imgsz 640] > report.txt
Variant codes: rc | rp << 4 (implicit GEMM), 0x100 | .. (3x3 LDS tile, cin % 32 == 0), 0x200 | ..
(3x3 LDS tile, small cin), 0x300 | .. (1x1 streaming), 0x400 | .. | log2(wp) << 12 (1x1 LDS tile), 0x500 (1x1 ring), 0x700 | log2(wp) << 12 (1x1 big tile, K-pipelined),
100 + v (depthwise variant v).
"""
import argparse
import ctypes as C
import sys
from collections import defaultdict
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
a = ap.parse_args()
dev = torch.device("cuda:0")
from bench import model_cfg  # noqa: E402  (the "-h8" BASELINE config)

model = DetectionModel(model_cfg(a.model))
model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in model.state_dict().items()], 0))
model.eval().to(dev)
eng = Engine(model, a.batch, a.imgsz, dev)
L = N.lib()
recs = defaultdict(list)
k = 0
op, code, ms = C.c_int(), C.c_int(), C.c_float()
while L.fce_net_tune_record(eng.net, k, C.byref(op), C.byref(code), C.byref(ms)):
    recs[op.value].append((code.value, ms.value * 1e3))
    k += 1
for i in range(eng.num_ops()):
    name, nbytes, flops = eng.op_info(i)
    ch = L.fce_net_op_variant(eng.net, i)
    cands = " ".join(f"{c:#x}:{t:.1f}" for c, t in sorted(recs.get(i, []), key=lambda r: r[1]))
    print(f"{i:3d} {name:20s} {nbytes / 1e6:7.2f}MB {flops / 1e9:6.2f}GF chosen {ch:#6x} | {cands}", flush=True)
