"""Phase timing of the device NMS on the bench workload (FCE_NMS_STOP=k ends the kernel after phase k: 1 candidates,
2 the sorted-prefix select + 2048-slot sort, 10 the full 8192-slot sort instead, 5 the greedy without its window
tests, 3 everything with the full sort, 12 fixed frontier steps, 0 the shipped kernel)."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402

fce_pkg.load()
from fce_yolo_amd.engine import NMS, Engine  # noqa: E402
from fce_yolo_amd.parser import DetectionModel  # noqa: E402
from fce_yolo_amd.weights import seeded_state_dict  # noqa: E402

dev = torch.device("cuda:0")
model = DetectionModel("yolo11n-fce.yaml")
model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in model.state_dict().items()], 0))
model.eval().to(dev)
B = int(os.environ.get("B", 32))
x = torch.rand(B, 3, 640, 640, generator=torch.Generator().manual_seed(1000)).half().to(dev)
eng = Engine(model, B, 640, dev)
pred = eng(x).clone()
nms = NMS(B, eng.anchors, eng.nc, dev)
ncand = (pred[:, 4:].amax(1) > 0.25).sum(1)
print("candidates per image: min", int(ncand.min()), "max", int(ncand.max()), "of", eng.anchors, flush=True)
bsc, bcl = pred[:, 4:].max(1)
for b in range(2):  # best-class spread of the candidates (how many kept boxes a candidate could share a class with)
    h = torch.bincount(bcl[b][bsc[b] > 0.25], minlength=eng.nc).sort(descending=True).values
    print(f"image {b}: classes used {int((h > 0).sum())}, largest class shares {(h[:4].float() / h.sum()).tolist()}")
for stop in ("1", "2", "10", "5", "3", "12", "0"):
    os.environ["FCE_NMS_STOP"] = stop
    for _ in range(3):
        nms(pred)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        nms(pred)
    e1.record()
    torch.cuda.synchronize()
    print(f"stop={stop}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per call", flush=True)
print("kept", nms.counts.tolist()[:8])
# the shipped call: best-class keys from the Detect cls epilogue (score bits << 32 | ~class), no arg-max pass
os.environ["FCE_NMS_STOP"] = "0"
best = (((bsc.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF) << 32) | (0xFFFFFFFF - bcl)).contiguous()
for _ in range(3):
    nms(pred, best)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    nms(pred, best)
e1.record()
torch.cuda.synchronize()
print(f"with epilogue keys (the bench path): {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per call", flush=True)
os.environ["FCE_NMS_STOP"] = "9"
nms(pred)
torch.cuda.synchronize()
t = nms.dets[:4, :2, :].reshape(4, 12)[:, :8].cpu().tolist()
print("segment clocks [select, colmask, resolve, window, tiles, extensions, ext-tests, tail] (s_memtime):")
for r in t:
    print("  ", [int(v) for v in r])
# greedy depth: sorted rank (score desc, anchor asc) of the last kept candidate per image
os.environ["FCE_NMS_STOP"] = "0"
nms(pred)
torch.cuda.synchronize()
sc, cl = pred[:, 4:].max(1)
depth = []
for b in range(min(B, 8)):
    s = sc[b].double().cpu()
    cand = torch.nonzero(s > 0.25).flatten()
    order = sorted(cand.tolist(), key=lambda a: (-float(s[a]), a))
    rank = {a: i for i, a in enumerate(order)}
    k = nms.keep[b, : int(nms.counts[b])].cpu().tolist()
    same = sum(1 for i in range(len(order) - 1) if float(s[order[i]]) == float(s[order[i + 1]]))
    depth.append((max(rank[a] for a in k) + 1 if k else 0, len(order), same))
print("greedy depth (last kept rank + 1, candidates, equal-score neighbours):", depth)
