"""Two forwards in flight: two Engines (own arenas) on two streams, batches alternating between them, so
the latency-bound 40^2 / 20^2 tail of one batch shares the CUs with the next batch's 320^2 / 160^2 head.
Forward-only throughput against one engine on one stream (n-fce 640 bs32)."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402

fce_pkg.load()
from fce_yolo_amd.engine import Engine  # noqa: E402
from fce_yolo_amd.parser import DetectionModel  # noqa: E402
from fce_yolo_amd.weights import seeded_state_dict  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "yolo11n-fce.yaml"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
S = int(sys.argv[3]) if len(sys.argv) > 3 else 640
dev = torch.device("cuda:0")
model = DetectionModel(cfg)
model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in model.state_dict().items()], 0))
model.eval().to(dev)
xs = [torch.rand(B, 3, S, S, generator=torch.Generator().manual_seed(i)).half().to(dev) for i in range(2)]
NL = int(sys.argv[4]) if len(sys.argv) > 4 else 2
engs = [Engine(model, B, S, dev)]
engs += [engs[0].clone() for _ in range(NL - 1)]
streams = [torch.cuda.Stream(dev) for _ in range(NL)]
ref = [engs[0](xs[i]).clone() for i in range(2)]
torch.cuda.synchronize()  # the side streams below do not order against the null stream
K = 40


def run(n_eng):
    for i in range(6):
        k = i % n_eng
        with torch.cuda.stream(streams[k]):
            engs[k](xs[i % 2])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        k = i % n_eng
        with torch.cuda.stream(streams[k]):
            engs[k](xs[i % 2])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e3


for n in list(range(1, NL + 1)) * 2:
    print(f"engines {n}: {run(n):.4f} ms per batch", flush=True)
bad = 0
for k in range(NL):
    for j in range(2):
        with torch.cuda.stream(streams[k]):
            y = engs[k](xs[j]).clone()
        torch.cuda.synchronize()
        if not torch.equal(y, ref[j]):
            bad += 1
            d = (y - ref[j]).abs()
            idx = (d > 0).nonzero()
            print(f"engine {k} input {j}: max diff {d.max().item():.3e}, {idx.shape[0]} elements differ; rows "
                  f"{sorted(set(idx[:, 1].tolist()))[:12]}, anchors {idx[:, 2].min().item()}..{idx[:, 2].max().item()}, "
                  f"images {sorted(set(idx[:, 0].tolist()))[:8]}", flush=True)
e3 = Engine(model, B, S, dev)
y3 = e3(xs[1]).clone()
torch.cuda.synchronize()
print("fresh third engine equal to engine 0:", torch.equal(y3, ref[1]), flush=True)
print("outputs bitwise equal to the single-engine forward" if not bad else f"{bad} mismatches", flush=True)
