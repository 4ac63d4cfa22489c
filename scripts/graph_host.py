"""Host cost of one forward submission, direct launches vs hipGraph replay (n-fce 640 bs32): the
enqueue time of one call, and 20 back-to-back calls enqueued vs completed."""
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

dev = torch.device("cuda:0")
model = DetectionModel("yolo11n-fce.yaml")
model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in model.state_dict().items()], 0))
model.eval().to(dev)
x = torch.rand(32, 3, 640, 640, generator=torch.Generator().manual_seed(1000)).half().to(dev)
eng = Engine(model, 32, 640, dev)
for graph in (False, True):
    for _ in range(3):
        eng(x, graph=graph)
    torch.cuda.synchronize()
    one = []
    for _ in range(5):
        t0 = time.perf_counter()
        eng(x, graph=graph)
        one.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        eng(x, graph=graph)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"graph={int(graph)}: one call enqueue {1e3 * min(one):.3f} ms; 20 calls: host {1e3 * (t1 - t0) / 20:.3f} ms/call,"
          f" done {1e3 * (t2 - t0) / 20:.3f} ms/call", flush=True)
