"""Do HIP streams run concurrently here?  8 single-workgroup NMS launches (1 image each): serial vs
one per stream.  Concurrent streams -> the multi-stream time is ~ one launch."""
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402

fce_pkg.load()
from fce_yolo_amd.engine import NMS  # noqa: E402

dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
A = 8400
p = np.zeros((1, 84, A), np.float32)
p[0, 0] = rng.random(A) * 640
p[0, 1] = rng.random(A) * 640
p[0, 2:4] = rng.random((2, A)) * 100 + 5
p[0, 4] = 0.3 + 0.7 * rng.random(A)
pred = torch.from_numpy(p).to(dev)
nmss = [NMS(1, A, 80, dev) for _ in range(8)]
streams = [torch.cuda.Stream(dev) for _ in range(8)]
for n in nmss:
    n(pred)
torch.cuda.synchronize()


def serial():
    for n in nmss:
        n(pred)


def parallel():
    cur = torch.cuda.current_stream(dev)
    for n, s in zip(nmss, streams):
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            n(pred)
    for s in streams:
        cur.wait_stream(s)


for name, f in (("serial", serial), ("8 streams", parallel), ("serial", serial), ("8 streams", parallel)):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t) / 10 * 1e6:.1f} us per 8 launches", flush=True)
print("GPU_MAX_HW_QUEUES", os.environ.get("GPU_MAX_HW_QUEUES"))
