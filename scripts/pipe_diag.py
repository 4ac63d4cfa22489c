"""Pipeline diagnostics: host enqueue time of one forward, the fork op, and where the deferred NMS starts
relative to the forward (event timestamps)."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402

fce_pkg.load()
from fce_yolo_amd import _native as N  # noqa: E402
from fce_yolo_amd.engine import Engine, Pipeline  # noqa: E402
from fce_yolo_amd.parser import DetectionModel  # noqa: E402
from fce_yolo_amd.weights import seeded_state_dict  # noqa: E402

dev = torch.device("cuda:0")
model = DetectionModel("yolo11n-fce.yaml")
model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in model.state_dict().items()], 0))
model.eval().to(dev)
x = torch.rand(32, 3, 640, 640, generator=torch.Generator().manual_seed(1000)).half().to(dev)
eng = Engine(model, 32, 640, dev)
print("fork hint op", N.lib().fce_net_fork_hint(eng.net), "of", eng.num_ops(), flush=True)
for _ in range(3):
    eng(x)
torch.cuda.synchronize()
for _ in range(3):
    t0 = time.perf_counter()
    eng(x)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e3 * (t1 - t0):.3f} ms, enqueue->done {1e3 * (t2 - t0):.3f} ms", flush=True)
pipe = Pipeline(eng, 2)
for _ in range(5):
    pipe.submit(x)
pipe.flush()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    pipe.submit(x)
t1 = time.perf_counter()
pipe.flush()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"pipeline: host {1e3 * (t1 - t0) / 20:.3f} ms/step, total {1e3 * (t2 - t0) / 20:.3f} ms/step", flush=True)
# when does a side stream waiting on the fork event get released?
side = torch.cuda.Stream(dev)
main = torch.cuda.current_stream(dev)
for trial in range(3):
    e0 = torch.cuda.Event(enable_timing=True)
    e_side = torch.cuda.Event(enable_timing=True)
    e_end = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(main)
    eng(x)
    e_end.record(main)
    N.call("fce_net_wait_fork", eng.net, side.cuda_stream)
    e_side.record(side)
    torch.cuda.synchronize()
    print(f"fork released at {e0.elapsed_time(e_side):.3f} ms of a {e0.elapsed_time(e_end):.3f} ms forward", flush=True)
# step time of each mode, interleaved repetitions (same process, same inputs)
from fce_yolo_amd.engine import NMS  # noqa: E402

nms = NMS(32, eng.anchors, eng.nc, dev)
pipes = {"defer": Pipeline(eng, 2, defer=True), "nodefer": Pipeline(eng, 2, defer=False)}


def run(mode, steps=20):
    def one():
        if mode == "fwd":
            eng(x)
        elif mode == "seq":
            nms(eng(x), eng.best)
        else:
            pipes[mode].submit(x)
    for _ in range(3):
        one()
    if mode in pipes:
        pipes[mode].flush()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    if mode in pipes:
        pipes[mode].flush()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


res = {m: [] for m in ("fwd", "seq", "defer", "nodefer")}
for rep in range(5):
    for m in res:
        res[m].append(run(m))
print({m: round(sorted(v)[len(v) // 2], 4) for m, v in res.items()}, "ms/step (median of 5)")
