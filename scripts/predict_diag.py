"""Host-image predict path diagnostics: pinned H2D bandwidth (one / three streams), host packing rate per worker
count, and Predictor.stream throughput over lanes x workers (n-fce 640, 32 x 480x640 BGR images per batch).

    python scripts/predict_diag.py
"""

import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402

fce_pkg.load()
from fce_yolo_amd.parser import DetectionModel  # noqa: E402
from fce_yolo_amd.predict import Predictor  # noqa: E402
from fce_yolo_amd.weights import seeded_state_dict  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B = 32
    rng = np.random.default_rng(0)
    imgs = [rng.integers(0, 256, (480, 640, 3), dtype=np.uint8) for _ in range(B)]
    nbytes = sum(im.nbytes for im in imgs)
    host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    devb = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(3)]
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    for ns in (1, 3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for it in range(10):
            for k in range(ns):
                with torch.cuda.stream(streams[k]):
                    devb[k].copy_(host, non_blocking=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f"pinned H2D {nbytes / 1e6:.1f} MB x {10 * ns} on {ns} stream(s): {10 * ns * nbytes / el / 1e9:.1f} GB/s",
              flush=True)
    hnp = host.numpy()
    for w in (1, 4, 8, 16):
        pool = ThreadPoolExecutor(w)
        t0 = time.perf_counter()
        for _ in range(10):
            off = 0
            futs = []
            for im in imgs:
                futs.append(pool.submit(np.copyto, hnp[off:off + im.nbytes].reshape(im.shape), im))
                off += im.nbytes
            for f in futs:
                f.result()
        el = time.perf_counter() - t0
        print(f"host packing, {w} workers: {10 * nbytes / el / 1e9:.1f} GB/s ({el / 10 * 1e3:.2f} ms per batch)", flush=True)
        pool.shutdown()
    model = DetectionModel("yolo11n-fce.yaml")
    model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in model.state_dict().items()], 0))
    model.eval().to(dev)
    cfgs = [(5, 4, True, False), (6, 4, True, False), (6, 8, True, False), (7, 4, True, False), (8, 4, True, False)]
    for lanes, workers, cs, tiny in cfgs + cfgs + [(6, 4, True, True), (8, 4, True, True)]:
        p = Predictor(model, B, 640, dev, lanes=lanes, workers=workers, copy_stream=cs)
        if tiny:  # 32x32 sources: no packing / PCIe cost to speak of
            batches = [[im[:32, :32].copy() for im in imgs]] * 2
        else:
            batches = [imgs, imgs[::-1]]
        for _ in p.stream([batches[i % 2] for i in range(2 * lanes)]):
            pass
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        for d in p.stream(batches[i % 2] for i in range(30)):
            n += len(d)
        el = time.perf_counter() - t0
        # host-side share: submit() time alone
        ts = 0.0
        q = []
        for i in range(6):
            t1 = time.perf_counter()
            q.append(p.submit(batches[i % 2]))
            ts += time.perf_counter() - t1
            if len(q) == lanes:
                p.result(q.pop(0))
        for t in q:
            p.result(t)
        print(f"Predictor lanes {lanes} workers {workers} copy_stream {cs}{' 32x32 sources' if tiny else ''}: "
              f"{n / el:.0f} images/s ({el / 30 * 1e3:.2f} ms per batch; submit() {ts / 6 * 1e3:.2f} ms)", flush=True)
        p.close()


if __name__ == "__main__":
    main()
