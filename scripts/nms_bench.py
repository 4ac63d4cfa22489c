"""Device NMS on the bench batch (n-fce 640 bs32 predictions of the seeded model): the one-workgroup kernel
(default) against the multi-workgroup path (FCE_NMS_V2=1): bitwise-equal outputs, event-timed per call.

    python scripts/nms_bench.py [--batch 32] [--imgsz 640] [--iters 50]
"""

import argparse
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


def timed(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--imgsz", type=int, default=640)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = DetectionModel("yolo11n-fce.yaml")
    model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in model.state_dict().items()], 0))
    model.eval().to(dev)
    eng = Engine(model, a.batch, a.imgsz, dev)
    x = torch.rand(a.batch, 3, a.imgsz, a.imgsz, generator=torch.Generator().manual_seed(1000)).half().to(dev)
    pred = eng(x).clone()
    best = eng.best.clone()
    nms = NMS(a.batch, eng.anchors, eng.nc, dev)
    res = {}
    for mode in ("v2", "v1"):
        if mode == "v2":
            os.environ["FCE_NMS_V2"] = "1"
        else:
            os.environ.pop("FCE_NMS_V2", None)
        nms(pred, best)
        torch.cuda.synchronize()
        out = nms.buf.clone()
        t_keys = timed(lambda: nms(pred, best), a.iters)
        t_plain = timed(lambda: nms(pred), a.iters)
        res[mode] = out
        print(f"{mode}: nms with keys {t_keys:.1f} us, with its own arg-max {t_plain:.1f} us; kept per image "
              f"{nms.counts[:4].tolist()}", flush=True)
    print("v1 == v2 bitwise:", torch.equal(res["v1"], res["v2"]))


if __name__ == "__main__":
    main()
