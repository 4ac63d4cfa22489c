"""Time the stem conv on the bench input shape."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402

fce_pkg.load()
from fce_yolo_amd import modules as M  # noqa: E402

dev = torch.device("cuda:0")
conv = M.Conv(3, 16, 3, 2).to(dev).eval()
x = torch.rand(32, 3, 640, 640, device=dev).half()
with torch.no_grad():
    for _ in range(3):
        y = conv(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        y = conv(x)
    e1.record()
    torch.cuda.synchronize()
print(f"stem 3->16 s2 @ 32x640x640: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us", flush=True)
