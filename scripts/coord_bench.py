"""Standalone BiCoordCrossAtt timing at the bench shapes (run under rocprofv3 --kernel-trace --stats)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402

fce_pkg.load()
from fce_yolo_amd import modules as M  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = ((32, 128, 80, 80, 4, 8), (32, 128, 40, 40, 4, 8), (32, 512, 80, 80, 4, 8), (16, 512, 160, 160, 8, 8))
if len(sys.argv) > 1:  # only the shapes whose x is at least this many MB
    SHAPES = [t for t in SHAPES if t[0] * t[1] * t[2] * t[3] * 2 >= float(sys.argv[1]) * 2**20]
for (N, C, H, W, heads, red) in SHAPES:
    torch.manual_seed(0)
    m = M.BiCoordCrossAtt(C, C, red, heads).to(dev).eval()
    x = torch.randn(N, C, H, W, device=dev).half().contiguous(memory_format=torch.channels_last)
    for _ in range(3):
        y = m(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        y = m(x)
    e1.record()
    torch.cuda.synchronize()
    print(f"N{N} C{C} {H}x{W} heads{heads}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per call", flush=True)
