"""One dense conv shape, timed per kernel variant (HIP events, back-to-back launches), for kernel work
and for rocprofv3 --pmc passes over a single kernel family.

    python scripts/conv_probe.py --cin 256 --cout 256 --k 3 --hw 80 --batch 32 --codes 0x2141,0x8122
"""
import argparse
import ctypes as C
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402

fce_pkg.load()
from fce_yolo_amd import _native as N  # noqa: E402
from fce_yolo_amd import modules as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cin", type=int, default=256)
ap.add_argument("--cout", type=int, default=256)
ap.add_argument("--k", type=int, default=3)
ap.add_argument("--stride", type=int, default=1)
ap.add_argument("--hw", type=int, default=80)
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--codes", default="", help="comma-separated variant codes (default: all candidates)")
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
k, s, H = a.k, a.stride, a.hw
w = torch.randn(a.cout, a.cin, k, k, generator=g) * (1.0 / (a.cin * k * k) ** 0.5)
b = torch.randn(a.cout, generator=g) * 0.1
desc = N.ConvDesc(a.cin, a.cout, k, s, 1, N.ACT_SILU, 0, 0, None, 0, 0)
wp = M.pack_conv(desc, w, dev)
bd = b.float().to(dev)
x = torch.randn(a.batch, H, H, a.cin, generator=g).half().to(dev)
Ho = (H + 2 * (k // 2) - k) // s + 1
y = torch.empty(a.batch, Ho, Ho, a.cout, dtype=torch.float16, device=dev)
xt = N.Tensor(x.data_ptr(), N.F16, N.NHWC, a.batch, a.cin, H, H, a.cin, 0)
yt = N.Tensor(y.data_ptr(), N.F16, N.NHWC, a.batch, a.cout, Ho, Ho, a.cout, 0)
if a.codes:
    codes = [int(c, 0) for c in a.codes.split(",")]
else:
    arr = (C.c_int * 128)()
    codes = list(arr[:N.lib().fce_conv_variants(C.byref(desc), H, arr, 128)])
flops = 2.0 * a.batch * Ho * Ho * a.cout * a.cin * k * k


def launch(code):
    N.call("fce_conv2d_variant", C.byref(desc), C.byref(xt), wp.data_ptr(), bd.data_ptr(), None, C.byref(yt), code,
           None)


ref = None
for code in codes:
    try:
        launch(code)
    except RuntimeError as e:
        print(f"{code:#7x} skipped: {e}", flush=True)
        continue
    torch.cuda.synchronize()
    if ref is None:
        ref = y.clone()
    same = torch.equal(y, ref)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        launch(code)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.reps
    print(f"{code:#7x} {us:8.1f} us {flops / us / 1e6:7.1f} TF/s {'' if same else 'MISMATCH'}", flush=True)
