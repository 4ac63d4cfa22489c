"""Fused Bottleneck chain (csrc/bneck.hip) in isolation on the n32 shapes: fce_bneck_fused time per call (events, best
of 3 windows of 20 calls) for each instantiated chain, and (FCE_BNECK_DIAG=1) block 0's per-stage clocks.

    python scripts/bneck_probe.py [batch]
"""
import ctypes as C
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402

fce_pkg.load()
from fce_yolo_amd import _native as N  # noqa: E402
from fce_yolo_amd import modules as M  # noqa: E402

dev = torch.device("cuda:0")
batch = int(sys.argv[1]) if len(sys.argv) > 1 else 32
cfgs = [("n L7 C3k pair", 32, 32, 2, 40), ("n L10/L24 C3k pair", 64, 64, 2, 20), ("n L15/L21 Bottleneck", 64, 32, 1, 40)]
s = torch.cuda.current_stream(dev).cuda_stream
for name, c, cm, nb, hw in cfgs:
    g = torch.Generator().manual_seed(1)
    d = N.BneckDesc()
    d.c, d.c_mid, d.n, d.shortcut = c, cm, nb, 1
    keep = []
    for j, (ci, co) in enumerate([(c, cm), (cm, c)] * nb):
        cd = N.ConvDesc(ci, co, 3, 1, 1, N.ACT_SILU, 0, N.EPI_STORE, None, 0, 0)
        w = M.pack_conv(cd, torch.randn(co, ci, 3, 3, generator=g) * (1.0 / (ci * 9) ** 0.5), dev)
        b = (torch.randn(co, generator=g) * 0.1).to(dev)
        keep += [w, b]
        d.w[j], d.b[j] = w.data_ptr(), b.data_ptr()
    x = torch.randn(batch, hw, hw, c, generator=g).half().to(dev)
    y = torch.empty_like(x)
    xt = N.Tensor(x.data_ptr(), N.F16, N.NHWC, batch, c, hw, hw, c, 0)
    yt = N.Tensor(y.data_ptr(), N.F16, N.NHWC, batch, c, hw, hw, c, 0)
    call = lambda: N.call("fce_bneck_fused", C.byref(d), C.byref(xt), C.byref(yt), s)  # noqa: E731
    for _ in range(3):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(20):
            call()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / 20 * 1e3)
    gf = 2.0 * batch * hw * hw * nb * 18 * c * cm / 1e9
    print(f"{name} <{c},{cm},{nb}> {hw}^2 bs{batch}: {best:.1f} us  ({gf / best * 1e3:.0f} TF/s)  env "
          f"{ {k: v for k, v in os.environ.items() if k.startswith('FCE_BNECK')} }", flush=True)
    if os.environ.get("FCE_BNECK_DIAG") == "1":
        call()
        torch.cuda.synchronize()
