"""Every pw2 instantiation (csrc/pw2.hip) standalone through the C-ABI against the two fce_conv2d calls, on a small map
with a partial last tile, one configuration per child process (a fault stops the run at that configuration); with
--time, the n32 shapes timed fused against the two convs.

    python scripts/pw2_probe.py [--time]
"""
import ctypes as C
import os
import subprocess
import sys
from pathlib import Path

CFGS = [(128, 128, 64, 64, "pre"), (64, 64, 192, 128, "post"), (256, 256, 128, 128, "pre"), (64, 256, 128, 128, "pre"),
        (128, 128, 384, 256, "post"), (256, 256, 128, 256, "pre"), (128, 128, 128, 256, "same"),
        (256, 128, 256, 256, "post")]


def one(i, timed):
    import torch

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import fce_pkg

    fce_pkg.load()
    from fce_yolo_amd import _native as N
    from fce_yolo_amd import modules as M

    cin1, cout1, cin2, cout2, mode = CFGS[i]
    dev = torch.device("cuda:0")
    n, H, W = (32, 20, 20) if timed else (3, 10, 10)
    g = torch.Generator().manual_seed(5)
    packed, bs, descs = [], [], []
    for cin, cout in ((cin1, cout1), (cin2, cout2)):
        d = N.ConvDesc(cin, cout, 1, 1, 1, N.ACT_SILU, 0, N.EPI_STORE, None, 0, 0)
        packed.append(M.pack_conv(d, torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5, dev))
        bs.append((torch.randn(cout, generator=g) * 0.1).to(dev))
        descs.append(d)
    x = torch.randn(n, H, W, cin1, generator=g).half().to(dev)
    if mode == "pre":
        width, hoff, x2off = cout1, 0, cout1 - cin2
    elif mode == "post":
        width, x2off = cin2, 0
        hoff = cin2 - cout1
    else:
        width, hoff, x2off = cout1, 0, 0
    base = torch.randn(n, H, W, width, generator=g).half().to(dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    T = lambda t, c, off: N.Tensor(t.data_ptr(), N.F16, N.NHWC, n, c, H, W, t.shape[-1], off)  # noqa: E731
    xt = T(x, cin1, 0)

    def run(fused, buf, y):
        ht, x2, yt = T(buf, cout1, hoff), T(buf, cin2, x2off), T(y, cout2, 0)
        if fused:
            d = N.Pw2Desc()
            d.cin1, d.cout1, d.cin2, d.cout2 = cin1, cout1, cin2, cout2
            for j in range(2):
                d.act[j], d.w[j], d.b[j] = N.ACT_SILU, packed[j].data_ptr(), bs[j].data_ptr()
            N.call("fce_pw2", C.byref(d), C.byref(xt), None, C.byref(ht), 1, C.byref(x2), None, C.byref(yt), None, 0, s)
        else:
            N.call("fce_conv2d", C.byref(descs[0]), C.byref(xt), packed[0].data_ptr(), bs[0].data_ptr(), None,
                   C.byref(ht), s)
            N.call("fce_conv2d", C.byref(descs[1]), C.byref(x2), packed[1].data_ptr(), bs[1].data_ptr(), None,
                   C.byref(yt), s)

    bf, bu = base.clone(), base.clone()
    yf = torch.zeros(n, H, W, cout2, dtype=torch.float16, device=dev)
    yu = torch.zeros_like(yf)
    run(True, bf, yf)
    run(False, bu, yu)
    torch.cuda.synchronize()
    dy = (yf.float() - yu.float()).abs().max().item()
    dh = (bf.float() - bu.float()).abs().max().item()
    line = f"{CFGS[i]}: equal y {torch.equal(yf, yu)} (max diff {dy:.3g}), equal h {torch.equal(bf, bu)} ({dh:.3g})"
    if timed:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        res = []
        for fused in (True, False):
            best = 1e9
            for _ in range(3):
                e0.record()
                for _ in range(20):
                    run(fused, bf, yf)
                e1.record()
                e1.synchronize()
                best = min(best, e0.elapsed_time(e1) / 20 * 1e3)
            res.append(best)
        line += f"; bs32 20^2: fused {res[0]:.1f} us, two convs (default variants) {res[1]:.1f} us"
    print(line, flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        one(int(sys.argv[2]), len(sys.argv) > 3)
        sys.exit(0)
    timed = "--time" in sys.argv
    for i in range(len(CFGS)):
        r = subprocess.run([sys.executable, __file__, "--child", str(i)] + (["t"] if timed else []), timeout=120)
        if r.returncode != 0:
            print(f"config {CFGS[i]}: exit {r.returncode}; stopping", flush=True)
            sys.exit(r.returncode)
