"""Drop-in nn.Modules for the FCE-YOLOv11 inference path.

Each class has the reference's name, constructor signature and state_dict layout (key names,
shapes and registration order), so ``yolo11-fce.yaml`` builds through a ``parse_model`` that
resolves module names to these classes (reference ``ultralytics/nn/tasks.py:1582-1588``) and
reference checkpoints' state_dicts load unchanged.  ``forward`` runs the HIP kernels through the
C-ABI (eager drop-in mode, NCHW-logical / NHWC-physical channels_last tensors); ``emit`` lowers the
same computation onto a backend (see ``backend.py``), which is how the whole-graph executor is
built.  There is no CPU arithmetic: a non-ROCm input only propagates shapes and returns ``meta``
tensors (``ShapeBackend``), which is what the reference's CPU stride probe at model construction
needs (``tasks.py:396-411``) and fails loudly wherever values are read.

BatchNorm eps is 1e-3 (reference ``utils/torch_utils.py:470`` sets it for every model; Q4), and
BN is folded into the conv at first use exactly like ``fuse_conv_and_bn`` (torch_utils.py:237-267).
"""

from __future__ import annotations

import ctypes as C
import math

import numpy as np
import torch
import torch.nn as nn

from . import _native as N
from .backend import EagerBackend, ShapeBackend, View

BN_EPS = 1e-3

__all__ = (
    "Conv", "DWConv", "Bottleneck", "C2f", "C3", "C3k", "C3k2", "SPPF", "Attention", "PSABlock", "C2PSA",
    "Concat", "Upsample", "BiFPN_Concat", "CoordAtt", "CoordCrossAtt", "BiCoordCrossAtt", "DFL", "Detect",
)


def autopad(k, p=None, d=1):
    """conv.py:30-36."""
    if d > 1:
        k = d * (k - 1) + 1 if isinstance(k, int) else [d * (x - 1) + 1 for x in k]
    if p is None:
        p = k // 2 if isinstance(k, int) else [x // 2 for x in k]
    return p


# ============================================================================ native weight cache
def _tkey(t: torch.Tensor):
    """Identity of a weight tensor's contents: storage, version counter, dtype.  Inference tensors (e.g.
    buffers of a module moved inside ``torch.inference_mode``) have no version counter; they are keyed by
    storage and dtype only."""
    try:
        return t.data_ptr(), t._version, t.dtype
    except RuntimeError:
        return t.data_ptr(), -1, t.dtype


def _state_key(mod: nn.Module, device):
    ts = list(mod.parameters()) + list(mod.buffers())
    return (str(device),) + tuple(_tkey(t) for t in ts)


def _cached(mod: nn.Module, device, build, slot: str = "_fce_native"):
    """Native (folded / packed / fp32) copies of a module's weights, rebuilt when any of its
    tensors changes (data_ptr / version counter / dtype) or the device differs."""
    key = _state_key(mod, device)
    c = mod.__dict__.get(slot)
    if c is None or c[0] != key:
        c = (key, build())
        mod.__dict__[slot] = c
    return c[1]


def fold_bn(conv: nn.Conv2d, bn: nn.BatchNorm2d | None):
    """fp32 (w, b) with BN folded (torch_utils.py:237-267)."""
    with torch.no_grad():
        w = conv.weight.detach().float()
        b = conv.bias.detach().float() if conv.bias is not None else torch.zeros(w.shape[0], device=w.device)
        if bn is not None:
            g, beta = bn.weight.detach().float(), bn.bias.detach().float()
            mean, var = bn.running_mean.detach().float(), bn.running_var.detach().float()
            s = g / torch.sqrt(bn.eps + var)
            w = (w.view(w.shape[0], -1) * s[:, None]).view(w.shape)
            b = s * b + (beta - g * mean / torch.sqrt(var + bn.eps))
    return w, b


def fuse_conv_bn(m: "Conv") -> None:
    """One step of ``BaseModel.fuse`` (tasks.py:231-237) with ``fuse_conv_and_bn`` (torch_utils.py:237-267):
    BN folded into ``conv.weight`` / ``conv.bias`` (eps 1e-3), ``bn`` deleted, forward -> forward_fuse.
    The kernels fold BN themselves, so this only changes the module's state_dict layout (a fused
    checkpoint loads after it)."""
    w, b = fold_bn(m.conv, m.bn)
    conv = m.conv
    with torch.no_grad():
        conv.weight.data = w.to(conv.weight.dtype)
        if conv.bias is None:
            conv.register_parameter("bias", nn.Parameter(b.to(conv.weight.dtype)))
        else:
            conv.bias.data = b.to(conv.bias.dtype)
    conv.requires_grad_(False)
    del m.bn
    m.forward = m.forward_fuse


def pack_conv(desc: N.ConvDesc, w: torch.Tensor, device) -> torch.Tensor:
    """Pack an OIHW fp32 weight into the kernel's image (C-ABI fce_conv_pack_weights) on `device`."""
    wh = np.ascontiguousarray(w.detach().float().cpu().numpy())
    nb = N.lib().fce_conv_weight_bytes(C.byref(desc))
    out = np.empty(nb, dtype=np.uint8)
    N.call("fce_conv_pack_weights", C.byref(desc), wh.ctypes.data, out.ctypes.data)
    return torch.from_numpy(out).to(device)


class _ConvNative:
    __slots__ = ("desc", "w", "b")

    def __init__(self, desc, w, b):
        self.desc, self.w, self.b = desc, w, b


def conv_native(conv: nn.Conv2d, bn: nn.BatchNorm2d | None, act: bool, device) -> _ConvNative:
    def build():
        if conv.dilation != (1, 1) or conv.kernel_size[0] != conv.kernel_size[1]:
            raise NotImplementedError("fce_yolo_amd: dilated / non-square convs are not on the YOLO11 path")
        k = conv.kernel_size[0]
        if conv.padding != (k // 2, k // 2):
            raise NotImplementedError("fce_yolo_amd: only 'same' (k//2) padding")
        w, b = fold_bn(conv, bn)
        g = conv.groups
        desc = N.ConvDesc(conv.in_channels, conv.out_channels, k, conv.stride[0], g, N.ACT_SILU if act else N.ACT_NONE,
                          0, N.EPI_STORE, None, 0, 0)
        if g not in (1, conv.in_channels) or (g > 1 and conv.in_channels != conv.out_channels):
            raise NotImplementedError("fce_yolo_amd: grouped convs other than depthwise")
        return _ConvNative(desc, pack_conv(desc, w, device), b.to(device).contiguous())

    # cached on the conv module; the key covers the conv's and the BN's tensors
    ts = list(conv.parameters()) + list(conv.buffers()) + (list(bn.parameters()) + list(bn.buffers()) if bn else [])
    key = (str(device), act) + tuple(_tkey(t) for t in ts)
    c = conv.__dict__.get("_fce_conv")
    if c is None or c[0] != key:
        c = (key, build())
        conv.__dict__["_fce_conv"] = c
    return c[1]


def _desc_copy(d: N.ConvDesc, **kw) -> N.ConvDesc:
    n = N.ConvDesc()
    C.pointer(n)[0] = d
    for k, v in kw.items():
        setattr(n, k, v)
    return n


def emit_conv(be, conv: nn.Conv2d, bn, act: bool, x: View, out: View | None = None, res: View | None = None,
              epilogue: int = N.EPI_STORE, fusion=None, out_dtype=N.F16, dup=None) -> View:
    k, s = conv.kernel_size[0], conv.stride[0]
    ho = (x.h + 2 * (k // 2) - k) // s + 1
    wo = (x.w + 2 * (k // 2) - k) // s + 1
    y = out if out is not None else be.alloc(x.n, conv.out_channels, ho, wo, out_dtype)
    assert (y.h, y.w, y.c) == (ho, wo, conv.out_channels), "output view mismatch"
    if be.shape_only:
        return y
    nat = conv_native(conv, bn, act, be.device)
    fw, fn, fi = fusion if fusion is not None else (None, 0, 0)
    desc = _desc_copy(nat.desc, epilogue=epilogue, fusion_w=fw, fusion_n=fn, fusion_i=fi)
    if x.layout == N.NCHW and conv.in_channels > 4:
        x = be.from_torch(x.buf) if isinstance(be, EagerBackend) else x
    if x.up and (k != 1 or conv.groups != 1):
        x = be.materialize(x)
    if dup is not None:
        be.conv(desc, x, y, nat.w.data_ptr(), nat.b.data_ptr(), res, dup=dup)
    else:
        be.conv(desc, x, y, nat.w.data_ptr(), nat.b.data_ptr(), res)
    return y


def conv_native_cat(owner: nn.Module, convs, act: bool, device) -> _ConvNative:
    """ONE packed 1x1 conv computing several 1x1 stride-1 convs of the same input side by side: their folded weights
    and biases concatenated along the output channels, in the order given (cached on `owner`, keyed by every conv's
    and BN's tensors).  Bitwise the separate convs: each output channel sums the same K-steps in the same order
    whatever the cout tiling, and the epilogue is per channel."""
    ts = [t for c, bn in convs for t in list(c.parameters()) + list(c.buffers()) +
          (list(bn.parameters()) + list(bn.buffers()) if bn is not None else [])]
    key = (str(device), act) + tuple(_tkey(t) for t in ts)

    def build():
        ws, bs = zip(*(fold_bn(c, bn) for c, bn in convs))
        w, b = torch.cat(ws), torch.cat(bs)
        c0 = convs[0][0]
        desc = N.ConvDesc(c0.in_channels, w.shape[0], 1, 1, 1, N.ACT_SILU if act else N.ACT_NONE, 0, N.EPI_STORE, None,
                          0, 0)
        return _ConvNative(desc, pack_conv(desc, w, device), b.to(device).contiguous())

    c = owner.__dict__.get("_fce_cat")
    if c is None or c[0] != key:
        c = (key, build())
        owner.__dict__["_fce_cat"] = c
    return c[1]


def _no_dup() -> bool:
    """C2f / C3k2 bottlenecks read their chunk from the concat record unless FCE_DUP=1 (dense copy from cv1's
    epilogue): measured on n32 the copy takes ~20 us off the 3x3 family and puts ~20 us onto the 1x1 family
    (forward 1.567-1.583 ms either way), so it stays opt-in."""
    import os

    return os.environ.get("FCE_DUP", "0") in ("", "0")


def _backend(xs):
    """EagerBackend for ROCm inputs; ShapeBackend (meta outputs, no arithmetic) for anything else."""
    devs = {t.device.type for t in xs}
    if devs == {"cuda"}:
        return EagerBackend(xs[0].device)
    if "cuda" in devs:
        raise RuntimeError(f"fce_yolo_amd: inputs on mixed devices {sorted(devs)}")
    return ShapeBackend()


def _run_eager(mod, x, *, keep_nchw=False, out_dtype=None):
    """Drop-in forward: NCHW tensor(s) in, channels_last tensor out (input dtype preserved).  A non-ROCm
    input gives a ``meta`` tensor of the output shape (see ``ShapeBackend``), never CPU arithmetic."""
    xs = x if isinstance(x, (list, tuple)) else [x]
    be = _backend(xs)
    views = [be.from_torch(t, keep_nchw=keep_nchw) for t in xs]
    y = mod.emit(be, views if isinstance(x, (list, tuple)) else views[0])
    dt = out_dtype or xs[0].dtype
    if dt not in (torch.float16, torch.float32):
        dt = torch.float16
    return be.to_torch(y, dt)


# ============================================================================ conv.py
class Conv(nn.Module):
    """conv.py:39-89: SiLU(BN(conv(x)))."""

    default_act = nn.SiLU()

    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, d=1, act=True):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, autopad(k, p, d), groups=g, dilation=d, bias=False)
        self.bn = nn.BatchNorm2d(c2, eps=BN_EPS)
        self.act = self.default_act if act is True else act if isinstance(act, nn.Module) else nn.Identity()

    def _act(self) -> bool:
        if isinstance(self.act, nn.SiLU):
            return True
        if isinstance(self.act, nn.Identity):
            return False
        raise NotImplementedError(f"fce_yolo_amd: activation {type(self.act).__name__} is not on the YOLO11 path")

    def emit(self, be, x, out=None, res=None, epilogue=N.EPI_STORE, fusion=None, out_dtype=N.F16, dup=None):
        return emit_conv(be, self.conv, getattr(self, "bn", None), self._act(), x, out, res, epilogue, fusion,
                         out_dtype, dup)

    def forward(self, x):
        return _run_eager(self, x, keep_nchw=self.conv.in_channels <= 4)

    def forward_fuse(self, x):
        """BaseModel.fuse (tasks.py:231-237) rebinds ``forward`` to this; BN folding is in conv_native."""
        return _run_eager(self, x, keep_nchw=self.conv.in_channels <= 4)


def stem_alt(be, m0, m1, first: int, saved: bool):
    """Graph backend, after the backbone's first two layers were emitted as ops [first, first + 2): where they are
    Conv(3, c0, 3, 2) -> Conv(c0, c1, 3, 2) (SiLU) with an instantiated (c0, c1) and the stem's output read by nothing
    else (`saved`: a later layer takes it), record the one-kernel form (csrc/stem_fused.hip) as their alternative.
    FCE_FUSE_STEM: unset / "auto" -- the plan keeps the faster, "1" -- the fused kernel, "0" -- the two convs only."""
    import os

    if os.environ.get("FCE_FUSE_STEM", "auto") == "0" or saved or not hasattr(be, "stem_alt"):
        return
    if type(m0) is not Conv or type(m1) is not Conv or getattr(m1, "f", -1) != -1 or be.num_ops() - first != 2:
        return
    c0, c1 = m0.conv, m1.conv
    if (c0.in_channels, c0.kernel_size[0], c0.stride[0], c0.groups) != (3, 3, 2, 1) or \
            (c1.in_channels, c1.kernel_size[0], c1.stride[0], c1.groups) != (c0.out_channels, 3, 2, 1):
        return
    if not (isinstance(m0.act, nn.SiLU) and isinstance(m1.act, nn.SiLU)):
        return
    d = N.Stem2Desc()
    d.c0, d.c1 = c0.out_channels, c1.out_channels
    for j, m in enumerate((m0, m1)):
        nat = conv_native(m.conv, getattr(m, "bn", None), True, be.device)
        d.w[j], d.b[j] = nat.w.data_ptr(), nat.b.data_ptr()
    if N.lib().fce_stem_fused_supported(C.byref(d)):
        be.stem_alt(d, first, 2)


def bneck_alt(be, blocks, x, y, first: int):
    """Graph backend, after the Bottlenecks `blocks` (a chain: the first reads `x`, each the previous one's output, the
    last writes `y`) were emitted as ops [first, first + 2 len(blocks)): where every block is a shortcut Bottleneck of
    3x3 SiLU convs with an instantiated (c, c_mid, n), record the one-kernel chain (csrc/bneck.hip) as their
    alternative.  FCE_FUSE_BNECK: unset / "auto" -- the plan keeps the faster, "1" -- the fused kernel (where the map
    width is instantiated), "0" -- the convs only."""
    import os

    if os.environ.get("FCE_FUSE_BNECK", "auto") == "0" or be.shape_only or not hasattr(be, "bneck_alt"):
        return
    n = len(blocks)
    if n not in (1, 2) or be.num_ops() - first != 2 * n or x.up or x.layout != N.NHWC or x.dtype != N.F16:
        return
    c, cm = blocks[0].cv1.conv.in_channels, blocks[0].cv1.conv.out_channels
    for m in blocks:
        if type(m) is not Bottleneck or not m.add:
            return
        for cv, ci, co in ((m.cv1, c, cm), (m.cv2, cm, c)):
            k = cv.conv
            if (k.in_channels, k.out_channels, k.kernel_size[0], k.stride[0], k.groups) != (ci, co, 3, 1, 1) or \
                    not isinstance(cv.act, nn.SiLU):
                return
    d = N.BneckDesc()
    d.c, d.c_mid, d.n, d.shortcut = c, cm, n, 1
    for j, cv in enumerate(cv for m in blocks for cv in (m.cv1, m.cv2)):
        nat = conv_native(cv.conv, getattr(cv, "bn", None), True, be.device)
        d.w[j], d.b[j] = nat.w.data_ptr(), nat.b.data_ptr()
    if N.lib().fce_bneck_supported(C.byref(d)):
        be.bneck_alt(d, x, y, first, 2 * n)


def pw2_alt(be, first: int, nat1, nat2, epi1=None):
    """Graph backend, after two 1x1 convs were emitted as ops first, first + 1 (the second reading channels of the
    first's output buffer; nat1 / nat2 their packed _ConvNative): where the channel counts are instantiated, record the
    one-kernel pair (csrc/pw2.hip) as their alternative.  `epi1` = (epilogue, fusion weights ptr, n, i) when op 1 is a
    BiFPN_Concat realign conv.  FCE_FUSE_PW2: unset / "auto" -- the plan keeps the faster, "1" -- the fused kernel,
    "0" -- the two convs only."""
    import os

    if os.environ.get("FCE_FUSE_PW2", "auto") == "0" or be.shape_only or not hasattr(be, "pw2_alt"):
        return
    if be.num_ops() - first != 2:
        return
    d = N.Pw2Desc()
    d.cin1, d.cout1, d.cin2, d.cout2 = nat1.desc.cin, nat1.desc.cout, nat2.desc.cin, nat2.desc.cout
    for j, nat in enumerate((nat1, nat2)):
        if nat.desc.k != 1 or nat.desc.stride != 1 or nat.desc.groups != 1:
            return
        d.act[j] = nat.desc.act
        d.w[j], d.b[j] = nat.w.data_ptr(), nat.b.data_ptr()
    if epi1 is not None:
        d.epi1, d.fw, d.fn, d.fi = epi1
    if N.lib().fce_pw2_supported(C.byref(d)):
        be.pw2_alt(d, first)


def _nat(m: "Conv", device):
    return conv_native(m.conv, getattr(m, "bn", None), m._act(), device)


class DWConv(Conv):
    """conv.py:185-200."""

    def __init__(self, c1, c2, k=1, s=1, d=1, act=True):
        super().__init__(c1, c2, k, s, g=math.gcd(c1, c2), d=d, act=act)


class Concat(nn.Module):
    """conv.py:616-641: torch.cat along channels as channel-offset copies into one buffer."""

    def __init__(self, dimension=1):
        super().__init__()
        self.d = dimension

    def emit(self, be, xs, out=None):
        assert self.d == 1
        c = sum(v.c for v in xs)
        y = out if out is not None else be.alloc(xs[0].n, c, xs[0].h, xs[0].w)
        off = 0
        for v in xs:
            be.wadd(v, y.slice(off, v.c), None, 0)
            off += v.c
        return y

    def forward(self, x):
        return _run_eager(self, list(x))


class Upsample(nn.Upsample):
    """nn.Upsample(None, 2, 'nearest') fused into the consumer's loads (lazy view)."""

    def emit(self, be, x, out=None):
        if self.mode != "nearest" or float(self.scale_factor) != 2.0:
            raise NotImplementedError("fce_yolo_amd: only nearest x2 upsampling")
        v = x.upsampled(2)
        return v if out is None else be.wadd(v, out, None, 0) or out

    def forward(self, x):
        return _run_eager(self, x)


# ============================================================================ block.py
class Bottleneck(nn.Module):
    """block.py:452-476."""

    def __init__(self, c1, c2, shortcut=True, g=1, k=(3, 3), e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, k[0], 1)
        self.cv2 = Conv(c_, c2, k[1], 1, g=g)
        self.add = shortcut and c1 == c2

    def emit(self, be, x, out=None):
        h = self.cv1.emit(be, x)
        return self.cv2.emit(be, h, out=out, res=x if self.add else None)

    def forward(self, x):
        return _run_eager(self, x)


class C2f(nn.Module):
    """block.py:270-315: cv1 -> chunk(2) -> n blocks -> cat -> cv2; the cat is one buffer."""

    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5):
        super().__init__()
        self.c = int(c2 * e)
        self.cv1 = Conv(c1, 2 * self.c, 1, 1)
        self.cv2 = Conv((2 + n) * self.c, c2, 1)
        self.m = nn.ModuleList(Bottleneck(self.c, self.c, shortcut, g, k=((3, 3), (3, 3)), e=1.0) for _ in range(n))

    def emit(self, be, x, out=None, bneck=True):
        """`bneck`: record each Bottleneck's one-kernel alternative (bneck_alt; off where the caller records the
        whole block's)."""
        c, n = self.c, len(self.m)
        # a BiFPN_Concat whose last term is a realign conv, emitted just before and read here whole: that conv and cv1
        # as a fused 1x1 pair (not where the block records its own one-kernel form, or cv1 opens a C3k pair)
        bifpn = be.__dict__.pop("_bifpn_last", None)
        buf = be.alloc(x.n, (2 + n) * c, x.h, x.w)
        # the chunk the first block reads (and adds back) is a c-channel slice of the (2 + n) c record: when that
        # slice is narrower than a 128-byte line (c < 64), whole-graph lowering can also store it densely from
        # cv1's epilogue (FCE_DUP=1), so the block's 3x3 convs read whole cache lines (n32: 1.5-2.3x the
        # algorithmic bytes are fetched through the slice)
        dense = None
        k1 = be.num_ops() if hasattr(be, "num_ops") else None
        if getattr(be, "supports_dup", False) and n and c % 8 == 0 and c < 64 and not _no_dup():
            dense = be.alloc(x.n, c, x.h, x.w)
            self.cv1.emit(be, x, out=buf.slice(0, 2 * c), dup=(dense, c))
        else:
            self.cv1.emit(be, x, out=buf.slice(0, 2 * c))
        if n and isinstance(self.m[0], C3) and dense is None and k1 is not None and not be.shape_only:
            self.m[0]._pre_pair = (k1, _nat(self.cv1, be.device))  # cv1 -> the C3k's merged cv1 / cv2 (pw2_alt)
        elif bifpn is not None and bneck and k1 is not None and bifpn[0] + 1 == k1 and bifpn[1] == (x.buf, x.coff, x.c, x.up):
            pw2_alt(be, bifpn[0], bifpn[2], _nat(self.cv1, be.device), bifpn[3])  # realign (ACCUM) -> cv1
        for i, m in enumerate(self.m):
            src = dense if (i == 0 and dense is not None) else buf.slice((1 + i) * c, c)
            first = be.num_ops() if hasattr(be, "num_ops") else None
            y = m.emit(be, src, out=buf.slice((2 + i) * c, c))
            if bneck and first is not None and type(m) is Bottleneck:
                bneck_alt(be, [m], src, y, first)
        k2 = be.num_ops() if hasattr(be, "num_ops") else None
        y = self.cv2.emit(be, buf, out=out)
        if n and isinstance(self.m[-1], C3) and k2 is not None and not be.shape_only:
            pw2_alt(be, k2 - 1, _nat(self.m[-1].cv3, be.device), _nat(self.cv2, be.device))  # C3k cv3 -> cv2
        return y

    def forward(self, x):
        return _run_eager(self, x)


class C3(nn.Module):
    """block.py:318-340."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.cv3 = Conv(2 * c_, c2, 1)
        self.m = nn.Sequential(*(Bottleneck(c_, c_, shortcut, g, k=((1, 1), (3, 3)), e=1.0) for _ in range(n)))

    def _cat_ok(self) -> bool:
        """cv1 and cv2 (both 1x1 s1 over x, block.py:337-339) can run as one conv with concatenated weights
        (FCE_C3_CAT=0: two convs)."""
        import os

        if os.environ.get("FCE_C3_CAT", "1") == "0" or not len(self.m):
            return False
        c1, c2 = self.cv1.conv, self.cv2.conv
        return all(c.kernel_size[0] == 1 and c.stride[0] == 1 and c.groups == 1 for c in (c1, c2)) and \
            self.cv1._act() == self.cv2._act() and c1.out_channels % 8 == 0 and c2.out_channels % 8 == 0

    def emit(self, be, x, out=None):
        c_ = self.cv1.conv.out_channels
        pre = self.__dict__.pop("_pre_pair", None)  # set by an enclosing C3k2 (C2f.emit) for the cv1 -> cv1 / cv2 pair
        if self._cat_ok():
            # rec = [m | b | a]: cv3 reads [m | b] (cat(m(cv1(x)), cv2(x)), block.py:340), and b = cv2(x), a = cv1(x)
            # come from ONE conv over x (x read once, one launch); below 64 channels a dense copy of a is stored too
            # (the bottlenecks' 3x3 then reads whole lines, as FCE_DUP does for C2f)
            c2 = self.cv2.conv.out_channels
            rec = be.alloc(x.n, 2 * c_ + c2, x.h, x.w)
            y = rec.slice(c_, c2 + c_)
            a = rec.slice(c_ + c2, c_)
            if not be.shape_only:
                nat = conv_native_cat(self, [(self.cv2.conv, getattr(self.cv2, "bn", None)),
                                             (self.cv1.conv, getattr(self.cv1, "bn", None))], self.cv1._act(), be.device)
                xin = be.from_torch(x.buf) if (x.layout == N.NCHW and isinstance(be, EagerBackend)) else x
                if getattr(be, "supports_dup", False) and c_ < 64 and not x.up:
                    a = be.alloc(x.n, c_, x.h, x.w)
                    be.conv(nat.desc, xin, y, nat.w.data_ptr(), nat.b.data_ptr(), None, dup=(a, c2))
                else:
                    be.conv(nat.desc, xin, y, nat.w.data_ptr(), nat.b.data_ptr(), None)
                if pre is not None:  # the enclosing C3k2's cv1 was the op before: the pair as one kernel
                    pw2_alt(be, pre[0], pre[1], nat)
            first, x0 = (be.num_ops() if hasattr(be, "num_ops") else None), a
            for i, m in enumerate(self.m):
                a = m.emit(be, a, out=rec.slice(0, c_) if i == len(self.m) - 1 else None)
            if first is not None:
                bneck_alt(be, list(self.m), x0, a, first)
            return self.cv3.emit(be, rec.slice(0, c_ + c2), out=out)
        buf = be.alloc(x.n, 2 * c_, x.h, x.w)
        a = self.cv1.emit(be, x) if len(self.m) else self.cv1.emit(be, x, out=buf.slice(0, c_))
        first, x0 = (be.num_ops() if hasattr(be, "num_ops") else None), a
        for i, m in enumerate(self.m):
            a = m.emit(be, a, out=buf.slice(0, c_) if i == len(self.m) - 1 else None)
        if first is not None and len(self.m):
            bneck_alt(be, list(self.m), x0, a, first)
        self.cv2.emit(be, x, out=buf.slice(c_, c_))
        return self.cv3.emit(be, buf, out=out)

    def forward(self, x):
        return _run_eager(self, x)


class C3k(C3):
    """block.py:1087-1108."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5, k=3):
        super().__init__(c1, c2, n, shortcut, g, e)
        c_ = int(c2 * e)
        self.m = nn.Sequential(*(Bottleneck(c_, c_, shortcut, g, k=(k, k), e=1.0) for _ in range(n)))


class C3k2(C2f):
    """block.py:1064-1084.  With c3k = False and one Bottleneck repeat (the n / s scales' C3k2 at
    160^2 .. 40^2) the whole block can run as ONE persistent kernel (csrc/fused.hip: x read once, the
    intermediates in LDS, bitwise equal to the four convs).  FCE_FUSE_C3K2 (whole-graph lowering):
    unset / "auto" -- both forms are recorded (fce_net_add_c3k2_alt) and the plan-time autotune keeps the
    faster per block; "1" -- always the fused kernel (also in the eager drop-in forward); "0" -- never;
    a number N > 1 -- fused (forced) where h * w <= N."""

    def __init__(self, c1, c2, n=1, c3k=False, e=0.5, g=1, shortcut=True):
        super().__init__(c1, c2, n, shortcut, g, e)
        self.m = nn.ModuleList(
            C3k(self.c, self.c, 2, shortcut, g) if c3k else Bottleneck(self.c, self.c, shortcut, g) for _ in range(n)
        )

    @staticmethod
    def _mode() -> str:
        import os

        return os.environ.get("FCE_FUSE_C3K2", "auto") or "auto"

    def _fused_desc(self, be, x):
        mode = self._mode()
        if be.shape_only or mode == "0" or not hasattr(be, "c3k2"):
            return None
        if mode not in ("1", "auto") and x.h * x.w > int(mode):
            return None
        if len(self.m) != 1 or type(self.m[0]) is not Bottleneck or not self.m[0].add:
            return None
        if x.up or x.layout != N.NHWC or x.dtype != N.F16:
            return None
        bt = self.m[0]
        convs = (self.cv1, bt.cv1, bt.cv2, self.cv2)
        for cv, k in zip(convs, (1, 3, 3, 1)):
            c = cv.conv
            if (c.kernel_size[0] != k or c.stride[0] != 1 or c.groups != 1 or not isinstance(cv.act, nn.SiLU)):
                return None
        d = N.C3k2Desc()
        d.cin, d.c, d.c_mid, d.cout = self.cv1.conv.in_channels, self.c, bt.cv1.conv.out_channels, self.cv2.conv.out_channels
        if bt.cv1.conv.in_channels != self.c or bt.cv2.conv.out_channels != self.c:
            return None
        for i, cv in enumerate(convs):
            nat = conv_native(cv.conv, getattr(cv, "bn", None), True, be.device)
            d.w[i], d.b[i] = nat.w.data_ptr(), nat.b.data_ptr()
        return d if N.lib().fce_c3k2_supported(C.byref(d)) else None

    def emit(self, be, x, out=None):
        d = self._fused_desc(be, x)
        if d is None:
            return super().emit(be, x, out)
        if self._mode() == "auto":
            if not hasattr(be, "c3k2_alt"):  # eager drop-in: the four convs (no plan-time choice there)
                return super().emit(be, x, out)
            # both forms: the four convs, then the fused op as their alternative (the plan keeps the faster)
            first = be.num_ops()
            y = super().emit(be, x, out, bneck=False)
            n = be.num_ops() - first
            if n == 4:
                be.c3k2_alt(d, x, y, first, n)
            return y
        y = out if out is not None else be.alloc(x.n, self.cv2.conv.out_channels, x.h, x.w)
        be.c3k2(d, x, y)
        return y


class SPPF(nn.Module):
    """block.py:205-232; the three chained MaxPool2d(5,1,2) run as one kernel into the concat buffer."""

    def __init__(self, c1, c2, k=5):
        super().__init__()
        c_ = c1 // 2
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_ * 4, c2, 1, 1)
        self.m = nn.MaxPool2d(kernel_size=k, stride=1, padding=k // 2)

    def emit(self, be, x, out=None):
        c_ = self.cv1.conv.out_channels
        buf = be.alloc(x.n, 4 * c_, x.h, x.w)
        self.cv1.emit(be, x, out=buf.slice(0, c_))
        be.maxpool_chain(buf, c_, self.m.kernel_size if isinstance(self.m.kernel_size, int) else self.m.kernel_size[0])
        return self.cv2.emit(be, buf, out=out)

    def forward(self, x):
        return _run_eager(self, x)


class Attention(nn.Module):
    """block.py:1247-1304."""

    def __init__(self, dim, num_heads=8, attn_ratio=0.5):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.key_dim = int(self.head_dim * attn_ratio)
        self.scale = self.key_dim**-0.5
        nh_kd = self.key_dim * num_heads
        h = dim + nh_kd * 2
        self.qkv = Conv(dim, h, 1, act=False)
        self.proj = Conv(dim, dim, 1, act=False)
        self.pe = Conv(dim, dim, 3, 1, g=dim, act=False)

    def _pe(self, device):
        def build():
            w, b = fold_bn(self.pe.conv, getattr(self.pe, "bn", None))
            return w.reshape(w.shape[0], 9).t().contiguous().to(device), b.contiguous().to(device)  # [9][C]

        return _cached(self.pe, device, build, "_fce_pe")

    def emit(self, be, x, out=None, res=None):
        qkv = self.qkv.emit(be, x)
        pre = self.__dict__.pop("_pre_pair", None)
        if pre is not None:  # C2PSA's cv1 was the op before: the pair as one kernel
            pw2_alt(be, pre[0], pre[1], _nat(self.qkv, be.device))
        o = be.alloc(x.n, self.num_heads * self.head_dim, x.h, x.w)
        if not be.shape_only:
            pw, pb = self._pe(be.device)
            be.psa(qkv, self.num_heads, self.key_dim, self.head_dim, pw.data_ptr(), pb.data_ptr(), o)
        return self.proj.emit(be, o, out=out, res=res)

    def forward(self, x):
        return _run_eager(self, x)


class PSABlock(nn.Module):
    """block.py:1307-1354."""

    def __init__(self, c, attn_ratio=0.5, num_heads=4, shortcut=True):
        super().__init__()
        self.attn = Attention(c, attn_ratio=attn_ratio, num_heads=num_heads)
        self.ffn = nn.Sequential(Conv(c, c * 2, 1), Conv(c * 2, c, 1, act=False))
        self.add = shortcut

    def emit(self, be, x, out=None):
        x1 = self.attn.emit(be, x, res=x if self.add else None)
        k = be.num_ops() if hasattr(be, "num_ops") else None
        f = self.ffn[0].emit(be, x1)
        if k is not None and not be.shape_only:  # attn.proj (+ x) -> ffn[0]
            pw2_alt(be, k - 1, _nat(self.attn.proj, be.device), _nat(self.ffn[0], be.device))
        return self.ffn[1].emit(be, f, out=out, res=x1 if self.add else None)

    def forward(self, x):
        return _run_eager(self, x)


class C2PSA(nn.Module):
    """block.py:1412-1464."""

    def __init__(self, c1, c2, n=1, e=0.5):
        super().__init__()
        assert c1 == c2
        self.c = int(c1 * e)
        self.cv1 = Conv(c1, 2 * self.c, 1, 1)
        self.cv2 = Conv(2 * self.c, c1, 1)
        self.m = nn.Sequential(*(PSABlock(self.c, attn_ratio=0.5, num_heads=self.c // 64) for _ in range(n)))

    def emit(self, be, x, out=None):
        c = self.c
        k1 = be.num_ops() if hasattr(be, "num_ops") else None
        buf = self.cv1.emit(be, x)  # [a | b]
        if len(self.m) and k1 is not None and not be.shape_only:
            self.m[0].attn._pre_pair = (k1, _nat(self.cv1, be.device))  # cv1 -> attn.qkv (pw2_alt)
        b = buf.slice(c, c)
        for i, m in enumerate(self.m):
            b = m.emit(be, b, out=buf.slice(c, c) if i == len(self.m) - 1 else None)
        k2 = be.num_ops() if hasattr(be, "num_ops") else None
        y = self.cv2.emit(be, buf, out=out)
        if len(self.m) and k2 is not None and not be.shape_only:  # the last ffn[1] (+ x1) -> cv2
            pw2_alt(be, k2 - 1, _nat(self.m[-1].ffn[1], be.device), _nat(self.cv2, be.device))
        return y

    def forward(self, x):
        return _run_eager(self, x)


# ============================================================================ fce_block.py
class BiFPN_Concat(nn.Module):
    """fce_block.py:13-63: sum_i relu(w_i)/(sum relu(w)+1e-4) * realign_i(x_i).

    Realign convs run with a weighted-store / accumulate epilogue into one output buffer; Identity
    branches (and upsampled inputs) use the weighted-add kernel; the normalised weights are
    computed on the device from ``w`` so a captured graph needs no host round trip."""

    def __init__(self, c1, c2=None):
        super().__init__()
        self.output_ch = c2 if c2 else max(c1)
        self.realign_convs = nn.ModuleList()
        for ch in c1:
            if ch != self.output_ch:
                self.realign_convs.append(Conv(ch, self.output_ch, 1, 1))
            else:
                self.realign_convs.append(nn.Identity())
        self.w = nn.Parameter(torch.ones(len(c1), dtype=torch.float32), requires_grad=True)
        self.epsilon = 1e-4

    def _w32(self, device):
        return _cached(self, device, lambda: self.w.detach().float().to(device).contiguous(), "_fce_w")

    def emit(self, be, xs, out=None):
        h, w = xs[0].h, xs[0].w
        y = out if out is not None else be.alloc(xs[0].n, self.output_ch, h, w)
        wp = None if be.shape_only else self._w32(be.device).data_ptr()
        n = len(xs)
        for i, (x, m) in enumerate(zip(xs, self.realign_convs)):
            assert (x.h, x.w) == (h, w), "BiFPN_Concat inputs must share the spatial size"
            if isinstance(m, nn.Identity):
                be.wadd(x, y, (wp, n, i), accumulate=int(i > 0))
            else:
                k = be.num_ops() if hasattr(be, "num_ops") and not be.shape_only else None
                epi = N.EPI_ACCUM if i else N.EPI_WSTORE
                m.emit(be, x, out=y, epilogue=epi, fusion=(wp, n, i))
                if k is not None and i == n - 1 and i > 0 and x.up == 0:  # the last term: a pair with the consumer's cv1
                    be._bifpn_last = (k, (y.buf, y.coff, y.c, y.up), _nat(m, be.device), (epi, wp, n, i))
        return y

    def forward(self, x):
        return _run_eager(self, list(x))


def _dense(mod: nn.Conv2d, device):
    """fp32 transposed [in][out] matrix + bias of a 1x1 nn.Conv2d (device)."""

    def build():
        w = mod.weight.detach().float().reshape(mod.out_channels, -1).t().contiguous().to(device)
        b = (mod.bias.detach().float() if mod.bias is not None else torch.zeros(mod.out_channels)).to(device)
        return w, b.contiguous()

    return _cached(mod, device, build, "_fce_dense")


def _coord_desc(inp, oup, mid, heads, scale, mats, identity, device):
    d = N.CoordDesc()
    d.inp, d.oup, d.mid, d.heads, d.scale = inp, oup, mid, heads, float(scale)
    for i, (w, b) in enumerate(mats):
        d.w[i] = w.data_ptr()
        d.b[i] = b.data_ptr()
    if isinstance(identity, nn.Conv2d):
        nat = conv_native(identity, None, False, device)
        d.id_w, d.id_b = nat.w.data_ptr(), nat.b.data_ptr()
    return d


class CoordAtt(nn.Module):
    """fce_block.py:65-116."""

    def __init__(self, inp, oup, reduction=32):
        super().__init__()
        self.pool_h = nn.AdaptiveAvgPool2d((None, 1))
        self.pool_w = nn.AdaptiveAvgPool2d((1, None))
        mip = max(8, inp // reduction)
        self.cv1 = Conv(inp, mip, k=1, s=1, p=0)
        self.cv_h = nn.Conv2d(mip, oup, kernel_size=1, stride=1, padding=0)
        self.cv_w = nn.Conv2d(mip, oup, kernel_size=1, stride=1, padding=0)
        self.identity = nn.Conv2d(inp, oup, 1) if inp != oup else nn.Identity()

    def emit(self, be, x, out=None):
        inp, mip, oup = self.cv1.conv.in_channels, self.cv1.conv.out_channels, self.cv_h.out_channels
        if be.shape_only:
            return out if out is not None else be.alloc(x.n, oup, x.h, x.w)

        def build():
            w, b = fold_bn(self.cv1.conv, getattr(self.cv1, "bn", None))
            return w.reshape(mip, inp).t().contiguous().to(be.device), b.contiguous().to(be.device)

        cv1 = _cached(self.cv1, be.device, build, "_fce_cv1")
        d = _coord_desc(inp, oup, mip, 1, 1.0, [cv1, _dense(self.cv_h, be.device), _dense(self.cv_w, be.device)],
                        self.identity, be.device)
        y = out if out is not None else be.alloc(x.n, oup, x.h, x.w)
        be.coord(1, d, x, y)
        return y

    def forward(self, x):
        return _run_eager(self, x)


class CoordCrossAtt(nn.Module):
    """fce_block.py:119-180 (oup must equal inp, Q3)."""

    def __init__(self, inp, oup, reduction=32, num_heads=1):
        super().__init__()
        self.mip = max(8, inp // reduction)
        self.num_heads = num_heads
        self.scale = (self.mip // num_heads) ** -0.5
        self.pool_h = nn.AdaptiveAvgPool2d((None, 1))
        self.pool_w = nn.AdaptiveAvgPool2d((1, None))
        self.cv1 = nn.Conv2d(inp, self.mip, kernel_size=1)
        self.q_conv = nn.Conv2d(self.mip, self.mip, 1)
        self.k_conv = nn.Conv2d(self.mip, self.mip, 1)
        self.v_conv = nn.Conv2d(self.mip, self.mip, 1)
        self.proj = nn.Conv2d(self.mip, oup, 1)
        self.gate = nn.Sigmoid()

    def emit(self, be, x, out=None):
        inp, oup = self.cv1.in_channels, self.proj.out_channels
        if inp != oup:
            raise RuntimeError("CoordCrossAtt: oup != inp cannot broadcast x * y_att (reference fce_block.py:180)")
        if be.shape_only:
            return out if out is not None else be.alloc(x.n, oup, x.h, x.w)
        mats = [_dense(m, be.device) for m in (self.cv1, self.q_conv, self.k_conv, self.v_conv, self.proj)]
        d = _coord_desc(inp, oup, self.mip, self.num_heads, self.scale, mats, None, be.device)
        y = out if out is not None else be.alloc(x.n, oup, x.h, x.w)
        be.coord(2, d, x, y)
        return y

    def forward(self, x):
        return _run_eager(self, x)


class BiCoordCrossAtt(nn.Module):
    """fce_block.py:183-284: x * sigmoid(gate_h[H] + gate_w[W]) with axial cross-attention gates."""

    def __init__(self, inp, oup, reduction=32, num_heads=4):
        super().__init__()
        self.num_heads = num_heads
        self.dim_head = max(8, inp // reduction) // num_heads
        self.mid_dim = self.dim_head * num_heads
        self.scale = self.dim_head**-0.5
        self.pool_h = nn.AdaptiveAvgPool2d((None, 1))
        self.pool_w = nn.AdaptiveAvgPool2d((1, None))
        self.proj_q_h = nn.Conv2d(inp, self.mid_dim, 1)
        self.proj_k_h = nn.Conv2d(inp, self.mid_dim, 1)
        self.proj_v_h = nn.Conv2d(inp, self.mid_dim, 1)
        self.out_h = nn.Conv2d(self.mid_dim, oup, 1)
        self.proj_q_w = nn.Conv2d(inp, self.mid_dim, 1)
        self.proj_k_w = nn.Conv2d(inp, self.mid_dim, 1)
        self.proj_v_w = nn.Conv2d(inp, self.mid_dim, 1)
        self.out_w = nn.Conv2d(self.mid_dim, oup, 1)
        self.gate = nn.Sigmoid()
        self.identity = nn.Conv2d(inp, oup, 1) if inp != oup else nn.Identity()

    def emit(self, be, x, out=None):
        inp, oup = self.proj_q_h.in_channels, self.out_h.out_channels
        if be.shape_only:
            return out if out is not None else be.alloc(x.n, oup, x.h, x.w)
        mods = (self.proj_q_h, self.proj_k_h, self.proj_v_h, self.proj_q_w, self.proj_k_w, self.proj_v_w,
                self.out_h, self.out_w)
        d = _coord_desc(inp, oup, self.mid_dim, self.num_heads, self.scale, [_dense(m, be.device) for m in mods],
                        self.identity, be.device)
        y = out if out is not None else be.alloc(x.n, oup, x.h, x.w)
        be.coord(0, d, x, y)
        return y

    def forward(self, x):
        return _run_eager(self, x)


# ============================================================================ head.py
class DFL(nn.Module):
    """block.py:58-80 (the fixed arange(c1) projection; the decode kernel applies it)."""

    def __init__(self, c1=16):
        super().__init__()
        self.conv = nn.Conv2d(c1, 1, 1, bias=False).requires_grad_(False)
        x = torch.arange(c1, dtype=torch.float)
        self.conv.weight.data[:] = nn.Parameter(x.view(1, c1, 1, 1))
        self.c1 = c1


class Detect(nn.Module):
    """head.py:26-212 (legacy=False cls branch, Q5).

    Eval mode returns ``(y, maps)`` and train mode the raw ``maps`` list, as ``head.py:114-124`` does;
    the reference's stride probe (``tasks.py:396-411``) runs train mode on a CPU tensor, which goes
    through ``ShapeBackend`` (meta maps of the right shapes).  ``anchors`` / ``strides`` are the
    reference's class-level tensors, so ``BaseModel._apply`` (``tasks.py:276-293``) can move them."""

    dynamic = False
    export = False
    format = None
    end2end = False
    max_det = 300
    shape = None
    anchors = torch.empty(0)
    strides = torch.empty(0)
    legacy = False
    xyxy = False

    def __init__(self, nc=80, ch=()):
        super().__init__()
        self.nc = nc
        self.nl = len(ch)
        self.reg_max = 16
        self.no = nc + self.reg_max * 4
        self.stride = torch.zeros(self.nl)
        c2, c3 = max((16, ch[0] // 4, self.reg_max * 4)), max(ch[0], min(self.nc, 100))
        self.cv2 = nn.ModuleList(
            nn.Sequential(Conv(x, c2, 3), Conv(c2, c2, 3), nn.Conv2d(c2, 4 * self.reg_max, 1)) for x in ch
        )
        self.cv3 = (
            nn.ModuleList(nn.Sequential(Conv(x, c3, 3), Conv(c3, c3, 3), nn.Conv2d(c3, self.nc, 1)) for x in ch)
            if self.legacy
            else nn.ModuleList(
                nn.Sequential(
                    nn.Sequential(DWConv(x, x, 3), Conv(x, c3, 1)),
                    nn.Sequential(DWConv(c3, c3, 3), Conv(c3, c3, 1)),
                    nn.Conv2d(c3, self.nc, 1),
                )
                for x in ch
            )
        )
        self.dfl = DFL(self.reg_max) if self.reg_max > 1 else nn.Identity()

    def level_strides(self) -> list[float]:
        s = [float(v) for v in self.stride]
        if not all(s):
            raise RuntimeError("Detect.stride is not set (DetectionModel sets [8, 16, 32])")
        return s

    def bias_init(self):
        """head.py:169-180 (box bias 1, cls bias log(5 / nc / (640 / s)^2)); needs the strides."""
        for a, b, s in zip(self.cv2, self.cv3, self.stride):
            a[-1].bias.data[:] = 1.0
            b[-1].bias.data[: self.nc] = math.log(5 / self.nc / (640 / s) ** 2)

    def _branches(self, be, x, i):
        """Features feeding the last 1x1 convs of level i: (box branch, cls branch)."""
        b = self.cv2[i][1].emit(be, self.cv2[i][0].emit(be, x))
        seq = self.cv3[i]
        if self.legacy:
            c = seq[1].emit(be, seq[0].emit(be, x))
        else:
            c = seq[0][1].emit(be, seq[0][0].emit(be, x))
            c = seq[1][1].emit(be, seq[1][0].emit(be, c))
        return b, c

    def _finals(self, i):
        return ((0, self.cv2[i][2]), (1, self.cv3[i][2]))

    def _raw_map(self, be, feats, i):
        """cat(cv2[i](x), cv3[i](x)) as one fp32 (B, no, h, w) buffer (head.py:118)."""
        b, c = feats
        mp = be.alloc(b.n, self.no, b.h, b.w, N.F32)
        emit_conv(be, self.cv2[i][2], None, False, b, out=mp.slice(0, 4 * self.reg_max))
        emit_conv(be, self.cv3[i][2], None, False, c, out=mp.slice(4 * self.reg_max, self.nc))
        return mp

    def emit_maps(self, be, xs):
        """Train-mode head (head.py:118-120): the raw maps only, no decode (strides not needed)."""
        return [self._raw_map(be, self._branches(be, x, i), i) for i, x in enumerate(xs)]

    def emit(self, be, xs, out=None):
        """Graph backend: the box / cls logits never leave the last convs (fp32 DFL decode + sigmoid in
        the epilogue, written straight into pred).  Eager backend: the same fused kernels produce pred
        (bit-identical to the graph path) and fp32 raw maps are also written for the reference's
        ``(y, x)`` return (head.py:122-124)."""
        fused_only = getattr(be, "fused_detect", False)
        A = sum(v.h * v.w for v in xs)
        if be.shape_only:
            pred = torch.empty((xs[0].n, 4 + self.nc, A), dtype=torch.float32, device="meta")
            return pred, self.emit_maps(be, xs)
        strides = self.level_strides()
        pred, maps = None, []
        if not fused_only:
            pred = torch.empty((xs[0].n, 4 + self.nc, A), dtype=torch.float32, device=be.device)
        off = 0
        for i, x in enumerate(xs):
            if fused_only:
                self._emit_level(be, x, i, strides[i])
                continue
            feats = self._branches(be, x, i)
            maps.append(self._raw_map(be, feats, i))
            for (part, conv), v in zip(self._finals(i), feats):
                nat = conv_native(conv, None, False, be.device)
                be.conv_detect(nat.desc, v, pred, A, off, part, strides[i], self.nc, self.reg_max,
                               nat.w.data_ptr(), nat.b.data_ptr())
            off += x.h * x.w
        return pred, maps

    def _tail(self, be, part, conv, v, i, stride):
        nat = conv_native(conv, None, False, be.device)
        be.conv_detect(nat.desc, v, part, i, stride, self.nc, self.reg_max, nat.w.data_ptr(), nat.b.data_ptr())

    def _emit_level(self, be, x, i, stride):
        """Graph backend, level i: the box branch and its DFL tail, then the cls branch and its sigmoid tail (the box
        tail zeroes the level's best-class keys that the cls tail maxes into).  Where csrc/detect_cls.hip has the
        level's (c0, c3, nc), the cls branch's five ops get the one-kernel form as their alternative
        (fce_net_add_detect_cls_alt; FCE_FUSE_DCLS: unset / "auto" -- the plan keeps the faster, "1" -- the fused
        kernel, "0" -- the five ops only)."""
        self._tail(be, 0, self.cv2[i][2], self.cv2[i][1].emit(be, self.cv2[i][0].emit(be, x)), i, stride)
        d = self._dcls_desc(be, x, i)
        first = be.num_ops() if d is not None else 0
        seq = self.cv3[i]
        if self.legacy:
            c = seq[1].emit(be, seq[0].emit(be, x))
        else:
            c = seq[0][1].emit(be, seq[0][0].emit(be, x))
            c = seq[1][1].emit(be, seq[1][0].emit(be, c))
        self._tail(be, 1, seq[2], c, i, stride)
        if d is not None and be.num_ops() - first == 5:
            be.detect_cls_alt(d, x, first, 5)

    def _dcls_desc(self, be, x, i):
        """fce_dcls_desc of level i's cls branch, or None where the one-kernel form does not apply."""
        import os

        if os.environ.get("FCE_FUSE_DCLS", "auto") == "0" or self.legacy or not hasattr(be, "detect_cls_alt"):
            return None
        if x.up or x.layout != N.NHWC or x.dtype != N.F16:
            return None
        seq = self.cv3[i]
        convs = (seq[0][0], seq[0][1], seq[1][0], seq[1][1])
        for cv, k in zip(convs, (3, 1, 3, 1)):
            c = cv.conv
            if c.kernel_size[0] != k or c.stride[0] != 1 or not isinstance(cv.act, nn.SiLU):
                return None
        d = N.DclsDesc()
        d.c0, d.c3, d.nc = x.c, seq[0][1].conv.out_channels, self.nc
        for j, cv in enumerate(convs):
            nat = conv_native(cv.conv, getattr(cv, "bn", None), True, be.device)
            d.w[j], d.b[j] = nat.w.data_ptr(), nat.b.data_ptr()
        nat = conv_native(seq[2], None, False, be.device)
        d.w[4], d.b[4] = nat.w.data_ptr(), nat.b.data_ptr()
        return d if N.lib().fce_detect_cls_supported(C.byref(d)) else None

    def forward(self, x):
        xs = list(x)
        be = _backend(xs)
        views = [be.from_torch(t) for t in xs]
        if self.training:
            return [be.to_torch(m, torch.float32) for m in self.emit_maps(be, views)]
        pred, maps = self.emit(be, views)
        return pred, [be.to_torch(m, torch.float32) for m in maps]
