"""Backends for the same module lowering (``Module.emit(be, x, out=None)``):

* ``EagerBackend`` — drop-in mode: each op runs immediately through the C-ABI on torch-allocated
  channels_last fp16 buffers on the current HIP stream (what ``nn.Module.forward`` uses).
* ``NetBackend``  — whole-graph mode: each op is recorded into a native ``fce_net`` (buffer
  arena + launch list, hipGraph replay).  The Python side only lowers once.
* ``ShapeBackend`` — shape propagation only (``meta`` tensors out) for non-ROCm inputs, such as
  the reference's CPU stride probe while it builds a model.

A ``View`` is an NHWC channel slice [coff, coff+c) of a buffer with ``cstride`` channels, at
logical size (h, w); ``up`` > 0 marks a lazily nearest-upsampled view of a (h>>up, w>>up) buffer
(nn.Upsample fused into the consumer's loads).  The network input is an NCHW view.
"""

from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, replace

import torch

from . import _native as N


@dataclass
class View:
    buf: object  # torch.Tensor (eager) | int buffer id (net; -1 = network input)
    n: int
    c: int
    h: int
    w: int
    cstride: int
    coff: int = 0
    dtype: int = N.F16
    layout: int = N.NHWC
    up: int = 0

    def slice(self, coff: int, c: int) -> "View":
        assert self.layout == N.NHWC and self.up == 0 and coff + c <= self.c
        return replace(self, coff=self.coff + coff, c=c)

    def upsampled(self, f: int = 2) -> "View":
        assert f == 2, "only nearest x2 upsampling is fused"
        return replace(self, h=self.h * 2, w=self.w * 2, up=self.up + 1)


_TORCH_DT = {N.F16: torch.float16, N.F32: torch.float32, N.U8: torch.uint8}
_FCE_DT = {torch.float16: N.F16, torch.float32: N.F32, torch.uint8: N.U8}


def _fusion(fusion):
    if fusion is None:
        return None, 0, 0
    w, n, i = fusion
    return w, n, i


class EagerBackend:
    """Runs every op immediately (drop-in nn.Module path)."""

    shape_only = False

    def __init__(self, device: torch.device):
        self.device = device
        self.stream = torch.cuda.current_stream(device).cuda_stream

    # ---------------------------------------------------------------- buffers
    def alloc(self, n, c, h, w, dtype=N.F16) -> View:
        t = torch.empty((n, c, h, w), dtype=_TORCH_DT[dtype], device=self.device, memory_format=torch.channels_last)
        return View(t, n, c, h, w, c, 0, dtype)

    def from_torch(self, x: torch.Tensor, keep_nchw: bool = False) -> View:
        if x.device.type != "cuda":
            raise RuntimeError("fce_yolo_amd: the HIP path needs a ROCm device tensor (no CPU fallback)")
        n, c, h, w = x.shape
        if keep_nchw and x.dtype in _FCE_DT and x.is_contiguous():
            return View(x, n, c, h, w, c, 0, _FCE_DT[x.dtype], N.NCHW)
        if x.dtype == torch.float16 and x.is_contiguous(memory_format=torch.channels_last):
            return View(x, n, c, h, w, c)
        if x.dtype not in _FCE_DT:
            x = x.float()
        if not (x.is_contiguous() or x.is_contiguous(memory_format=torch.channels_last)):
            x = x.contiguous()
        nchw = x.is_contiguous()
        src = View(x, n, c, h, w, c, 0, _FCE_DT[x.dtype], N.NCHW if nchw else N.NHWC)
        dst = self.alloc(n, c, h, w)
        N.call("fce_copy", C.byref(self.t(src)), C.byref(self.t(dst)), self.stream)
        return dst

    def to_torch(self, v: View, dtype=torch.float16) -> torch.Tensor:
        v = self.materialize(v)
        t = v.buf[:, v.coff : v.coff + v.c] if (v.coff or v.c != v.cstride) else v.buf
        return t if t.dtype == dtype else t.to(dtype)

    def t(self, v: View) -> N.Tensor:
        assert v.up == 0
        return N.Tensor(v.buf.data_ptr(), v.dtype, v.layout, v.n, v.c, v.h, v.w, v.cstride, v.coff)

    def src_t(self, v: View) -> N.Tensor:
        """Tensor struct of the *source* buffer of a (possibly upsampled) view."""
        s = v.up
        return N.Tensor(v.buf.data_ptr(), v.dtype, v.layout, v.n, v.c, v.h >> s, v.w >> s, v.cstride, v.coff)

    def materialize(self, v: View) -> View:
        if v.up == 0:
            return v
        y = self.alloc(v.n, v.c, v.h, v.w)
        self.wadd(v, y, None, accumulate=0)
        return y

    def workspace(self, nbytes: int) -> torch.Tensor:
        return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=self.device)

    # ---------------------------------------------------------------- ops
    def conv(self, desc: N.ConvDesc, x: View, y: View, w_ptr: int, b_ptr: int, res: View | None = None):
        desc.up = x.up
        N.call("fce_conv2d", C.byref(desc), C.byref(self.src_t(x)), w_ptr, b_ptr,
               C.byref(self.t(res)) if res is not None else None, C.byref(self.t(y)), self.stream)

    def maxpool_chain(self, buf: View, c: int, k: int):
        x, y1, y2, y3 = (buf.slice(i * c, c) for i in range(4))
        N.call("fce_maxpool_chain", *(C.byref(self.t(v)) for v in (x, y1, y2, y3)), k, self.stream)

    def wadd(self, x: View, y: View, fusion, accumulate: int):
        w, n, i = _fusion(fusion)
        if w is None:  # plain (upsampling) copy: alpha = 1 via a one-element weight
            w, n, i = _ONE.get(self.device), 1, 0
        N.call("fce_weighted_add", C.byref(self.src_t(x)), x.up, w, n, i, accumulate, C.byref(self.t(y)), self.stream)

    def coord(self, kind: int, desc: N.CoordDesc, x: View, y: View):
        x = self.materialize(x)
        nb = N.lib().fce_coord_workspace_bytes(C.byref(desc), x.n, x.h, x.w)
        ws = self.workspace(nb)
        fn = ("fce_bicoordcrossatt", "fce_coordatt", "fce_coordcrossatt")[kind]
        N.call(fn, C.byref(desc), C.byref(self.t(x)), C.byref(self.t(y)), ws.data_ptr(), nb, self.stream)
        self._keep = ws  # keep alive until the stream has consumed it (caching allocator is stream-ordered)

    def c3k2(self, desc: N.C3k2Desc, x: View, y: View):
        N.call("fce_c3k2", C.byref(desc), C.byref(self.t(x)), C.byref(self.t(y)), self.stream)

    def psa(self, qkv: View, heads: int, kd: int, hd: int, pe_w: int, pe_b: int, y: View):
        N.call("fce_psa_attention", C.byref(self.t(qkv)), heads, kd, hd, pe_w, pe_b, C.byref(self.t(y)), self.stream)

    def conv_detect(self, desc: N.ConvDesc, x: View, pred: torch.Tensor, anchors: int, offset: int, part: int,
                    stride: float, nc: int, reg_max: int, w_ptr: int, b_ptr: int):
        x = self.materialize(x)
        e = N.DetectEpi(pred.data_ptr(), anchors, offset, nc, reg_max, part, float(stride))
        N.call("fce_conv2d_detect", C.byref(desc), C.byref(self.t(x)), w_ptr, b_ptr, C.byref(e), self.stream)

    def detect(self, maps: list[View], strides: list[float], reg_max: int) -> torch.Tensor:
        nl = len(maps)
        A = sum(m.h * m.w for m in maps)
        nc = maps[0].c - 4 * reg_max
        out = torch.empty((maps[0].n, 4 + nc, A), dtype=torch.float32, device=self.device)
        box = (N.Tensor * nl)(*[self.t(m.slice(0, 4 * reg_max)) for m in maps])
        cls = (N.Tensor * nl)(*[self.t(m.slice(4 * reg_max, nc)) for m in maps])
        st = torch.tensor(strides, dtype=torch.float32)
        sts = (C.c_float * nl)(*st.tolist())
        N.call("fce_detect_decode", box, cls, nl, C.cast(sts, C.c_void_p), reg_max, out.data_ptr(), self.stream)
        return out


class ShapeBackend:
    """Shape propagation only: no device, no data, no arithmetic.

    This is the drop-ins' answer to a non-ROCm input, e.g. the CPU ``torch.zeros(1, ch, 256, 256)``
    stride probe that the reference runs while building a model (``tasks.py:396-411``). Outputs are
    ``meta`` tensors of the reference's output shape: anything that reads their values fails loudly, so
    this is never a numeric CPU fallback."""

    shape_only = True
    fused_detect = False
    device = torch.device("meta")

    def alloc(self, n, c, h, w, dtype=N.F16) -> View:
        return View(None, n, c, h, w, c, 0, dtype)

    def from_torch(self, x: torch.Tensor, keep_nchw: bool = False) -> View:
        n, c, h, w = x.shape
        return View(None, n, c, h, w, c, 0, N.F16, N.NCHW if keep_nchw else N.NHWC)

    def to_torch(self, v: View, dtype=torch.float16) -> torch.Tensor:
        return torch.empty((v.n, v.c, v.h, v.w), dtype=dtype, device="meta")

    def materialize(self, v: View) -> View:
        return self.alloc(v.n, v.c, v.h, v.w) if v.up else v

    def conv(self, *a, **k):
        pass

    maxpool_chain = wadd = coord = psa = conv_detect = conv


class _OneCache:
    def __init__(self):
        self.t = {}

    def get(self, device):
        if device not in self.t:
            self.t[device] = torch.ones(1, dtype=torch.float32, device=device)
        return self.t[device].data_ptr()


_ONE = _OneCache()


class NetBackend:
    """Records ops into a native fce_net for an input of logical size (H, W)."""

    fused_detect = True  # Detect tail fused into the last convs' epilogues (no fp32 maps)
    shape_only = False

    def __init__(self, H: int, W: int, device: torch.device):
        self.H, self.W = H, W
        self.device = device
        self.net = N.lib().fce_net_create()
        if not self.net:
            raise N.FceError("fce_net_create failed")
        self.keep = []  # device tensors whose pointers the net holds

    def close(self):
        if self.net:
            N.lib().fce_net_destroy(self.net)
            self.net = None

    def _shift(self, h, w):
        s = int(round(math.log2(self.H / h)))
        if (self.H >> s) != h or (self.W >> s) != w:
            raise ValueError(f"buffer size {h}x{w} is not input/{1 << s}")
        return s

    def alloc(self, n, c, h, w, dtype=N.F16) -> View:
        bid = N.lib().fce_net_add_buffer(self.net, c, self._shift(h, w), dtype)
        if bid < 0:
            N.check(bid, "fce_net_add_buffer")
        return View(bid, n, c, h, w, c, 0, dtype)

    def input_view(self, n, c) -> View:
        return View(-1, n, c, self.H, self.W, c, 0, N.F16, N.NCHW)

    def materialize(self, v: View) -> View:
        if v.up == 0:
            return v
        y = self.alloc(v.n, v.c, v.h, v.w)
        self.wadd(v, y, None, accumulate=0)
        return y

    supports_dup = True  # fce_net_add_conv_dup: a second, dense store of some output channels

    def conv(self, desc: N.ConvDesc, x: View, y: View, w_ptr: int, b_ptr: int, res: View | None = None,
             dup: tuple | None = None):
        """`dup` = (dense View, first output channel): those output channels are also stored there."""
        desc.up = x.up
        args = (self.net, C.byref(desc), x.buf, x.coff, y.buf, y.coff, res.buf if res is not None else -1,
                res.coff if res is not None else 0, w_ptr, b_ptr)
        if dup is None:
            N.call("fce_net_add_conv", *args)
        else:
            dv, lo = dup
            assert dv.coff == 0 and dv.c == dv.cstride
            N.call("fce_net_add_conv_dup", *args, dv.buf, lo, dv.c)

    def maxpool_chain(self, buf: View, c: int, k: int):
        N.call("fce_net_add_maxpool_chain", self.net, buf.buf, buf.coff, c, k)

    def wadd(self, x: View, y: View, fusion, accumulate: int):
        w, n, i = _fusion(fusion)
        if w is None:
            w, n, i = _ONE.get(self.device), 1, 0
        N.call("fce_net_add_weighted_add", self.net, x.buf, x.coff, x.c, x.up, w, n, i, accumulate, y.buf, y.coff)

    def coord(self, kind: int, desc: N.CoordDesc, x: View, y: View):
        x = self.materialize(x)
        N.call("fce_net_add_coord", self.net, kind, C.byref(desc), x.buf, x.coff, y.buf, y.coff)

    def c3k2(self, desc: N.C3k2Desc, x: View, y: View):
        N.call("fce_net_add_c3k2", self.net, C.byref(desc), x.buf, x.coff, y.buf, y.coff)

    def num_ops(self) -> int:
        return N.lib().fce_net_num_ops(self.net)

    def c3k2_alt(self, desc: N.C3k2Desc, x: View, y: View, first_op: int, nops: int):
        """The fused C3k2 as the alternative of ops [first_op, first_op + nops) (its four convs): the plan-time
        autotune keeps the faster form (fce_net_add_c3k2_alt)."""
        N.call("fce_net_add_c3k2_alt", self.net, C.byref(desc), x.buf, x.coff, y.buf, y.coff, first_op, nops)

    def bneck_alt(self, desc: N.BneckDesc, x: View, y: View, first_op: int, nops: int):
        """The fused Bottleneck chain as the alternative of ops [first_op, first_op + nops) (its 3x3 convs): the plan keeps
        the faster form, or the convs where no instantiation covers the map width (fce_net_add_bneck_alt)."""
        N.call("fce_net_add_bneck_alt", self.net, C.byref(desc), x.buf, x.coff, y.buf, y.coff, first_op, nops)

    def pw2_alt(self, desc: N.Pw2Desc, first_op: int):
        """The fused 1x1 pair as the alternative of ops first_op, first_op + 1 (fce_net_add_pw2_alt)."""
        N.call("fce_net_add_pw2_alt", self.net, C.byref(desc), first_op)

    def stem_alt(self, desc: N.Stem2Desc, first_op: int, nops: int):
        """The one-kernel stem pair as the alternative of ops [first_op, first_op + nops) (the stem and the second conv):
        the plan keeps the faster form, or the two convs when anything else reads the stem's output
        (fce_net_add_stem_alt)."""
        N.call("fce_net_add_stem_alt", self.net, C.byref(desc), first_op, nops)

    def detect_cls_alt(self, desc: N.DclsDesc, x: View, first_op: int, nops: int):
        """The one-kernel Detect cls branch as the alternative of ops [first_op, first_op + nops) (its two depthwise and
        two 1x1 convs and its cls tail): the plan-time autotune keeps the faster form (fce_net_add_detect_cls_alt)."""
        N.call("fce_net_add_detect_cls_alt", self.net, C.byref(desc), x.buf, x.coff, first_op, nops)

    def psa(self, qkv: View, heads: int, kd: int, hd: int, pe_w: int, pe_b: int, y: View):
        assert qkv.coff == 0 and qkv.c == qkv.cstride
        N.call("fce_net_add_psa_attention", self.net, qkv.buf, heads, kd, hd, pe_w, pe_b, y.buf, y.coff)

    def conv_detect(self, desc: N.ConvDesc, x: View, part: int, level: int, stride: float, nc: int, reg_max: int,
                    w_ptr: int, b_ptr: int):
        assert x.up == 0
        N.call("fce_net_add_conv_detect", self.net, C.byref(desc), x.buf, x.coff, part, level, float(stride), nc,
               reg_max, w_ptr, b_ptr)

    def detect(self, maps: list[View], strides: list[float], reg_max: int):
        nl = len(maps)
        ids = (C.c_int * nl)(*[m.buf for m in maps])
        sts = (C.c_float * nl)(*[float(s) for s in strides])
        N.call("fce_net_add_detect", self.net, nl, C.cast(ids, C.c_void_p), C.cast(sts, C.c_void_p), reg_max)
        return None
