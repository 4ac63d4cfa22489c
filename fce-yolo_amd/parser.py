"""The reference model parser restated for the drop-in modules, and the detection model.

``parse_model`` follows ``ultralytics/nn/tasks.py:1489-1743`` (channel arithmetic, depth gain,
the FCE branches :1630-1708 including the BiFPN double width scaling (Q1), the C3k2 ``c3k``
override for m/l/x (Q6), ``Detect.legacy`` set at parse time (Q5) and the adaptive FCE
defaults (Q7)); ``load_cfg`` follows ``yaml_model_load`` / ``guess_model_scale`` (:1746-1782, Q8).
``DetectionModel`` restates ``DetectionModel.__init__`` (:367-420, strides from a shape pass) and
``BaseModel._predict_once`` (:160-188).
"""

from __future__ import annotations

import ast
import contextlib
import math
import re
from copy import deepcopy
from pathlib import Path

import torch
import torch.nn as nn

from . import _native as N
from . import cfg as _cfg
from . import modules as M
from .backend import EagerBackend, View

MODULES = {name: getattr(M, name) for name in M.__all__}
BASE = {M.Conv, M.DWConv, M.Bottleneck, M.SPPF, M.C2f, M.C3k2, M.C3, M.C2PSA}
REPEAT = {M.C2f, M.C3k2, M.C3, M.C2PSA}


def make_divisible(x, divisor):
    """ops.py:137-149."""
    if isinstance(divisor, torch.Tensor):
        divisor = int(divisor.max())
    return math.ceil(x / divisor) * divisor


def guess_model_scale(path) -> str:
    """tasks.py:1769-1782."""
    m = re.search(r"yolo(e-)?[v]?\d+([nslmx])", Path(str(path)).stem)
    return m.group(2) if m else ""


def load_cfg(path) -> dict:
    """tasks.py:1746-1766.  'yolo11n-fce.yaml' -> the yolo11-fce graph at scale 'n'.  A real YAML file
    path is read as-is (e.g. the reference's own cfg files); otherwise the built-in graph of the
    unified name is used."""
    p = Path(str(path))
    unified = re.sub(r"(\d+)([nslmx])(.+)?$", r"\1\3", p.stem) + p.suffix
    for cand in (p.with_name(unified), p):
        if cand.is_file():
            import yaml

            d = yaml.safe_load(cand.read_text())
            break
    else:
        if unified not in _cfg.BUILTIN:
            raise FileNotFoundError(f"{path}: no such file and no built-in graph '{unified}'")
        d = _cfg.BUILTIN[unified]()
    d["scale"] = guess_model_scale(p)
    d["yaml_file"] = str(p)
    return d


def _resolve(name: str):
    if name.startswith("nn."):
        name = name[3:]
        if name == "Upsample":
            return M.Upsample
        return getattr(torch.nn, name)
    if name not in MODULES:
        raise KeyError(f"module '{name}' is not part of the FCE-YOLOv11 inference path")
    return MODULES[name]


def parse_model(d: dict, ch: int = 3, verbose: bool = False):
    """tasks.py:1489-1743 restated; returns (nn.Sequential, save list)."""
    legacy = True
    max_channels = float("inf")
    nc, scales = d.get("nc"), d.get("scales")
    depth, width = d.get("depth_multiple", 1.0), d.get("width_multiple", 1.0)
    scale = d.get("scale")
    if scales:
        if not scale:
            scale = next(iter(scales.keys()))
        depth, width, max_channels = scales[scale]
    if d.get("activation"):
        raise NotImplementedError("custom activations are not on the FCE-YOLOv11 path")
    chs = [ch]
    layers, save = [], []
    for i, (f, n, m, args) in enumerate(d["backbone"] + d["head"]):
        m = _resolve(m)
        args = list(args)
        for j, a in enumerate(args):
            if isinstance(a, str):
                with contextlib.suppress(ValueError):
                    args[j] = nc if a == "nc" else ast.literal_eval(a)
        n = n_ = max(round(n * depth), 1) if n > 1 else n
        if m in BASE:
            c1, c2 = chs[f], args[0]
            if c2 != nc:
                c2 = make_divisible(min(c2, max_channels) * width, 8)
            args = [c1, c2, *args[1:]]
            if m in REPEAT:
                args.insert(2, n)
                n = 1
            if m is M.C3k2:
                legacy = False
                if scale in "mlx":
                    args[3] = True
        elif m is M.Concat:
            c2 = sum(chs[x] for x in f)
        elif m is M.BiFPN_Concat:
            c1 = [chs[x] for x in f] if isinstance(f, list) else [chs[f]]
            c2 = args[0] if args else max(c1)
            c2 = make_divisible(min(c2, max_channels) * width, 8)
            args = [c1, c2]
        elif m in (M.CoordAtt, M.CoordCrossAtt, M.BiCoordCrossAtt):
            inp = chs[f]
            oup = args[0] if args else inp
            if args:
                oup = make_divisible(min(oup, max_channels) * width, 8)
            reduction = args[1] if len(args) > 1 else max(8, min(32, int(inp**0.5)))
            c2 = oup
            if m is M.CoordAtt:
                args = [inp, oup, reduction]
            else:
                if len(args) > 2:
                    heads = args[2]
                else:
                    base_dim = max(8, inp // reduction)
                    heads = max(1, min(8, inp // 32))
                    while heads > 1 and base_dim // heads < 8:
                        heads -= 1
                args = [inp, oup, reduction, heads]
        elif m is M.Detect:
            args.append([chs[x] for x in f])
            M.Detect.legacy = legacy
        else:
            c2 = chs[f]
        m_ = nn.Sequential(*(m(*args) for _ in range(n))) if n > 1 else m(*args)
        m_.np = sum(x.numel() for x in m_.parameters())
        m_.i, m_.f, m_.type = i, f, m.__name__
        m_.args = args
        if verbose:
            print(f"{i:>3}{f!s:>20}{n_:>3}{m_.np:10.0f}  {m.__name__:<45}{args!s:<30}")
        save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
        layers.append(m_)
        if i == 0:
            chs = []
        chs.append(c2)
    return nn.Sequential(*layers), sorted(save)


def _shape_strides(model: nn.Sequential, save, s: int = 256):
    """Stride probe (tasks.py:396-411) as a spatial-size pass: stride_i = s / height of Detect input i."""
    y = []
    hw = (s, s)
    for m in model:
        if m.f != -1:
            hw = y[m.f] if isinstance(m.f, int) else [hw if j == -1 else y[j] for j in m.f]
        if isinstance(m, M.Detect):
            return torch.tensor([s / v[0] for v in hw])
        if isinstance(m, M.Conv):
            st = m.conv.stride[0]
            k = m.conv.kernel_size[0]
            hw = tuple((v + 2 * (k // 2) - k) // st + 1 for v in hw)
        elif isinstance(m, nn.Upsample):
            hw = tuple(int(v * m.scale_factor) for v in hw)
        elif isinstance(hw, list):
            hw = hw[0]
        y.append(hw if m.i in save else None)
    raise RuntimeError("model has no Detect head")


class DetectionModel(nn.Module):
    """tasks.py:339-420 for inference: parse, strides, forward = _predict_once on the HIP kernels."""

    def __init__(self, cfg="yolo11n-fce.yaml", ch=3, nc=None, verbose=False):
        super().__init__()
        self.yaml = cfg if isinstance(cfg, dict) else load_cfg(cfg)
        self.yaml["channels"] = ch
        if nc and nc != self.yaml["nc"]:
            self.yaml["nc"] = nc
        self.model, self.save = parse_model(deepcopy(self.yaml), ch=ch, verbose=verbose)
        self.names = {i: f"{i}" for i in range(self.yaml["nc"])}
        det = self.model[-1]
        det.stride = _shape_strides(self.model, self.save)
        self.stride = det.stride
        for m in self.modules():  # initialize_weights (torch_utils.py:463-473): BN eps 1e-3
            if isinstance(m, nn.BatchNorm2d):
                m.eps = 1e-3

    def emit(self, be, x):
        """_predict_once over a backend; returns (pred, maps)."""
        y = []
        first = be.num_ops() if hasattr(be, "stem_alt") else None
        for m in self.model:
            if m.f != -1:
                x = y[m.f] if isinstance(m.f, int) else [x if j == -1 else y[j] for j in m.f]
            x = m.emit(be, x)
            y.append(x if m.i in self.save else None)
            if m.i == 1 and first is not None:  # the stem pair's one-kernel alternative (modules.stem_alt)
                M.stem_alt(be, self.model[0], self.model[1], first, 0 in self.save)
        return x

    def forward(self, x):
        """Eager (per-op launch) forward on a ROCm device: (B,3,H,W) -> ((B, 4+nc, A), maps)."""
        if x.device.type != "cuda":
            raise RuntimeError("DetectionModel: fce_yolo_amd runs on ROCm devices only; no CPU fallback")
        be = EagerBackend(x.device)
        pred, maps = self.emit(be, be.from_torch(x, keep_nchw=True))
        return pred, [be.to_torch(m, torch.float32) for m in maps]

    def is_fused(self) -> bool:
        return not any(isinstance(m, nn.BatchNorm2d) for m in self.modules())

    def fuse(self, verbose=False):
        """tasks.py:223-252: fold every Conv / DWConv BN into its conv (eps 1e-3) and drop the BN.  The
        kernels fold BN when they pack weights, so a fused and an unfused model compute the same; this
        gives the fused state_dict layout (``*.conv.bias``, no ``*.bn.*``) that AutoBackend's models have."""
        for m in self.model.modules():
            if isinstance(m, M.Conv) and hasattr(m, "bn"):
                M.fuse_conv_bn(m)
        return self
