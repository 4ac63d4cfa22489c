"""Oracle restatement of the reference model parser (layer table only).

Follows `ultralytics/nn/tasks.py:1489-1743` (`parse_model`), `:1746-1782`
(`yaml_model_load` / `guess_model_scale`) and `ultralytics/utils/ops.py:137-149`
(`make_divisible`).  Produces a plain layer table consumed by
`oracle.fce_oracle.forward`; no nn.Module is built.  TEST INFRASTRUCTURE ONLY.
"""

from __future__ import annotations

import ast
import math
import re
from pathlib import Path

import yaml

# tasks.py:1524-1561 / :1562-1580 (restricted to the module types the YOLO11 / -fce / -bifpn graphs use)
BASE = {"Conv", "DWConv", "Bottleneck", "SPPF", "C2f", "C3k2", "C3", "C2PSA"}
REPEAT = {"C2f", "C3k2", "C3", "C2PSA"}


def make_divisible(x, divisor: int) -> int:
    """ops.py:137-149: ceil(x / divisor) * divisor."""
    return math.ceil(x / divisor) * divisor


def guess_scale(path: str) -> str:
    """tasks.py:1769-1782."""
    m = re.search(r"yolo(e-)?[v]?\d+([nslmx])", Path(path).stem)
    return m.group(2) if m else ""


def load_yaml(path: str, cfg_dir: str | None = None) -> dict:
    """tasks.py:1746-1766: 'yolo11n-fce.yaml' -> reads 'yolo11-fce.yaml', scale 'n'."""
    p = Path(path)
    unified = re.sub(r"(\d+)([nslmx])(.+)?$", r"\1\3", p.stem) + p.suffix
    cand = [Path(cfg_dir) / unified, Path(cfg_dir) / p.name] if cfg_dir else [p.with_name(unified), p]
    for c in cand:
        if c.exists():
            d = yaml.safe_load(c.read_text())
            break
    else:
        raise FileNotFoundError(path)
    d["scale"] = guess_scale(str(p))
    d["yaml_file"] = str(p)
    return d


def parse(d: dict, ch: int = 3):
    """tasks.py:1489-1743 restated.  Returns (layers, save, legacy).

    Each layer: dict(i, f, n, type, args, c2).  `args` are the constructor
    arguments exactly as the reference passes them to the module class.
    """
    nc, scales = d.get("nc"), d.get("scales")
    depth, width = d.get("depth_multiple", 1.0), d.get("width_multiple", 1.0)
    max_ch = float("inf")
    scale = d.get("scale")
    if scales:
        if not scale:
            scale = next(iter(scales.keys()))  # tasks.py:1511-1513
        depth, width, max_ch = scales[scale]
    chs = [ch]
    layers, save = [], []
    legacy = True
    for i, (f, n, m, args) in enumerate(d["backbone"] + d["head"]):
        args = list(args)
        m = m[3:] if m.startswith("nn.") else m
        for j, a in enumerate(args):  # tasks.py:1589-1592
            if isinstance(a, str):
                if a == "nc":
                    args[j] = nc
                else:
                    try:
                        args[j] = ast.literal_eval(a)
                    except ValueError:
                        pass
        n = max(round(n * depth), 1) if n > 1 else n  # tasks.py:1593
        if m in BASE:
            c1, c2 = chs[f], args[0]
            if c2 != nc:
                c2 = make_divisible(min(c2, max_ch) * width, 8)
            args = [c1, c2, *args[1:]]
            if m in REPEAT:
                args.insert(2, n)
                n = 1
            if m == "C3k2":
                legacy = False
                if scale in "mlx":
                    args[3] = True
        elif m == "Concat":
            c2 = sum(chs[x] for x in f)
        elif m == "BiFPN_Concat":  # tasks.py:1630-1635 (Q1: width applied to max(c1) again)
            c1 = [chs[x] for x in f] if isinstance(f, list) else [chs[f]]
            c2 = args[0] if args else max(c1)
            c2 = make_divisible(min(c2, max_ch) * width, 8)
            args = [c1, c2]
        elif m in ("CoordAtt", "CoordCrossAtt", "BiCoordCrossAtt"):  # tasks.py:1636-1708
            inp = chs[f]
            oup = args[0] if args else inp
            if args:
                oup = make_divisible(min(oup, max_ch) * width, 8)
            reduction = args[1] if len(args) > 1 else max(8, min(32, int(inp**0.5)))
            c2 = oup
            if m == "CoordAtt":
                args = [inp, oup, reduction]
            else:
                if len(args) > 2:
                    heads = args[2]
                else:
                    base = max(8, inp // reduction)
                    heads = max(1, min(8, inp // 32))
                    while heads > 1 and base // heads < 8:
                        heads -= 1
                args = [inp, oup, reduction, heads]
        elif m == "Detect":
            args = list(args) + [[chs[x] for x in f]]
        else:  # Upsample and friends: c2 = ch[f]
            c2 = chs[f]
        layers.append(dict(i=i, f=f, n=n, type=m, args=args, c2=c2))
        save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
        if i == 0:
            chs = []
        chs.append(c2)
    for L in layers:
        if L["type"] == "Detect":
            L["legacy"] = legacy  # class attribute set at parse time (tasks.py:1716), Q5
    return layers, sorted(save), legacy
