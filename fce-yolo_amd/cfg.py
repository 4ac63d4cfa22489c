"""Built-in architecture definitions (the YOLO11 / FCE / BiFPN graphs) as plain data.

Same schema as the reference's model YAMLs (``ultralytics/cfg/models/11/yolo11{,-fce,-bifpn}.yaml``):
``nc``, ``scales`` {scale: [depth, width, max_channels]}, ``backbone`` / ``head`` rows
``[from, repeats, module, args]``.  ``parser.load_cfg`` also accepts the reference YAML files
themselves (they parse unchanged); these built-ins let the GPU box, where the reference does not
exist, build the same graphs.
"""

from __future__ import annotations

import copy

SCALES = {
    "n": [0.50, 0.25, 1024],
    "s": [0.50, 0.50, 1024],
    "m": [0.50, 1.00, 512],
    "l": [1.00, 1.00, 512],
    "x": [1.00, 1.50, 512],
}

_STEM = [
    [-1, 1, "Conv", [64, 3, 2]],
    [-1, 1, "Conv", [128, 3, 2]],
    [-1, 2, "C3k2", [256, False, 0.25]],
    [-1, 1, "Conv", [256, 3, 2]],
    [-1, 2, "C3k2", [512, False, 0.25]],
]


def _yolo11(fuse: str, coord: bool) -> dict:
    """fuse: 'Concat' (yolo11) or 'BiFPN_Concat'; coord: insert BiCoordCrossAtt after P3 / P4 (yolo11-fce)."""
    bb = copy.deepcopy(_STEM)
    if coord:
        bb += [[-1, 1, "BiCoordCrossAtt", [512, 8, 4]]]  # 5
    p3 = len(bb) - 1
    bb += [[-1, 1, "Conv", [512, 3, 2]], [-1, 2, "C3k2", [512, True]]]
    if coord:
        bb += [[-1, 1, "BiCoordCrossAtt", [512, 8, 4]]]  # 8
    p4 = len(bb) - 1
    bb += [[-1, 1, "Conv", [1024, 3, 2]], [-1, 2, "C3k2", [1024, True]], [-1, 1, "SPPF", [1024, 5]],
           [-1, 2, "C2PSA", [1024]]]
    p5 = len(bb) - 1
    fa = [1] if fuse == "Concat" else []
    i = len(bb)
    head = [
        [-1, 1, "nn.Upsample", [None, 2, "nearest"]],
        [[-1, p4], 1, fuse, list(fa)],
        [-1, 2, "C3k2", [512, False]],  # i+2
        [-1, 1, "nn.Upsample", [None, 2, "nearest"]],
        [[-1, p3], 1, fuse, list(fa)],
        [-1, 2, "C3k2", [256, False]],  # i+5  (P3/8)
        [-1, 1, "Conv", [256, 3, 2]],
        [[-1, p4, i + 2] if fuse == "BiFPN_Concat" else [-1, i + 2], 1, fuse, list(fa)],
        [-1, 2, "C3k2", [512, False]],  # i+8  (P4/16)
        [-1, 1, "Conv", [512, 3, 2]],
        [[-1, p5], 1, fuse, list(fa)],
        [-1, 2, "C3k2", [1024, True]],  # i+11 (P5/32)
        [[i + 5, i + 8, i + 11], 1, "Detect", ["nc"]],
    ]
    return {"nc": 80, "scales": copy.deepcopy(SCALES), "backbone": bb, "head": head}


BUILTIN = {
    "yolo11.yaml": lambda: _yolo11("Concat", False),
    "yolo11-fce.yaml": lambda: _yolo11("BiFPN_Concat", True),
    "yolo11-bifpn.yaml": lambda: _yolo11("BiFPN_Concat", False),
}
