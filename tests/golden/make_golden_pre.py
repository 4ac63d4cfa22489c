"""Golden vectors for the pre/post-processing rows, from the REFERENCE itself.

    python tests/golden/make_golden_pre.py      # here only; writes tests/golden/prepost.npz

1. LetterBox geometry (data/augment.py:1555-1610, the predictor's pre_transform settings
   predictor.py:184-201: auto=False, center=True, stride 32): the reference's own LetterBox.__call__ is
   run on zero images of many source shapes.  cv2 is absent here, so the cv2 stub's ``resize`` and
   ``copyMakeBorder`` RECORD their arguments (dsize = new_unpad; top/bottom/left/right/value) and return
   arrays of the requested shape — the pixel arithmetic of cv2.resize is not exercised (its restatement
   in csrc/preprocess.hip + oracle/preprocess_oracle.py is "parity unpinned"), the integer placement is.
2. scale_boxes + clip_boxes (utils/ops.py:102-176), CPU fp32: random xyxy boxes mapped from a letterboxed
   canvas back to source shapes — exact expected outputs.
"""

from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
from make_golden import import_reference  # noqa: E402

SHAPES = [(480, 640), (640, 480), (720, 1280), (1080, 1920), (375, 500), (333, 517), (640, 640), (100, 100),
          (1, 1), (17, 999), (999, 17), (427, 640), (612, 612), (5, 6), (2048, 1536), (321, 321)]
IMGSZ = [(640, 640), (320, 320), (1280, 1280), (384, 640), (640, 384)]


def main():
    import_reference()
    import cv2  # the stub installed by import_reference

    from ultralytics.data.augment import LetterBox
    from ultralytics.utils import ops

    rec = {}

    def resize(img, dsize, interpolation=None):
        rec["resize"] = tuple(int(v) for v in dsize)
        return np.zeros((dsize[1], dsize[0]) + img.shape[2:], img.dtype)

    def copy_make_border(img, top, bottom, left, right, border, value=None):
        rec["border"] = (int(top), int(bottom), int(left), int(right), int(value[0]))
        h, w = img.shape[:2]
        return np.zeros((h + top + bottom, w + left + right) + img.shape[2:], img.dtype)

    cv2.resize = resize
    cv2.copyMakeBorder = copy_make_border
    cv2.BORDER_CONSTANT = 0
    geo = []
    for H, W in IMGSZ:
        lb = LetterBox((H, W), auto=False, stride=32)
        for h0, w0 in SHAPES:
            rec.clear()
            out = lb(image=np.zeros((h0, w0, 3), np.uint8))
            new_w, new_h = rec.get("resize", (w0, h0))
            top, bottom, left, right, value = rec["border"]
            assert out.shape == (H, W, 3), (out.shape, H, W, h0, w0)
            geo.append([H, W, h0, w0, new_h, new_w, top, bottom, left, right, value])
    out = {"geometry": np.array(geo, np.int64)}

    g = torch.Generator().manual_seed(7)
    cases = []
    for i, ((H, W), (h0, w0)) in enumerate([(s, t) for s in IMGSZ[:3] for t in SHAPES[:10]]):
        n = 64
        xy = torch.rand(n, 2, generator=g) * torch.tensor([W, H]) * 1.2 - 20
        wh = torch.rand(n, 2, generator=g) * 200
        boxes = torch.cat([xy, xy + wh], 1).float()
        res = ops.scale_boxes((H, W), boxes.clone(), (h0, w0, 3))
        out[f"sb{i}/boxes"] = boxes.numpy()
        out[f"sb{i}/out"] = res.numpy()
        cases.append([H, W, h0, w0])
    out["sb_cases"] = np.array(cases, np.int64)
    np.savez_compressed(HERE / "prepost.npz", **out)
    print(f"wrote {HERE / 'prepost.npz'}: {len(geo)} geometries, {len(cases)} scale_boxes cases")


if __name__ == "__main__":
    main()
