"""CPU restatement of the reference's pre/post-processing around the detector (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the product
path (fce-yolo_amd) never does.

- letterbox_geometry:  data/augment.py:1555-1610 LetterBox.__call__ (auto=False, scale_fill=False,
  scaleup=True, center=True) — pinned by tests/golden/prepost.npz (the reference's own LetterBox run
  by tests/golden/make_golden_pre.py).
- resize_linear_u8:  cv2.resize(..., INTER_LINEAR) for uint8 HWC images (OpenCV imgproc resize.cpp
  fixed-point path, 11-bit coefficients, 16-lane SIMD vertical body + scalar tail).  opencv-python
  (the reference's dependency, unpinned in pyproject.toml) is NOT importable here: **parity unpinned**
  except for its identity case (no resize), which the geometry fixtures cover.
- preprocess:  engine/predictor.py:151-173 (stack, BGR->RGB, HWC->CHW, .half(), / 255).
- scale_boxes:  utils/ops.py:102-150 + clip_boxes :153-176 on CPU fp32 — pinned by prepost.npz.
"""

from __future__ import annotations

import numpy as np


def letterbox_geometry(h0: int, w0: int, H: int, W: int):
    """(new_h, new_w, top, bottom, left, right) — augment.py:1575-1605 (Python round = half-to-even)."""
    r = min(H / h0, W / w0)
    new_w, new_h = round(w0 * r), round(h0 * r)
    dw, dh = W - new_w, H - new_h
    dw /= 2
    dh /= 2
    top, bottom = round(dh - 0.1), round(dh + 0.1)
    left, right = round(dw - 0.1), round(dw + 0.1)
    return new_h, new_w, top, bottom, left, right


def _axis(n_dst: int, n_src: int):
    """Source indices and 11-bit coefficients per destination index (resize.cpp, INTER_LINEAR)."""
    scale = n_src / n_dst  # double
    d = np.arange(n_dst, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    s[lo], f[lo] = 0, 0.0
    hi = s >= n_src - 1
    s[hi], f[hi] = n_src - 1, 0.0
    c0 = np.rint((np.float32(1.0) - f) * np.float32(2048.0)).astype(np.int64)
    c1 = np.rint(f * np.float32(2048.0)).astype(np.int64)
    return s, np.minimum(s + 1, n_src - 1), c0, c1


def resize_linear_u8(img: np.ndarray, new_w: int, new_h: int) -> np.ndarray:
    """cv2.resize(img, (new_w, new_h), interpolation=INTER_LINEAR) for uint8 HWC (restated; see module doc)."""
    h0, w0, c = img.shape
    if (w0, h0) == (new_w, new_h):
        return img.copy()
    xs0, xs1, a0, a1 = _axis(new_w, w0)
    ys0, ys1, b0, b1 = _axis(new_h, h0)
    S = img.astype(np.int64)
    hr = S[:, xs0, :] * a0[None, :, None] + S[:, xs1, :] * a1[None, :, None]  # (h0, new_w, c) horizontal pass
    h0r, h1r = hr[ys0], hr[ys1]  # (new_h, new_w, c)
    B0, B1 = b0[:, None, None], b1[:, None, None]
    simd = (((B0 * (h0r >> 4)) >> 16) + ((B1 * (h1r >> 4)) >> 16) + 2) >> 2
    scalar = (B0 * h0r + B1 * h1r + (1 << 21)) >> 22
    e = (np.arange(new_w)[:, None] * c + np.arange(c)[None, :])[None]  # element index within the row
    out = np.where(e < (new_w * c // 16) * 16, simd, scalar)
    return np.clip(out, 0, 255).astype(np.uint8)


def letterbox(img: np.ndarray, H: int, W: int, pad: int = 114) -> np.ndarray:
    """LetterBox(new_shape=(H, W))(image=img): uint8 HWC canvas (augment.py:1592-1605)."""
    h0, w0 = img.shape[:2]
    new_h, new_w, top, bottom, left, right = letterbox_geometry(h0, w0, H, W)
    im = resize_linear_u8(img, new_w, new_h)
    out = np.full((H, W, img.shape[2]), pad, np.uint8)
    out[top:top + new_h, left:left + new_w] = im
    return out


def preprocess(imgs, H: int, W: int):
    """predictor.py:151-173: (u8 NCHW RGB batch, fp16 NCHW batch = u8.half() / 255)."""
    x = np.stack([letterbox(im, H, W) for im in imgs])[..., ::-1].transpose(0, 3, 1, 2)
    x = np.ascontiguousarray(x)
    import torch

    return x, (torch.from_numpy(x).half() / 255)


def scale_boxes(img1_shape, boxes: np.ndarray, img0_shape) -> np.ndarray:
    """ops.py:102-150 (ratio_pad=None, padding=True, xyxy) + clip_boxes, fp32 like the CPU reference."""
    gain = min(img1_shape[0] / img0_shape[0], img1_shape[1] / img0_shape[1])
    pad_x = round((img1_shape[1] - img0_shape[1] * gain) / 2 - 0.1)
    pad_y = round((img1_shape[0] - img0_shape[0] * gain) / 2 - 0.1)
    b = np.array(boxes, np.float32, copy=True)
    b[..., [0, 2]] -= np.float32(pad_x)
    b[..., [1, 3]] -= np.float32(pad_y)
    b[..., :4] = (b[..., :4] / np.float32(gain)).astype(np.float32)
    h, w = img0_shape[:2]
    b[..., [0, 2]] = b[..., [0, 2]].clip(0, w)
    b[..., [1, 3]] = b[..., [1, 3]].clip(0, h)
    return b
