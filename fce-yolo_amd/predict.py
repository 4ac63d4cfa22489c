"""Batched detection predictor on the device: decoded uint8 images in, boxes in source-image pixels out.

The MI355X form of the reference's predict loop for detection (ultralytics/engine/predictor.py:151-201
preprocess / pre_transform, models/yolo/detect/predict.py:33-121 postprocess + construct_result):

    uint8 HWC BGR images --(fce_letterbox: resize + pad 114 + BGR->RGB, on the GPU)--> u8 NCHW batch
      --(Engine: forward; the stem divides by 255 with the fp16 rounding of `im.half() / 255`)--> pred
      --(NMS: conf / iou / max_det, bit-exact TorchNMS)--> (k, 6) per image
      --(fce_scale_boxes: ops.scale_boxes + clip_boxes)--> boxes in each source image's pixel frame

Letterbox placement is computed on the host exactly as LetterBox.__call__ does (augment.py:1575-1605,
Python round); images of any size share one (H, W) canvas (auto=False, the predictor's setting for
batched inputs of mixed shapes).
"""

from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _native as N
from .engine import NMS, Engine


class LetterboxImg(C.Structure):  # fce_letterbox_img
    _fields_ = [("src", C.c_void_p), ("h0", C.c_int), ("w0", C.c_int), ("row_stride", C.c_int),
                ("new_h", C.c_int), ("new_w", C.c_int), ("top", C.c_int), ("left", C.c_int)]


class BoxScale(C.Structure):  # fce_box_scale
    _fields_ = [("gain", C.c_float), ("pad_x", C.c_int), ("pad_y", C.c_int), ("h0", C.c_int), ("w0", C.c_int)]


def letterbox_geometry(h0: int, w0: int, H: int, W: int):
    """augment.py:1575-1605 (auto=False, scaleup=True, center=True): (new_h, new_w, top, left)."""
    r = min(H / h0, W / w0)
    new_w, new_h = round(w0 * r), round(h0 * r)
    dw, dh = (W - new_w) / 2, (H - new_h) / 2
    return new_h, new_w, round(dh - 0.1), round(dw - 0.1)


def box_scale(H: int, W: int, h0: int, w0: int):
    """ops.py:122-130 (ratio_pad=None): (gain, pad_x, pad_y) mapping canvas (H, W) back to (h0, w0)."""
    gain = min(H / h0, W / w0)
    return gain, round((W - w0 * gain) / 2 - 0.1), round((H - h0 * gain) / 2 - 0.1)


class Letterbox:
    """Device letterbox of up to `batch` uint8 HWC BGR images into a (batch, 3, H, W) uint8 canvas."""

    def __init__(self, batch: int, imgsz, device, pad_value: int = 114):
        self.H, self.W = (imgsz, imgsz) if isinstance(imgsz, int) else imgsz
        self.batch, self.device, self.pad = batch, torch.device(device), pad_value
        self.out = torch.empty((batch, 3, self.H, self.W), dtype=torch.uint8, device=self.device)
        self.desc = torch.empty(batch * C.sizeof(LetterboxImg), dtype=torch.uint8, device=self.device)

    def __call__(self, imgs: list[torch.Tensor]) -> torch.Tensor:
        """imgs: uint8 (h, w, 3) BGR tensors on the device (row-contiguous).  Returns the canvas view."""
        if not 0 < len(imgs) <= self.batch:
            raise ValueError(f"Letterbox: 1..{self.batch} images per call")
        host = (LetterboxImg * len(imgs))()
        for i, im in enumerate(imgs):
            if im.device != self.device or im.dtype != torch.uint8 or im.dim() != 3 or im.shape[2] != 3:
                raise ValueError("Letterbox: images must be uint8 (h, w, 3) tensors on the canvas device")
            if im.stride(2) != 1 or im.stride(1) != 3:
                raise ValueError("Letterbox: image rows must be contiguous HWC")
            h0, w0 = int(im.shape[0]), int(im.shape[1])
            new_h, new_w, top, left = letterbox_geometry(h0, w0, self.H, self.W)
            host[i] = LetterboxImg(im.data_ptr(), h0, w0, int(im.stride(0)), new_h, new_w, top, left)
        nb = C.sizeof(host)
        staged = torch.frombuffer(bytearray(bytes(host)), dtype=torch.uint8)
        self.desc[:nb].copy_(staged, non_blocking=False)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        N.call("fce_letterbox", C.c_void_p(self.desc.data_ptr()), len(imgs), C.c_void_p(self.out.data_ptr()), self.H,
               self.W, self.pad, stream)
        return self.out[: len(imgs)]


class Predictor:
    """predict(images) -> per image (k, 6) [x1, y1, x2, y2, conf, cls] in source pixels (+ anchor indices).

    Fixed batch capacity; a call with fewer images pads the batch with the last canvas (their results are
    dropped).  All stages run on the device stream of the caller; one host sync at the end (counts)."""

    def __init__(self, model, batch: int, imgsz=640, device=None, conf=0.25, iou=0.7, max_det=300):
        self.engine = Engine(model, batch, imgsz, device)
        self.device = self.engine.device
        self.batch = batch
        self.lb = Letterbox(batch, (self.engine.H, self.engine.W), self.device)
        self.nms = NMS(batch, self.engine.anchors, self.engine.nc, self.device, conf, iou, max_det)
        self.scales = torch.empty(batch * C.sizeof(BoxScale), dtype=torch.uint8, device=self.device)

    def __call__(self, images, return_idxs: bool = False):
        if len(images) == 0:
            return ([], []) if return_idxs else []
        if len(images) > self.batch:
            raise ValueError(f"Predictor: at most {self.batch} images per call")
        imgs = [torch.as_tensor(np.ascontiguousarray(im)) if isinstance(im, np.ndarray) else im for im in images]
        imgs = [im.to(self.device, non_blocking=True) for im in imgs]
        canvas = self.lb(imgs)
        n = len(imgs)
        if n < self.batch:  # fixed-shape engine: pad the batch by repeating the last canvas
            full = self.lb.out
            full[n:].copy_(full[n - 1:n].expand(self.batch - n, -1, -1, -1))
            canvas = full
        pred = self.engine(canvas)
        dets, keep, counts = self.nms(pred)
        H, W = self.engine.H, self.engine.W
        host = (BoxScale * self.batch)()
        for i in range(self.batch):
            im = imgs[min(i, n - 1)]
            h0, w0 = int(im.shape[0]), int(im.shape[1])
            gain, px, py = box_scale(H, W, h0, w0)
            host[i] = BoxScale(gain, px, py, h0, w0)
        self.scales[: C.sizeof(host)].copy_(torch.frombuffer(bytearray(bytes(host)), dtype=torch.uint8))
        stream = torch.cuda.current_stream(self.device).cuda_stream
        N.call("fce_scale_boxes", C.c_void_p(dets.data_ptr()), C.c_void_p(counts.data_ptr()), self.batch,
               self.nms.max_det, C.c_void_p(self.scales.data_ptr()), stream)
        d, k = self.nms.results()
        d, k = d[:n], k[:n]
        return (d, k) if return_idxs else d

    def close(self):
        self.engine.close()
