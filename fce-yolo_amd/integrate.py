"""Hooks into the reference's own predict loop.

The reference predictor (ultralytics/engine/predictor.py:383-405 inference via
nn/autobackend.py:667-700 AutoBackend.forward) calls `self.model(im)` on a preprocessed (B, 3, H, W)
batch and hands the result to models/yolo/detect/predict.py postprocess (NMS + scale_boxes).  With
`patch_autobackend(predictor.model)` that call runs this package's whole-graph Engine on the MI355X
(one plan per input shape, direct launches), returning the same (B, 4+nc, A) prediction tensor, so
the reference's postprocess, Results and plotting stay untouched.  `device_postprocess(predictor)` in
addition swaps its NMS for the device NMS (bit-exact with TorchNMS).

Both take objects of the reference package but import nothing from it.
"""

from __future__ import annotations

import types

import torch

from .engine import Engine, non_max_suppression
from .parser import DetectionModel


def from_reference_model(ref_model, device=None) -> DetectionModel:
    """The reference DetectionModel (tasks.py:339) -> this package's DetectionModel of the same YAML and
    state_dict keys (fp32), on `device`."""
    yaml_d = {k: v for k, v in dict(ref_model.yaml).items() if k != "yaml_file"}
    model = DetectionModel(yaml_d)
    sd = {k: (v.float() if v.is_floating_point() else v) for k, v in ref_model.state_dict().items()}
    if not any(".bn." in k for k in sd) and not model.is_fused():
        model.fuse()  # AutoBackend fuses by default (autobackend.py:203-207): mirror the fused layout
    model.load_state_dict(sd)
    model.names = dict(getattr(ref_model, "names", model.names))
    model.eval()
    return model.to(device) if device is not None else model


def patch_autobackend(backend, device=None):
    """Replace `backend.forward` (an AutoBackend wrapping a PyTorch DetectionModel) by Engine replays."""
    dev = torch.device(device) if device is not None else torch.device(getattr(backend, "device", "cuda"))
    if dev.type != "cuda":
        raise RuntimeError("patch_autobackend: fce_yolo_amd runs on ROCm devices only; no CPU fallback")
    model = from_reference_model(backend.model, dev)
    engines: dict[tuple, Engine] = {}

    def forward(self, im, augment=False, visualize=False, embed=None, **kwargs):
        if augment or visualize or embed:
            raise NotImplementedError("fce_yolo_amd: augment / visualize / embed are not on the inference path")
        key = (im.shape[0], im.shape[2], im.shape[3])
        if key not in engines:
            engines[key] = Engine(model, im.shape[0], (im.shape[2], im.shape[3]), dev)
        return engines[key](im.contiguous())

    backend.forward = types.MethodType(forward, backend)
    backend._fce_engines = engines
    return engines


def device_postprocess(predictor):
    """Route the predictor's NMS (predict.py:33-78 -> utils/nms.py:13) through the device NMS kernel."""
    import sys

    nms_mod = sys.modules.get("ultralytics.utils.nms")
    if nms_mod is None:
        raise RuntimeError("device_postprocess: the reference package is not imported")
    orig = nms_mod.non_max_suppression

    def nms(prediction, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False, multi_label=False,
            labels=(), max_det=300, nc=0, max_time_img=0.05, max_nms=30000, max_wh=7680, rotated=False,
            end2end=False, return_idxs=False):
        """The signature of utils/nms.py:13-29; argument combinations off the device path go to `orig`."""
        pred = prediction[0] if isinstance(prediction, (list, tuple)) else prediction
        if len(labels) or nc or rotated or end2end or pred.device.type != "cuda":
            return orig(prediction, conf_thres=conf_thres, iou_thres=iou_thres, classes=classes, agnostic=agnostic,
                        multi_label=multi_label, labels=labels, max_det=max_det, nc=nc, max_time_img=max_time_img,
                        max_nms=max_nms, max_wh=max_wh, rotated=rotated, end2end=end2end, return_idxs=return_idxs)
        return non_max_suppression(pred, conf_thres, iou_thres, max_det, max_nms, max_wh, return_idxs,
                                   classes=classes, agnostic=agnostic, multi_label=multi_label)

    nms_mod.non_max_suppression = nms
    return orig
