"""numpy restatement of the reference NMS.  TEST INFRASTRUCTURE ONLY.

Follows ``ultralytics/utils/nms.py:13-166`` (``non_max_suppression``, including the
``classes`` / ``agnostic`` / ``multi_label`` arguments; no a-priori labels),
``ultralytics/utils/ops.py:224-240`` (``xywh2xyxy``) and ``nms.py:239-296``
(``TorchNMS.nms``, the backend taken when torchvision is not imported, Q10).
All arithmetic is float32 in the reference's operation order so kept indices are
bit-exact.  Ties in the descending score sort are broken by ascending candidate
position (``np.argsort(kind="stable")`` on the negated scores); the reference's
``torch.argsort(descending=True)`` leaves tie order unspecified.
"""

from __future__ import annotations

import numpy as np


def xywh2xyxy(b: np.ndarray) -> np.ndarray:
    """ops.py:224-240 in float32: xy -/+ wh/2."""
    b = b.astype(np.float32)
    y = np.empty_like(b)
    wh = b[:, 2:] / np.float32(2)
    y[:, :2] = b[:, :2] - wh
    y[:, 2:] = b[:, :2] + wh
    return y


def greedy_nms(boxes: np.ndarray, scores: np.ndarray, iou_thres: float) -> np.ndarray:
    """TorchNMS.nms (nms.py:239-296): keep box i, drop rest with IoU > thr."""
    if boxes.shape[0] == 0:
        return np.zeros((0,), np.int64)
    x1, y1, x2, y2 = (boxes[:, k].astype(np.float32) for k in range(4))
    areas = (x2 - x1) * (y2 - y1)
    order = np.argsort(-scores.astype(np.float32), kind="stable")
    keep = []
    thr = np.float32(iou_thres)
    while order.size > 0:
        i = order[0]
        keep.append(i)
        if order.size == 1:
            break
        rest = order[1:]
        xx1 = np.maximum(x1[i], x1[rest])
        yy1 = np.maximum(y1[i], y1[rest])
        xx2 = np.minimum(x2[i], x2[rest])
        yy2 = np.minimum(y2[i], y2[rest])
        w = np.maximum(xx2 - xx1, np.float32(0))
        h = np.maximum(yy2 - yy1, np.float32(0))
        inter = w * h
        if not np.any(inter):  # early exit of nms.py:285-288: no overlap, keep all remaining
            order = rest
            continue
        with np.errstate(divide="ignore", invalid="ignore"):
            iou = inter / ((areas[i] + areas[rest]) - inter)
        order = rest[iou <= thr]  # NaN IoU (zero-area pair) is dropped, as in torch
    return np.asarray(keep, np.int64)


def non_max_suppression(pred: np.ndarray, conf_thres=0.25, iou_thres=0.7, max_det=300, max_nms=30000, max_wh=7680,
                        classes=None, agnostic=False, multi_label=False):
    """nms.py:13-166 for a (B, 4+nc, A) prediction.  Returns (dets list of (k,6), keep-index list).

    classes / agnostic / multi_label follow nms.py:116-141: multi_label (when nc > 1) makes one candidate per
    (anchor, class) with score > conf_thres in torch.where's (anchor, class) order; classes keeps candidates
    whose class is listed; agnostic drops the per-class box offset."""
    pred = np.asarray(pred, np.float32)
    bs, no, A = pred.shape
    nc = no - 4
    multi_label = bool(multi_label) and nc > 1  # nms.py:96
    dets, keeps = [], []
    for b in range(bs):
        x = pred[b].T  # (A, 84)
        cls = x[:, 4:]
        xc = cls.max(1) > np.float32(conf_thres)
        idx = np.nonzero(xc)[0]
        x = x[idx]
        if x.shape[0] == 0:
            dets.append(np.zeros((0, 6), np.float32))
            keeps.append(np.zeros((0,), np.int64))
            continue
        box = xywh2xyxy(x[:, :4])
        if multi_label:
            i, j = np.nonzero(x[:, 4:] > np.float32(conf_thres))  # row-major, like torch.where
            box, conf, idx = box[i], x[i, 4 + j], idx[i]
        else:
            j = x[:, 4:].argmax(1)
            conf = x[np.arange(x.shape[0]), 4 + j]
            filt = conf > np.float32(conf_thres)
            box, conf, j, idx = box[filt], conf[filt], j[filt], idx[filt]
        if classes is not None:
            filt = np.isin(j, np.asarray(classes, np.int64))
            box, conf, j, idx = box[filt], conf[filt], j[filt], idx[filt]
        if box.shape[0] > max_nms:
            o = np.argsort(-conf, kind="stable")[:max_nms]
            box, conf, j, idx = box[o], conf[o], j[o], idx[o]
        c = j.astype(np.float32) * np.float32(0 if agnostic else max_wh)
        k = greedy_nms(box + c[:, None], conf, iou_thres)[:max_det]
        dets.append(np.concatenate([box[k], conf[k, None], j[k, None].astype(np.float32)], 1))
        keeps.append(idx[k])
    return dets, keeps
