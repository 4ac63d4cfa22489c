"""Batched detection predictor on the device: decoded uint8 images in, boxes in source-image pixels out.

The MI355X form of the reference's predict loop for detection (ultralytics/engine/predictor.py:151-201
preprocess / pre_transform, models/yolo/detect/predict.py:33-121 postprocess + construct_result):

    uint8 HWC BGR images --(fce_letterbox: resize + pad 114 + BGR->RGB, on the GPU)--> u8 NCHW batch
      --(Engine: forward; the stem divides by 255 with the fp16 rounding of `im.half() / 255`)--> pred
      --(NMS: conf / iou / max_det, bit-exact TorchNMS)--> (k, 6) per image
      --(fce_scale_boxes: ops.scale_boxes + clip_boxes)--> boxes in each source image's pixel frame

Letterbox placement is computed on the host exactly as LetterBox.__call__ does (augment.py:1575-1605,
Python round); images of any size share one (H, W) canvas (auto=False, the predictor's setting for
batched inputs of mixed shapes).  `Predictor` keeps several batches in flight (pinned staging, one H2D and
one D2H copy per batch, an executor lane with a captured hipGraph per slot).
"""

from __future__ import annotations

import ctypes as C
import threading

import numpy as np
import torch

from . import _native as N
from .engine import NMS, Engine, Poster


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


# numpy images of the C structs (fce_letterbox_img: pointer + 7 ints, padded to 40 bytes; fce_box_scale)
_LB_DT = np.dtype([("src", "<u8"), ("h0", "<i4"), ("w0", "<i4"), ("row_stride", "<i4"), ("new_h", "<i4"), ("new_w", "<i4"),
                   ("top", "<i4"), ("left", "<i4"), ("pad", "<i4")])
_BS_DT = np.dtype([("gain", "<f4"), ("pad_x", "<i4"), ("pad_y", "<i4"), ("h0", "<i4"), ("w0", "<i4")])


class _Lane:
    """An executor lane: the u8 canvas, an Engine clone (own arena, own stream, its captured hipGraph), NMS and
    the pinned host copy of its packed results."""

    def __init__(self, eng: Engine, batch: int, device, nms_kw):
        self.eng = eng
        self.stream = torch.cuda.Stream(device)
        self.canvas = torch.empty((batch, 3, eng.H, eng.W), dtype=torch.uint8, device=device)
        self.pred = torch.empty_like(eng.pred)
        self.best = eng.new_best()
        self.nms = NMS(batch, eng.anchors, eng.nc, device, **nms_kw)
        self.out_host = torch.empty(self.nms.buf.numel(), dtype=torch.uint8, pin_memory=True)
        self.send = self.gathered = None  # the multi-GPU gather's buffers (Predictor(gather=...))
        self.chain_done = torch.cuda.Event()  # the lane's chain (gathered path: the poster's host wait)
        self.posted = threading.Event()
        self.posted.set()
        self.done = torch.cuda.Event()
        self.ticket = None  # ticket whose results this lane holds (not yet collected)
        self.shapes = []


class _Stage:
    """A staging buffer: pinned host memory (descriptors + packed source images) and its device copy; `used`
    is recorded once the letterbox has read the device copy, after which both may be refilled."""

    def __init__(self):
        self.host = self.dev = None
        self.used = torch.cuda.Event()

    def reserve(self, nbytes: int, device):
        if self.host is None or self.host.numel() < nbytes:
            self.used.synchronize()
            cap = max(nbytes, 1 << 20)
            cap += cap // 4  # headroom: a slightly larger batch of images does not re-pin
            self.host = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
            self.dev = torch.empty(cap, dtype=torch.uint8, device=device)


def default_lanes(model) -> int:
    """Batches in flight for a model: 5 on the n / s scales, 3 on m / l / x (see Predictor)."""
    scale = (getattr(model, "yaml", None) or {}).get("scale") or "n"
    return 5 if scale in ("n", "s") else 3


def _host_image(im) -> np.ndarray:
    """A decoded image as a C-contiguous host array: numpy arrays and CPU tensors are accepted; a tensor on a
    device is refused (this path packs host images into pinned staging; device-resident images go through
    `Letterbox` + `Engine` + `NMS` directly)."""
    if isinstance(im, torch.Tensor):
        if im.device.type != "cpu":
            raise TypeError(f"Predictor: images must be host arrays (numpy or CPU tensors), got a {im.device} tensor; "
                            "for device-resident images use predict.Letterbox + Engine + NMS")
        im = im.numpy()
    return np.ascontiguousarray(im)


class Predictor:
    """predict(images) -> per image (k, 6) [x1, y1, x2, y2, conf, cls] in source pixels (+ anchor indices).

    The reference's predict loop (engine/predictor.py:151-182 preprocess, :276-381 stream_inference) as a
    pipeline of `lanes` batches in flight on the device.  `submit(images)` returns a ticket at once:

      * the decoded uint8 HWC images are packed by a host thread pool into a PINNED staging buffer behind the
        letterbox / box-scale descriptors (built on the host exactly as LetterBox.__call__ and ops.scale_boxes
        compute them), and go to the device in ONE async H2D copy;
      * device letterbox -> forward (the lane's executor replays its captured hipGraph) -> NMS with the Detect
        epilogue's best-class keys -> scale_boxes, all on the lane's stream;
      * the packed NMS outputs come back in one async D2H copy into pinned memory.

    Staging buffers (lanes + 1 of them) are separate from the lanes: a buffer is free again as soon as the
    letterbox of its batch has run, so `stream()` packs batch i + 1 while batches i - lanes + 1 .. i are on the
    device.  `result(ticket)` waits for that batch only and returns host tensors; a lane's results not
    collected when the lane is reused are kept on the host.  A call with fewer images than `batch` repeats the
    last canvas (those rows are dropped).  `__call__` = result(submit(...))."""

    def __init__(self, model, batch: int, imgsz=640, device=None, conf=0.25, iou=0.7, max_det=300,
                 lanes: int | None = None, graph: bool = True, workers: int | None = None, copy_stream: bool = True,
                 gather=None):
        """`lanes`: batches on the device at once; default by scale (`default_lanes`): 5 on the n / s scales
        (measured best for 32 x 480x640 images, scripts/predict_diag.py), 3 on m / l, where every lane's
        activation arena is large and more than three arenas overflow the MALL (bench.default_lanes).
        `workers`: host threads packing images into pinned memory (default min(8, cpus / 2); 4-8 reach ~31 GB/s
        on the MI355X box).  `copy_stream` (default): every H2D copy on one dedicated stream, lanes wait on it
        (18.9k against 15.9k images/s with the copy on the lane's own stream, scripts/predict_diag.py).
        `gather` (a `dist.DeviceGather`, set by dist.ShardedHostPredictor): every batch's packed NMS outputs are
        all-gathered over the ranks on one side stream in batch order before the D2H copy, and results are the
        whole global batch's (every submit must then carry exactly `batch` images)."""
        import os
        from concurrent.futures import ThreadPoolExecutor

        if lanes is None:
            lanes = default_lanes(model)
        self.engine = Engine(model, batch, imgsz, device, graph=graph)
        self.device = self.engine.device
        self.batch = batch
        self.max_det = max_det
        nms_kw = dict(conf=conf, iou=iou, max_det=max_det)
        engs = [self.engine] + [self.engine.clone() for _ in range(max(1, lanes) - 1)]
        for e in engs:
            e.graph = graph
        self.lanes = [_Lane(e, batch, self.device, nms_kw) for e in engs]
        self.gather = gather
        self.poster = None
        if gather is not None:
            self.poster = Poster(self.device)  # the collectives, in batch order, issued from a host thread
            for ln in self.lanes:
                ln.send, ln.gathered = gather.buffers(self.device)
                ln.out_host = torch.empty(gather.nbytes, dtype=torch.uint8, pin_memory=True)
        self.copy = torch.cuda.Stream(self.device) if copy_stream else None
        self.stages = [_Stage() for _ in range(len(self.lanes) + 1)]
        self.nms = self.lanes[0].nms  # lane 0's NMS (API compatibility)
        self.lb = Letterbox(batch, (self.engine.H, self.engine.W), self.device)  # standalone use
        self.workers = workers or max(1, min(8, (os.cpu_count() or 2) // 2))
        self.pool = ThreadPoolExecutor(self.workers)
        self._geom = {}  # (h0, w0) -> (letterbox placement, box-scale parameters)
        self._n = 0  # batches staged so far
        self._ready = {}  # ticket -> results collected early (lane reused before result())

    def _desc_bytes(self) -> int:
        return (self.batch * (C.sizeof(LetterboxImg) + C.sizeof(BoxScale)) + 255) // 256 * 256

    def _stage(self, images):
        """Host half of a submit: the next staging buffer (waiting only for the letterbox of its previous
        batch), descriptors written into it, and the packing of the images started on the host thread pool.
        Returns the record _issue consumes; the packing runs while the caller does other work."""
        if not 0 < len(images) <= self.batch:
            raise ValueError(f"Predictor: 1..{self.batch} images per call")
        if self.gather is not None and len(images) != self.batch:
            raise ValueError(f"Predictor: the gathered path takes whole {self.batch}-image shards, got {len(images)}")
        imgs = [_host_image(im) for im in images]
        for im in imgs:
            if im.dtype != np.uint8 or im.ndim != 3 or im.shape[2] != 3:
                raise ValueError("Predictor: images must be uint8 (h, w, 3) BGR arrays")
        i = self._n
        self._n += 1
        sb = self.stages[i % len(self.stages)]
        n = len(imgs)
        H, W = self.engine.H, self.engine.W
        db = self._desc_bytes()
        sizes = np.array([(im.nbytes + 255) // 256 * 256 for im in imgs], np.int64)
        offs = db + np.concatenate(([0], np.cumsum(sizes)[:-1]))
        off = int(db + sizes.sum())
        sb.reserve(off, self.device)
        sb.used.synchronize()  # the previous batch's letterbox has read this buffer
        hbase, dbase = sb.host.data_ptr(), sb.dev.data_ptr()
        hnp = sb.host.numpy()
        # one packing task per worker (a contiguous run of images), not one per image
        nw = min(self.workers, n)
        bounds = [n * w // nw for w in range(nw + 1)]

        def pack(lo, hi):
            for j in range(lo, hi):
                im = imgs[j]
                np.copyto(hnp[offs[j]:offs[j] + im.nbytes].reshape(im.shape), im)

        futs = [self.pool.submit(pack, bounds[w], bounds[w + 1]) for w in range(nw)]
        # descriptors: letterbox placement and box scaling per distinct source shape (host, reference rounding)
        lbd = np.zeros(n, _LB_DT)
        scd = np.zeros(self.batch, _BS_DT)
        shapes = [im.shape[:2] for im in imgs]
        for j, (h0, w0) in enumerate(shapes):
            g = self._geom.get((h0, w0))
            if g is None:
                g = self._geom[(h0, w0)] = (letterbox_geometry(h0, w0, H, W), box_scale(H, W, h0, w0))
            (new_h, new_w, top, left), (gain, px, py) = g
            lbd[j] = (dbase + int(offs[j]), h0, w0, w0 * 3, new_h, new_w, top, left, 0)
            scd[j] = (gain, px, py, h0, w0)
        scd[n:] = scd[n - 1]
        C.memmove(hbase, lbd.ctypes.data, lbd.nbytes)
        C.memmove(hbase + self.batch * C.sizeof(LetterboxImg), scd.ctypes.data, scd.nbytes)
        return i, sb, futs, n, off, shapes

    def _issue(self, staged) -> int:
        """Device half: lane i % lanes (its previous results collected first), once the packing is done one H2D
        copy and the whole chain on the lane's stream.  Returns the ticket."""
        i, sb, futs, n, off, shapes = staged
        ln = self.lanes[i % len(self.lanes)]
        if ln.ticket is not None:  # the lane's previous batch: collect it before its buffers are reused
            t = ln.ticket
            self._ready[t] = self._collect(ln)
        for f in futs:
            f.result()
        H, W = self.engine.H, self.engine.W
        dbase = sb.dev.data_ptr()
        nlb = self.batch * C.sizeof(LetterboxImg)
        main = torch.cuda.current_stream(self.device)
        ln.stream.wait_stream(main)
        if self.copy is not None:
            self.copy.wait_stream(main)
            with torch.cuda.stream(self.copy):
                sb.dev[:off].copy_(sb.host[:off], non_blocking=True)  # descriptors + images: one H2D copy
            ln.stream.wait_stream(self.copy)
        with torch.cuda.stream(ln.stream):
            if self.copy is None:
                sb.dev[:off].copy_(sb.host[:off], non_blocking=True)  # descriptors + images: one H2D copy
            st = ln.stream.cuda_stream
            N.call("fce_letterbox", C.c_void_p(dbase), n, C.c_void_p(ln.canvas.data_ptr()), H, W, self.lb.pad, st)
            # the box-scale descriptors are read by scale_boxes below: copy them out before the buffer is freed
            sc = self._scales_dev(ln)
            sc.copy_(sb.dev[nlb:nlb + sc.numel()])
            sb.used.record(ln.stream)
            if n < self.batch:  # fixed-shape engine: pad the batch by repeating the last canvas
                ln.canvas[n:].copy_(ln.canvas[n - 1:n].expand(self.batch - n, -1, -1, -1))
            ln.eng(ln.canvas, out=ln.pred, best=ln.best)
            dets, keep, counts = ln.nms(ln.pred, ln.best)
            N.call("fce_scale_boxes", C.c_void_p(dets.data_ptr()), C.c_void_p(counts.data_ptr()), self.batch,
                   self.max_det, C.c_void_p(sc.data_ptr()), st)
            if self.gather is None:
                ln.out_host.copy_(ln.nms.buf, non_blocking=True)  # packed keep | dets | counts: one D2H copy
                ln.done.record(ln.stream)
            else:
                ln.chain_done.record(ln.stream)
        if self.gather is not None:
            # every rank's packed outputs gathered once the lane's chain is done (host-ordered poster: no side-stream
            # wait on the device), then one D2H copy of the gathered block
            def fn(ln=ln):
                self.gather.issue(ln.nms, ln.send, ln.gathered)
                ln.out_host.copy_(ln.gathered, non_blocking=True)
                ln.done.record(self.poster.stream)

            self.poster.submit(ln.chain_done, fn, ln.posted)
        ln.ticket = i + 1
        ln.shapes = shapes
        return ln.ticket

    def _scales_dev(self, ln: _Lane) -> torch.Tensor:
        if not hasattr(ln, "scales"):
            ln.scales = torch.empty(self.batch * C.sizeof(BoxScale), dtype=torch.uint8, device=self.device)
        return ln.scales

    def submit(self, images) -> int:
        return self._issue(self._stage(images))

    def _collect(self, ln: _Lane):
        ln.posted.wait()
        if self.poster is not None:
            self.poster._check()  # a failed gather / D2H never records ln.done: out_host would hold an older batch
        ln.done.synchronize()
        if self.gather is not None:
            ln.ticket = None
            return self.gather.unpack(ln.out_host.clone())  # the whole global batch, unsharded order
        keep, dets, counts = NMS.unpack(ln.out_host.clone(), self.batch, self.max_det)  # one copy out of pinned memory
        n = len(ln.shapes)
        cnt = counts[:n].tolist()
        res = ([dets[i, :cnt[i]] for i in range(n)], [keep[i, :cnt[i]] for i in range(n)])
        ln.ticket = None
        return res

    def result(self, ticket: int, return_idxs: bool = False):
        """Per image (k, 6) HOST tensors of a submitted batch (+ kept anchor indices): the packed detections come
        back in one D2H copy per batch; `.to(device)` them if the caller's next step is on the GPU."""
        if ticket in self._ready:
            d, k = self._ready.pop(ticket)
        else:
            ln = next((x for x in self.lanes if x.ticket == ticket), None)
            if ln is None:
                raise KeyError(f"Predictor: unknown or already collected ticket {ticket}")
            d, k = self._collect(ln)
        return (d, k) if return_idxs else d

    def __call__(self, images, return_idxs: bool = False):
        if len(images) == 0:
            return ([], []) if return_idxs else []
        return self.result(self.submit(images), return_idxs)

    def stream(self, batches, return_idxs: bool = False):
        """Generator over an iterable of image batches with `lanes` batches in flight, results in order.  Batch
        i + 1 is staged (its images packed by the host pool) before batch i is issued, so the packing overlaps
        the host's launches and the device work of the batches in flight."""
        from collections import deque

        q = deque()
        it = iter(batches)
        nxt = next(it, None)
        staged = self._stage(nxt) if nxt is not None else None
        while staged is not None:
            nxt = next(it, None)
            ahead = self._stage(nxt) if nxt is not None else None
            q.append(self._issue(staged))  # may collect q[0] into _ready (its lane is reused)
            staged = ahead
            while q and (len(q) >= len(self.lanes) or staged is None or q[0] in self._ready):
                yield self.result(q.popleft(), return_idxs)

    def close(self):
        if self.poster is not None:
            self.poster.drain()
            self.poster.close()
        torch.cuda.synchronize(self.device)
        self.pool.shutdown()
        for ln in self.lanes:
            ln.eng.close()
