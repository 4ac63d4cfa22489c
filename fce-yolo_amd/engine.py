"""Whole-graph inference engine and NMS (the AutoBackend / predictor side of the path).

``Engine`` lowers a ``DetectionModel`` once into a native ``fce_net`` (buffer arena + launch list),
plans it for (batch, H, W) and runs it as one hipGraph replay per batch — the MI355X form of
``AutoBackend.forward`` (reference ``nn/autobackend.py:667-700``) + ``_predict_once``
(``nn/tasks.py:160-188``).  ``non_max_suppression`` runs the device NMS kernel with the predict
defaults of ``utils/nms.py:13-166`` / ``cfg/default.yaml:53-55`` (conf 0.25, iou 0.7, max_det 300,
max_nms 30000, max_wh 7680) and returns the same per-image (k, 6) tensors and kept anchor indices.
"""

from __future__ import annotations

import ctypes as C
import math
import os
import queue
import threading

import torch

from . import _native as N
from .backend import NetBackend

_DT = {torch.float16: N.F16, torch.float32: N.F32, torch.uint8: N.U8}


class Engine:
    def __init__(self, model, batch: int, imgsz: int | tuple[int, int], device=None, graph: bool = False,
                 autotune: bool | None = None):
        """`autotune`: time every conv's kernel variants at plan and keep the fastest (None: unless the
        environment sets FCE_AUTOTUNE=0)."""
        if isinstance(imgsz, int):
            imgsz = (imgsz, imgsz)
        self.H, self.W = imgsz
        self.batch = batch
        self.device = torch.device(device) if device is not None else next(model.parameters()).device
        if self.device.type != "cuda":
            raise RuntimeError("Engine: fce_yolo_amd runs on ROCm devices only; no CPU fallback")
        self.model = model
        self.graph = graph
        self.be = NetBackend(self.H, self.W, self.device)
        with torch.no_grad():
            x = self.be.input_view(batch, model.yaml.get("channels", 3))
            model.emit(self.be, x)
        if autotune is None:
            N.call("fce_net_plan", self.be.net, batch, self.H, self.W)
        else:
            N.call("fce_net_plan_ex", self.be.net, batch, self.H, self.W, 0 if autotune else N.PLAN_NO_AUTOTUNE)
        self.anchors = N.lib().fce_net_num_anchors(self.be.net)
        self.nc = model.model[-1].nc
        self.pred = torch.empty((batch, 4 + self.nc, self.anchors), dtype=torch.float32, device=self.device)
        self.best = self.new_best()

    def new_best(self) -> torch.Tensor:
        """A (batch, A) buffer for the per-anchor best-class keys the forward can emit for the NMS
        (score bits << 32 | ~class, fce_detect_epi.best)."""
        return torch.zeros((self.batch, self.anchors), dtype=torch.int64, device=self.device)

    def close(self):
        self.be.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def net(self):
        return self.be.net

    def _in(self, x: torch.Tensor) -> N.Tensor:
        if x.device != self.device or x.dtype not in _DT:
            raise ValueError("Engine: input must be f16/f32/u8 on the engine's device")
        if tuple(x.shape) != (self.batch, 3, self.H, self.W) or not x.is_contiguous():
            raise ValueError(f"Engine: input must be contiguous NCHW {(self.batch, 3, self.H, self.W)}")
        return N.Tensor(x.data_ptr(), _DT[x.dtype], N.NCHW, self.batch, 3, self.H, self.W, 3, 0)

    def __call__(self, x: torch.Tensor, out: torch.Tensor | None = None, graph: bool | None = None,
                 best: torch.Tensor | None = None) -> torch.Tensor:
        """Forward into `out` (default: self.pred, with its best-class keys in self.best).  `best`: a
        new_best() buffer that receives the keys of this forward (for NMS(pred, best))."""
        if out is None:
            out, best = self.pred, self.best if best is None else best
        if best is not None:
            assert best.dtype == torch.int64 and tuple(best.shape) == (self.batch, self.anchors) and best.is_contiguous()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        g = self.graph if graph is None else graph
        N.call("fce_net_forward_best", self.be.net, C.byref(self._in(x)), out.data_ptr(),
               best.data_ptr() if best is not None else None, int(bool(g)), stream)
        return out

    def clone(self) -> "Engine":
        """A second executor of the same model and shapes with its own arena, pinned to this one's kernel
        variants (no second autotune): a lane of a multi-lane Pipeline."""
        e = Engine(self.model, self.batch, (self.H, self.W), self.device, graph=self.graph, autotune=False)
        for i in range(self.num_ops()):
            if self.variants(i):
                e.set_variant(i, self.variant(i))
            f = self.alt_form(i)
            if f >= 0:
                e.set_alt_form(i, bool(f))
        return e

    def alt_form(self, i: int) -> int:
        """1: op i (a fused C3k2 or Detect cls branch with the ops it replaces as the alternative) runs fused; 0: the
        ops run; -1: other op."""
        return N.lib().fce_net_alt_form(self.be.net, i)

    def set_alt_form(self, i: int, fused: bool) -> None:
        N.call("fce_net_set_alt_form", self.be.net, i, int(bool(fused)))

    def c3k2_form(self, i: int) -> int:
        """1: op i (a fused C3k2 with its four convs as the alternative) runs fused; 0: the convs run; -1: other op."""
        return N.lib().fce_net_c3k2_form(self.be.net, i)

    def set_c3k2_form(self, i: int, fused: bool) -> None:
        N.call("fce_net_set_c3k2_form", self.be.net, i, int(bool(fused)))

    def skipped(self, i: int) -> bool:
        """Op i belongs to the inactive form of an alternative (launches nothing)."""
        return bool(N.lib().fce_net_op_skipped(self.be.net, i))

    def profile(self, x: torch.Tensor, launches: bool = False):
        """Eager run, every kernel timed by its own dispatch-attached event pair:
        [(name, bytes, flops, ms)] per op (+ kernel count per op when `launches`)."""
        n = N.lib().fce_net_num_ops(self.be.net)
        ms = (C.c_float * n)()
        nl = (C.c_int * n)()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        N.call("fce_net_profile", self.be.net, C.byref(self._in(x)), self.pred.data_ptr(), C.cast(ms, C.c_void_p),
               C.cast(nl, C.c_void_p), n, stream)
        if launches:
            return [(*self.op_info(i), float(ms[i]), int(nl[i])) for i in range(n)]
        return [(*self.op_info(i), float(ms[i])) for i in range(n)]

    def op_info(self, i: int):
        name = C.create_string_buffer(64)
        b, f = C.c_double(), C.c_double()
        N.call("fce_net_op_info", self.be.net, i, name, 64, C.byref(b), C.byref(f))
        return name.value.decode(), b.value, f.value

    def num_ops(self) -> int:
        return N.lib().fce_net_num_ops(self.be.net)

    def variants(self, i: int) -> list[int]:
        """Candidate kernel variants of conv op i (empty for other ops)."""
        codes = (C.c_int * 128)()
        nv = N.lib().fce_net_op_variants(self.be.net, i, C.cast(codes, C.c_void_p), 128)
        return list(codes[:nv])

    def variant(self, i: int) -> int:
        return N.lib().fce_net_op_variant(self.be.net, i)

    def set_variant(self, i: int, code: int) -> None:
        """Pin conv op i to one of its candidates (-1 = heuristic); every candidate is bitwise equal."""
        N.call("fce_net_set_op_variant", self.be.net, i, code)

    def arena_bytes(self) -> int:
        return N.lib().fce_net_arena_bytes(self.be.net)


class NMS:
    """Device NMS with persistent workspace/outputs (graph-capturable)."""

    def __init__(self, batch, anchors, nc, device, conf=0.25, iou=0.7, max_det=300, max_nms=30000, max_wh=7680,
                 classes=None, agnostic=False, multi_label=False, buf=None, layout_batch=None):
        """`classes` / `agnostic` / `multi_label`: the non-default arguments of nms.py:13-29 (fce_nms_ex).
        `buf` / `layout_batch`: the outputs go into the caller's packed buffer (packed_bytes(layout_batch)), laid out
        for `layout_batch` >= batch images, the first `batch` rows written (a multi-GPU gather sends a remainder
        shard in the largest shard's layout, and consecutive slots' buffers form one contiguous send block)."""
        self.batch, self.anchors, self.nc = batch, anchors, nc
        self.conf, self.iou, self.max_det, self.max_nms, self.max_wh = conf, iou, max_det, max_nms, max_wh
        self.opts = None
        if classes is not None or agnostic or multi_label:
            cls = [int(c) for c in (classes.tolist() if hasattr(classes, "tolist") else classes)] \
                if classes is not None else None
            self._classes = (C.c_int32 * max(len(cls), 1))(*cls) if cls is not None else None
            self.opts = N.NmsOpts(conf, iou, max_det, max_nms, float(max_wh), int(bool(agnostic)),
                                  int(bool(multi_label)), C.cast(self._classes, C.c_void_p) if cls is not None else None,
                                  len(cls) if cls is not None else 0)
            nb = N.lib().fce_nms_workspace_bytes_ex(batch, nc, anchors, C.byref(self.opts))
        else:
            nb = N.lib().fce_nms_workspace_bytes(batch, anchors, max_nms)
        self.ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=device)
        # outputs packed in one buffer (keep | dets | counts), so a multi-GPU gather is one collective
        lb = batch if layout_batch is None else int(layout_batch)
        assert lb >= batch
        nbp = self.packed_bytes(lb, max_det)
        if buf is None:
            buf = torch.zeros(nbp, dtype=torch.uint8, device=device)
        assert buf.dtype == torch.uint8 and buf.numel() == nbp and buf.is_contiguous()
        self.buf = buf
        keep, dets, counts = self.unpack(self.buf, lb, max_det)
        self.keep, self.dets, self.counts = keep[:batch], dets[:batch], counts[:batch]
        self.device = device

    @staticmethod
    def packed_bytes(batch: int, max_det: int) -> int:
        return batch * max_det * (8 + 24) + (batch * 4 + 15) // 16 * 16  # 16-byte multiple: blocks stay aligned

    @staticmethod
    def unpack(buf: torch.Tensor, batch: int, max_det: int):
        """(keep (b,max_det) i64, dets (b,max_det,6) f32, counts (b,) i32) views of a packed output buffer."""
        k, d = batch * max_det * 8, batch * max_det * 24
        keep = buf[:k].view(torch.int64).view(batch, max_det)
        dets = buf[k:k + d].view(torch.float32).view(batch, max_det, 6)
        counts = buf[k + d:k + d + batch * 4].view(torch.int32)
        return keep, dets, counts

    def __call__(self, pred: torch.Tensor, best: torch.Tensor | None = None):
        """`best`: the best-class keys the forward wrote with `pred` (Engine(..., best=)), which spares the
        class arg-max pass over pred; the results are the same either way."""
        assert pred.is_contiguous() and pred.dtype == torch.float32 and tuple(pred.shape) == (
            self.batch, 4 + self.nc, self.anchors)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        if self.opts is not None:
            if best is not None:
                assert best.dtype == torch.int64 and tuple(best.shape) == (self.batch, self.anchors)
            N.call("fce_nms_ex", pred.data_ptr(), best.data_ptr() if best is not None else None, self.batch, self.nc,
                   self.anchors, C.byref(self.opts), self.ws.data_ptr(), self.ws.numel(), self.dets.data_ptr(),
                   self.keep.data_ptr(), self.counts.data_ptr(), stream)
            return self.dets, self.keep, self.counts
        args = (self.batch, self.nc, self.anchors, self.conf, self.iou, self.max_det, self.max_nms,
                float(self.max_wh), self.ws.data_ptr(), self.ws.numel(), self.dets.data_ptr(), self.keep.data_ptr(),
                self.counts.data_ptr(), stream)
        if best is not None:
            assert best.dtype == torch.int64 and tuple(best.shape) == (self.batch, self.anchors)
            N.call("fce_nms_best", pred.data_ptr(), best.data_ptr(), *args)
        else:
            N.call("fce_nms", pred.data_ptr(), *args)
        return self.dets, self.keep, self.counts

    def results(self):
        counts = self.counts.cpu().tolist()
        return ([self.dets[b, :k] for b, k in enumerate(counts)], [self.keep[b, :k] for b, k in enumerate(counts)])


def non_max_suppression(pred: torch.Tensor, conf_thres=0.25, iou_thres=0.7, max_det=300, max_nms=30000, max_wh=7680,
                        return_idxs=False, classes=None, agnostic=False, multi_label=False):
    """nms.py:13-166 on the device: list of (k, 6) [x1,y1,x2,y2,conf,cls] per image (+ kept anchor indices).
    `classes`, `agnostic`, `multi_label` as in the reference (fce_nms_ex)."""
    if pred.device.type != "cuda":
        raise RuntimeError("non_max_suppression: ROCm device tensor required (no CPU fallback)")
    pred = pred.float().contiguous()
    b, no, a = pred.shape
    nms = NMS(b, a, no - 4, pred.device, conf_thres, iou_thres, max_det, max_nms, max_wh, classes=classes,
              agnostic=agnostic, multi_label=multi_label)
    nms(pred)
    dets, keep = nms.results()
    return (dets, keep) if return_idxs else dets


class Poster:
    """Post-processing of finished batches on a side stream, issued from a host thread in submission order.

    `submit(ready, fn, posted)`: once the GPU has passed `ready` (a host wait in the poster's thread), `fn()` runs
    with the poster's stream current and `posted` is set.  No GPU-side cross-stream wait is enqueued: with four
    lanes saturating the GPU, one barrier packet per batch on a side queue waiting for a lane's event cost 17 % of
    the pipelined n32 rate, whatever the side stream then did (a one-rank RCCL group: 29.9-30.1k images/s with a
    no-op post against 36.0-36.4k without one, profiles/r05s_*; more hardware queues made it worse, 25k at 10-24).
    Collectives issued here keep the submission order on every rank."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device)
        self.q: queue.Queue = queue.Queue()
        self.err = None
        self.thread = threading.Thread(target=self._run, name="fce-poster", daemon=True)
        self.thread.start()

    def _run(self):
        torch.cuda.set_device(self.device)
        while True:
            item = self.q.get()
            if item is None:
                self.q.task_done()
                return
            ready, fn, posted = item
            try:
                if self.err is None:
                    ready.synchronize()
                    with torch.cuda.stream(self.stream):
                        fn()
            except BaseException as e:  # surfaced by the next submit / drain
                self.err = e
            finally:
                posted.set()
                self.q.task_done()

    def _check(self):
        if self.err is not None:
            raise RuntimeError(f"post-processing failed: {self.err!r}") from self.err

    def submit(self, ready: torch.cuda.Event, fn, posted: threading.Event):
        self._check()
        posted.clear()
        self.q.put((ready, fn, posted))

    def drain(self):
        """Every submitted item has been issued (its GPU work enqueued, not necessarily finished)."""
        self.q.join()
        self._check()

    def close(self):
        if self.thread.is_alive():
            self.q.put(None)
            self.thread.join()


class Pipeline:
    """Batch pipeline: the NMS of batch i overlaps the forward of batch i+1.

    The forward runs on the caller's stream into one of `depth` pred buffers (+ best-class keys); the NMS
    of that buffer runs on a side stream.  A buffer (and its NMS outputs) is reused only after the NMS
    that read it has finished (event wait on the caller's stream), so every batch gets exactly the
    forward + NMS of the sequential path.

    With `defer` (default) the NMS of batch i is issued only after the forward of batch i+1 has been
    enqueued, and waits for that forward's fork point (``fce_net_set_fork`` at ``fce_net_fork_hint``: the
    first op at stride 32): it then runs while the forward is in its small coarse-resolution layers that
    leave most CUs idle, instead of competing with the full-width early layers.  `flush()` issues the
    last pending NMS; `wait` / `results` flush when needed.  `submit(x)` returns the slot whose `NMS`
    object holds that batch's results once `wait(slot)` (or a device sync after `flush()`) has passed.

    With `lanes` > 1 the pipeline keeps that many batches in flight: lane l = slot % lanes owns an
    executor (``Engine.clone``: its own arena, the same kernel variants) and a stream, and runs forward
    then NMS of its batches in order on that stream.  `x` is recorded on the lane stream
    (``record_stream``), so the caller may drop its reference right after `submit`.  The lanes share the GPU, so the latency-bound
    40^2 / 20^2 layers and the NMS of one batch run beside the full-width early layers of the next
    (n-fce 640 bs32: 1.48 -> 1.16 ms per batch, forward only, ``scripts/dual_engine.py``).  Every batch
    still gets the bitwise result of the sequential path.  A lane reads `x` asynchronously: the caller
    must not write into `x` until that batch's `wait(slot)` / `results(slot)`.  `post` runs on one
    side stream in submission order (collectives stay ordered across ranks).
    """

    def __init__(self, engine: Engine, depth: int = 2, post=None, defer: bool = True, lanes: int = 1,
                 post_every: int = 1, layout_batch: int | None = None, **nms_kw):
        """`post(k0, m)`, if given, runs on a side stream after the NMS of slots k0 .. k0 + m - 1 (e.g. the multi-GPU
        gather of their outputs, dist.ShardedPredictor); those slots' NMS outputs are reused only after it too has
        finished.  `post_every` = G (lanes only): one post per G consecutive batches, whose NMS outputs are then one
        contiguous block (`outbuf[k0 * nb : (k0 + m) * nb]`, nb = NMS.packed_bytes(layout_batch)), so a gather is one
        collective per G batches; `flush()` posts a partial group.  `layout_batch`: NMS outputs laid out for that
        many images (the largest shard of a sharded batch)."""
        self.lanes = max(1, int(lanes))
        self.G = max(1, int(post_every)) if (post is not None and self.lanes > 1) else 1
        unit = self.lanes * self.G // math.gcd(self.lanes, self.G)
        depth = max(depth, self.lanes, 2 * self.G if self.G > 1 else 1)
        depth = -(-depth // unit) * unit  # a multiple of lanes and of G
        if self.lanes > 1:
            defer = False  # each lane runs its NMS right after its own forward
        self.eng, self.depth, self.post, self.defer = engine, depth, post, defer
        dev = engine.device
        self.engs = [engine] + [engine.clone() for _ in range(self.lanes - 1)]
        self.lane_streams = [torch.cuda.Stream(dev) for _ in range(self.lanes)] if self.lanes > 1 else []
        self.in_ready = [torch.cuda.Event() for _ in range(depth)]
        self.lane_done = [torch.cuda.Event() for _ in range(depth)]
        self.preds = [torch.empty_like(engine.pred) for _ in range(depth)]
        self.bests = [engine.new_best() for _ in range(depth)]
        lb = engine.batch if layout_batch is None else int(layout_batch)
        self.nb = NMS.packed_bytes(lb, nms_kw.get("max_det", 300))
        self.outbuf = torch.zeros(depth * self.nb, dtype=torch.uint8, device=dev)  # slot k: [k nb, (k + 1) nb)
        self.nms = [NMS(engine.batch, engine.anchors, engine.nc, dev, buf=self.outbuf[k * self.nb:(k + 1) * self.nb],
                        layout_batch=lb, **nms_kw) for k in range(depth)]
        self.side = torch.cuda.Stream(dev)
        self.fwd_done = [torch.cuda.Event() for _ in range(depth)]
        self.nms_done = [torch.cuda.Event() for _ in range(depth)]
        self.used = [False] * depth
        self.pending = None  # slot whose NMS is not issued yet (defer)
        self.i = 0
        # diagnostics only (FCE_PIPE_SKIP_NMS=1): lanes run the forwards alone, so the NMS's share of the pipelined
        # step can be measured; the results are then meaningless
        self._skip_nms = os.environ.get("FCE_PIPE_SKIP_NMS") == "1"
        self._wait_always = os.environ.get("FCE_LANE_WAIT_ALWAYS") == "1"  # diagnostics: the pre-round-5 waits
        # lanes with post: the posts are issued by a host thread (Poster) once the lanes have finished the group's
        # batches; FCE_POST_DEVICE_WAIT=1 restores the device-side waits on the side stream (diagnostics)
        self.poster = None
        if self.lanes > 1 and post is not None and os.environ.get("FCE_POST_DEVICE_WAIT") != "1":
            self.poster = Poster(dev)
            self.side = self.poster.stream
        self._posted = [threading.Event() for _ in range(depth)]
        for e in self._posted:
            e.set()
        self._group = []  # slots of the current post group not posted yet
        self._groups = {}  # slot -> (first slot, slots) of the group it was last posted with
        if defer:
            N.call("fce_net_set_fork", engine.net, N.lib().fce_net_fork_hint(engine.net))

    def _issue_nms(self, k: int, fork: bool):
        self.side.wait_event(self.fwd_done[k])
        if fork:  # the next forward has reached its coarse layers
            N.call("fce_net_wait_fork", self.eng.net, self.side.cuda_stream)
        with torch.cuda.stream(self.side):
            self.nms[k](self.preds[k], self.bests[k])
            if self.post is not None:
                self.post(k, 1)
            self.nms_done[k].record(self.side)

    def _post_group(self):
        """Post the block of G slots the current group's batches went into (consecutive, in submission order).  A
        partial group (flush) posts the whole block too: its other slots still hold earlier batches whose results are
        live, and the block's gathered copy is laid out for all G slots."""
        ks, self._group = self._group, []
        if not ks:
            return
        k0, m = ks[0] - ks[0] % self.G, self.G
        # groups are aligned slot blocks: a group is posted when its block's last slot is submitted, a flushed partial
        # group leaves the rest of its block to the next post of the same block, so no group crosses a block boundary
        assert all(k0 <= k < k0 + m for k in ks), f"post group {ks} crosses the slot block [{k0}, {k0 + m})"
        block = range(k0, k0 + m)
        done = torch.cuda.Event()
        for k in block:
            self.nms_done[k] = done
            self._groups[k] = (k0, m)
        if self.poster is not None:
            ready = [self.lane_done[k] for k in block if self.used[k] or k in ks]

            def fn(k0=k0, m=m, ready=ready, done=done):
                for e in ready[:-1]:  # the poster waits for every lane's batch of the group on the host
                    e.synchronize()
                self.post(k0, m)
                done.record(self.poster.stream)

            # one poster item per group; the slots' `posted` flags are set together
            flag = threading.Event()
            self.poster.submit(ready[-1], fn, flag)
            for k in block:
                self._posted[k] = flag
        else:
            for k in block:
                if self.used[k] or k in ks:
                    self.side.wait_event(self.lane_done[k])
            with torch.cuda.stream(self.side):
                self.post(k0, m)
                done.record(self.side)

    def _submit_lane(self, x: torch.Tensor, k: int) -> int:
        lane = k % self.lanes
        s, eng = self.lane_streams[lane], self.engs[lane]
        main = torch.cuda.current_stream(self.eng.device)
        self.in_ready[k].record(main)  # x (and anything the caller queued before) is ready
        if self._wait_always or not self.in_ready[k].query():  # a cross-queue wait is enqueued only when needed
            s.wait_event(self.in_ready[k])
        x.record_stream(s)  # the lane reads x asynchronously: its block stays allocated until the lane has
        with torch.cuda.stream(s):
            eng(x, out=self.preds[k], best=self.bests[k])
            self.fwd_done[k].record(s)
            if self.used[k] and self.post is not None:
                # the post of the slot's previous batch has read nms[k] (pred / best are the lane's own: stream order)
                self.check_posted(k)
                if self._wait_always or not self.nms_done[k].query():
                    s.wait_event(self.nms_done[k])
            if not self._skip_nms:
                self.nms[k](self.preds[k], self.bests[k])
            self.lane_done[k].record(s)
        if self.post is None:
            self.nms_done[k] = self.lane_done[k]
        else:
            self._group.append(k)
            if k % self.G == self.G - 1:  # the last slot of its block (after a flushed partial group, the rest of it)
                self._post_group()
        self.used[k] = True
        return k

    def submit(self, x: torch.Tensor) -> int:
        k = self.i % self.depth
        self.i += 1
        if self.lanes > 1:
            return self._submit_lane(x, k)
        main = torch.cuda.current_stream(self.eng.device)
        if self.pending == k:  # depth 1: this slot's NMS must be issued before the slot is reused
            self.flush()
        if self.used[k]:
            main.wait_event(self.nms_done[k])  # pred[k] / nms[k] free again
        self.eng(x, out=self.preds[k], best=self.bests[k])
        self.fwd_done[k].record(main)
        self.used[k] = True
        if not self.defer:
            self._issue_nms(k, False)
            return k
        if self.pending is not None:
            self._issue_nms(self.pending, True)
        self.pending = k
        return k

    def flush(self):
        """Issue the NMS still pending (deferred mode) without waiting for another forward, the post of a partial
        group (lanes), and every post still queued on the host: afterwards a device synchronisation covers all
        submitted work."""
        if self.pending is not None:
            k, self.pending = self.pending, None
            self._issue_nms(k, False)
        if self._group:
            self._post_group()
        if self.poster is not None:
            self.poster.drain()

    def check_posted(self, k: int):
        """Wait until slot k's post has been issued, and raise if a post failed (its outputs would be stale)."""
        self._posted[k].wait()
        if self.poster is not None:
            self.poster._check()

    def close(self):
        """Issue what is still pending, then stop the poster thread.  A Pipeline with a `post` and lanes runs a host
        thread (Poster): close it (or use it as a context manager) when done."""
        try:
            self.flush()
        finally:
            if self.poster is not None:
                self.poster.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def group_of(self, k: int):
        """(first slot, slots) of the post group slot k was posted with (lanes with post)."""
        return self._groups.get(k, (k, 1))

    def wait(self, k: int | None = None):
        """Make the caller's stream wait for the NMS of slot k (all slots when None)."""
        if k is None or k == self.pending or (k is not None and k in self._group):
            self.flush()
        main = torch.cuda.current_stream(self.eng.device)
        for j in range(self.depth) if k is None else (k,):
            if self.used[j]:
                self.check_posted(j)
                main.wait_event(self.nms_done[j])

    def results(self, k: int):
        if k == self.pending or k in self._group:
            self.flush()
        self.check_posted(k)
        self.nms_done[k].synchronize()
        return self.nms[k].results()
