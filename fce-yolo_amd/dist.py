"""Multi-GPU batch sharding for inference: one process per GPU, images are independent.

* `shard_range` restates the reference's `ContiguousDistributedSampler._get_rank_indices`
  (ultralytics/data/build.py:115-215): contiguous batch-aligned chunks, the remainder batches to the
  lowest ranks, and a batch size >= the dataset degenerating to batch size 1.
* `broadcast_module` sends rank 0's weights to every rank once per model load (RCCL over xGMI on the
  GPU box, gloo on CPU).
* `DeviceGather` is the per-batch collective of both sharded predictors: one packed all-gather of the NMS
  outputs on a side stream (RCCL over xGMI), issued in batch order.
* `gather_detections` collects every rank's post-NMS detections on all ranks (variable sizes, host sync).
* `ShardedPredictor` is the per-step multi-GPU entry point (`bench.py --gpus N`): rank r runs its
  contiguous shard of each global batch through Engine + Pipeline, and the packed post-NMS outputs of
  every rank are all-gathered (one RCCL collective per batch, ~0.3 MB per rank at bs 32) on the NMS side
  stream, overlapped with the next batch's forward -- the reference's ``gather_object`` of validation
  results to rank 0 (models/yolo/detect/val.py:222-241), without a host round trip.  Per-image results
  come back in the unsharded order (`unpack_gathered`).
Images never cross GPUs; the gather is the only per-step collective and the bench scales weakly.
"""

from __future__ import annotations

import math
import os

import torch
import torch.distributed as dist


def shard_range(total: int, world: int, rank: int, batch_size: int) -> tuple[int, int]:
    """[start, end) sample indices of `rank` (data/build.py:168-186)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    if total <= 0:
        return 0, 0
    bs = 1 if batch_size >= total else batch_size
    num_batches = math.ceil(total / bs)
    base, rem = divmod(num_batches, world)
    mine = base + (1 if rank < rem else 0)
    start_batch = rank * base + min(rank, rem)
    return start_batch * bs, min((start_batch + mine) * bs, total)


@torch.no_grad()
def broadcast_module(module: torch.nn.Module, src: int = 0) -> None:
    """Every parameter and buffer of `module` := rank `src`'s (same architecture on all ranks).

    Bucketed: the tensors of each dtype are flattened into one buffer and sent with ONE broadcast
    (a few large collectives over xGMI instead of one per tensor), then copied back."""
    tensors = [t.data for t in list(module.parameters()) + list(module.buffers())]
    by_dtype: dict = {}
    for t in tensors:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    for ts in by_dtype.values():
        flat = torch.cat([t.reshape(-1) for t in ts])
        dist.broadcast(flat, src=src)
        off = 0
        for t in ts:
            n = t.numel()
            t.copy_(flat[off:off + n].view_as(t))
            off += n


def gather_detections(dets: torch.Tensor, keep: torch.Tensor, counts: torch.Tensor):
    """All ranks' (dets (b,max_det,6), keep (b,max_det), counts (b,)) -> per-image lists in rank order.

    Shards may differ in size by one batch (remainder rule); they are padded to the largest shard.
    """
    world = dist.get_world_size()
    b = torch.tensor([dets.shape[0]], dtype=torch.int64, device=dets.device)
    sizes = [torch.zeros_like(b) for _ in range(world)]
    dist.all_gather(sizes, b)
    bmax = int(max(int(s.item()) for s in sizes))

    def pad(t):
        if t.shape[0] == bmax:
            return t.contiguous()
        out = torch.zeros((bmax,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        out[: t.shape[0]] = t
        return out

    outs = []
    for t in (dets, keep, counts):
        p = pad(t)
        bufs = [torch.empty_like(p) for _ in range(world)]
        dist.all_gather(bufs, p)
        outs.append(bufs)
    res_d, res_k = [], []
    for r in range(world):
        n = int(sizes[r].item())
        cnt = outs[2][r][:n].tolist()
        res_d += [outs[0][r][i, : cnt[i]] for i in range(n)]
        res_k += [outs[1][r][i, : cnt[i]] for i in range(n)]
    return res_d, res_k


def shard_sizes(total: int, world: int, batch_size: int) -> list[int]:
    """Images of every rank under `shard_range`."""
    return [e - s for s, e in (shard_range(total, world, r, batch_size) for r in range(world))]


def unpack_gathered(gathered: torch.Tensor, sizes: list[int], max_det: int):
    """All ranks' packed NMS outputs (``engine.NMS`` layout, each padded to max(sizes) images, rank order)
    -> (dets, keep) per image in the unsharded order: rank r's images are global images
    [sum(sizes[:r]), sum(sizes[:r+1]))."""
    from .engine import NMS

    bmax = max(sizes)
    nb = NMS.packed_bytes(bmax, max_det)
    blocks = gathered.view(len(sizes), nb)
    dets, keep = [], []
    for r, n in enumerate(sizes):
        k, d, c = NMS.unpack(blocks[r], bmax, max_det)
        cnt = c[:n].tolist()
        dets += [d[i, : cnt[i]] for i in range(n)]
        keep += [k[i, : cnt[i]] for i in range(n)]
    return dets, keep


class DeviceGather:
    """One packed all-gather of a batch's NMS outputs (``engine.NMS`` layout: keep | dets | counts) per batch, on the
    device: every rank sends its shard padded to the largest shard's layout (a remainder shard is re-packed into
    a per-slot send buffer), RCCL's ``all_gather_into_tensor`` writes the ranks' blocks in rank order, and
    ``unpack`` cuts the host copy into per-image results in the unsharded order.  The caller issues it on one
    side stream in batch order, so every rank's collectives come in the same order (the reference gathers
    validation results to rank 0 with gather_object, models/yolo/detect/val.py:222-241, through the host).
    With gloo (CPU rehearsals of the GPU path) the send block goes through host memory."""

    def __init__(self, sizes: list[int], rank: int, max_det: int):
        from .engine import NMS

        self.sizes, self.rank, self.max_det = list(sizes), rank, max_det
        self.world, self.batch, self.bmax = len(sizes), sizes[rank], max(sizes)
        self.nb = NMS.packed_bytes(self.bmax, max_det)
        self.nbytes = self.world * self.nb  # gathered bytes per batch
        self.nccl = dist.get_backend() == "nccl"

    def buffers(self, device):
        """(send or None, gathered) device buffers for one in-flight slot."""
        send = torch.zeros(self.nb, dtype=torch.uint8, device=device) if self.batch < self.bmax else None
        return send, torch.zeros(self.nbytes, dtype=torch.uint8, device=device)

    def issue_block(self, src: torch.Tensor, gathered: torch.Tensor):
        """All-gather a contiguous block of m slots' outputs (m * nb bytes, each slot already in the bmax layout)
        into gathered[: world * m * nb] ([rank][slot] order) on the current stream: one collective."""
        dst = gathered[: self.world * src.numel()]
        if self.nccl or src.device.type == "cpu":
            dist.all_gather_into_tensor(dst, src)
        else:
            out = torch.empty(dst.numel(), dtype=torch.uint8)
            dist.all_gather_into_tensor(out, src.cpu())
            dst.copy_(out)

    def unpack_block(self, gathered: torch.Tensor, m: int, j: int):
        """Slot j of an m-slot block gathered by issue_block -> per-image (dets, keep) in the unsharded order."""
        blocks = gathered[: self.world * m * self.nb].view(self.world, m, self.nb)[:, j]
        return unpack_gathered(blocks.reshape(-1), self.sizes, self.max_det)

    def issue(self, nms, send, gathered):
        """Gather slot `nms`'s outputs into `gathered` on the current stream."""
        from .engine import NMS

        src = nms.buf
        if send is not None:  # a remainder shard: re-pack into the bmax layout every rank sends
            keep, dets, counts = NMS.unpack(send, self.bmax, self.max_det)
            keep[: self.batch].copy_(nms.keep)
            dets[: self.batch].copy_(nms.dets)
            counts[: self.batch].copy_(nms.counts)
            src = send
        if self.nccl or src.device.type == "cpu":
            dist.all_gather_into_tensor(gathered, src)
        else:
            out = torch.empty(self.nbytes, dtype=torch.uint8)
            dist.all_gather_into_tensor(out, src.cpu())
            gathered.copy_(out)

    def unpack(self, host: torch.Tensor):
        return unpack_gathered(host, self.sizes, self.max_det)


class ShardedPredictor:
    """Batch-sharded detection inference, one process per GPU.

    A global batch of `total` images is split by `shard_range` (reference ContiguousDistributedSampler,
    data/build.py:115-215; l256 on 8 GPUs = 8 x 32).  `submit(x)` takes this rank's shard, runs forward
    + NMS through `engine.Pipeline`, and all-gathers the packed NMS outputs of every rank on the NMS side
    stream (``dist.all_gather_into_tensor``; RCCL over xGMI on the GPU box), so the gather of batch i
    overlaps the forward of batch i+1.  `results(k)` unpacks slot k in the unsharded image order."""

    def __init__(self, model, total: int, imgsz, device, batch_size: int | None = None, depth: int = 2,
                 lanes: int = 1, gather: bool | None = None, **nms_kw):
        """`gather` (default: world > 1) forces the collective path; with one rank it rehearses the RCCL
        all-gather on the side stream (bench.py, FCE_DIST_FORCE=1)."""
        from .engine import NMS, Engine, Pipeline

        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.do_gather = self.world > 1 if gather is None else bool(gather) and dist.is_initialized()
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        bs = batch_size or -(-total // self.world)
        self.sizes = shard_sizes(total, self.world, bs)
        self.start, self.end = shard_range(total, self.world, self.rank, bs)
        self.batch = self.end - self.start
        if min(self.sizes) <= 0:  # decided from sizes every rank computes alike: all ranks raise, none hangs
            raise ValueError(f"empty shard(s) {self.sizes} of a {total}-image batch over {self.world} ranks "
                             f"(batch_size {bs}): every rank needs at least one image")
        self.bmax = max(self.sizes)
        self.engine = Engine(model, self.batch, imgsz, device)
        self.max_det = nms_kw.get("max_det", 300)
        lanes = max(1, int(lanes))
        # every rank's NMS outputs are laid out for bmax images (the remainder shards' rows padded), and with lanes
        # one all-gather covers `lanes` consecutive batches (the Pipeline's post groups: one contiguous block)
        self.gather = DeviceGather(self.sizes, self.rank, self.max_det) if self.do_gather else None
        G = lanes if (self.do_gather and lanes > 1) else 1
        self.pipe = Pipeline(self.engine, depth, post=self._gather if self.do_gather else None, lanes=lanes,
                             post_every=G, layout_batch=self.bmax, **nms_kw)
        self.G = self.pipe.G
        # one gathered buffer per group of slots (world x G slots)
        self.gathered = ([torch.zeros(self.world * self.G * self.pipe.nb, dtype=torch.uint8, device=device)
                          for _ in range(self.pipe.depth // self.G)] if self.do_gather else [])

    def _gather(self, k0: int, m: int):
        nb = self.pipe.nb
        self.gather.issue_block(self.pipe.outbuf[k0 * nb:(k0 + m) * nb], self.gathered[k0 // self.G])

    def submit(self, x: torch.Tensor) -> int:
        if x.shape[0] != self.batch:
            raise ValueError(f"rank {self.rank}: shard of {self.batch} images expected, got {x.shape[0]}")
        return self.pipe.submit(x)

    def flush(self):
        """Issue the last pending NMS (+ gather); call before timing / synchronising on a batch's results."""
        self.pipe.flush()

    def results(self, k: int):
        """(dets, keep) per image of the whole global batch, in the unsharded order (with gather=False: this
        rank's shard only)."""
        if k == self.pipe.pending or k in self.pipe._group:  # Pipeline.results' condition: post the slot's group
            self.pipe.flush()
        self.pipe.check_posted(k)
        self.pipe.nms_done[k].synchronize()
        if self.do_gather:
            k0, m = self.pipe.group_of(k)
            return self.gather.unpack_block(self.gathered[k0 // self.G], m, k - k0)
        # no collective: this rank's own images only (its shard, in order; the slot laid out for bmax images)
        nms = self.pipe.nms[k]
        cnt = nms.counts.tolist()
        return [nms.dets[i, : cnt[i]] for i in range(self.batch)], [nms.keep[i, : cnt[i]] for i in range(self.batch)]

    def close(self):
        self.pipe.close()  # flushes, then stops the poster
        torch.cuda.synchronize(self.engine.device)
        for e in self.pipe.engs:
            e.close()


def pack_detections(dets, keep, bmax: int, max_det: int):
    """Per-image (k, 6) detections + kept anchor indices -> (counts (bmax,), dets (bmax, max_det, 6) f32,
    keep (bmax, max_det) int64), zero padded: the fixed-size form every rank sends in a gather."""
    counts = torch.zeros(bmax, dtype=torch.int64)
    d = torch.zeros((bmax, max_det, 6), dtype=torch.float32)
    k = torch.zeros((bmax, max_det), dtype=torch.int64)
    for i, (di, ki) in enumerate(zip(dets, keep)):
        n = int(di.shape[0])
        counts[i] = n
        d[i, :n] = di.to("cpu", torch.float32)
        k[i, :n] = ki.to("cpu", torch.int64)
    return counts, d, k


class ShardedHostPredictor:
    """The host-image predict path sharded over ranks ("each rank loads its own shard").

    Rank r takes its contiguous shard (`shard_range`, the reference's ContiguousDistributedSampler rule,
    data/build.py:115-215) of every global batch of decoded uint8 HWC BGR images and runs it through
    `predict.Predictor` (pinned staging -> one H2D -> device letterbox -> forward -> NMS -> scale_boxes, several
    batches in flight; the reference's predictor.py:151-182 preprocess + inference + postprocess).  The per-image
    detections of every rank are all-gathered once per batch (fixed-size packed tensors: RCCL over xGMI on the
    device for the nccl backend, host tensors for gloo), so `stream` yields each global batch's results in the
    unsharded image order on every rank -- what one Predictor over the whole batch returns.  Images never cross
    GPUs; only ~7 KB of detections per image do.

    With the real Predictor the gather is device-side and asynchronous (`DeviceGather`): each batch's packed NMS
    outputs are all-gathered on the predictor's side stream, in batch order, right behind the batch's scale_boxes,
    and the ONE D2H copy of the batch brings the gathered block back, so the submit loop never waits on a
    collective.  A custom `predictor` (tests' host stubs) gets the host gather of its per-image results."""

    def __init__(self, model, total: int, imgsz, device, batch_size: int | None = None, lanes: int | None = None,
                 gather: bool | None = None, predictor=None, max_det: int = 300, **kw):
        """`predictor(batch)` builds the per-rank predictor (default: predict.Predictor(model, batch, imgsz,
        device, lanes=lanes, max_det=max_det, **kw)); anything with `stream(batches, return_idxs=True)` and
        `close()` fits (tests use a host stub)."""
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.do_gather = self.world > 1 if gather is None else bool(gather) and dist.is_initialized()
        bs = batch_size or -(-total // self.world)
        self.total = total
        self.sizes = shard_sizes(total, self.world, bs)
        self.start, self.end = shard_range(total, self.world, self.rank, bs)
        self.batch = self.end - self.start
        if min(self.sizes) <= 0:  # decided from sizes every rank computes alike: all ranks raise, none hangs
            raise ValueError(f"empty shard(s) {self.sizes} of a {total}-image batch over {self.world} ranks")
        self.bmax = max(self.sizes)
        self.max_det = max_det
        # FCE_HOST_GATHER=1: the per-image host gather for the real predictor too (A/B diagnostics)
        self.device_gather = predictor is None and self.do_gather and os.environ.get("FCE_HOST_GATHER") != "1"
        if predictor is None:
            from .predict import Predictor

            g = DeviceGather(self.sizes, self.rank, max_det) if self.device_gather else None
            self.pred = Predictor(model, self.batch, imgsz, device, lanes=lanes, max_det=max_det, gather=g, **kw)
        else:
            self.pred = predictor(self.batch)
        backend = dist.get_backend() if dist.is_initialized() else "gloo"
        self.comm_device = torch.device(device) if backend == "nccl" else torch.device("cpu")

    def shard(self, images):
        """This rank's images of a global batch (a full batch of `total` images, or already just the shard)."""
        if len(images) == self.batch and self.total != self.batch:
            return list(images)
        if len(images) != self.total:
            raise ValueError(f"rank {self.rank}: a global batch of {self.total} images (or its {self.batch}-image "
                             f"shard) expected, got {len(images)}")
        return list(images[self.start:self.end])

    def _gather(self, dets, keep):
        if not self.do_gather or self.device_gather:
            return dets, keep
        packed = [t.to(self.comm_device) for t in pack_detections(dets, keep, self.bmax, self.max_det)]
        outs = []
        for t in packed:
            bufs = [torch.empty_like(t) for _ in range(self.world)]
            dist.all_gather(bufs, t)
            outs.append([b.cpu() for b in bufs])
        res_d, res_k = [], []
        for r, n in enumerate(self.sizes):
            cnt = outs[0][r][:n].tolist()
            res_d += [outs[1][r][i, :cnt[i]] for i in range(n)]
            res_k += [outs[2][r][i, :cnt[i]] for i in range(n)]
        return res_d, res_k

    def stream(self, batches):
        """Per global batch, (dets, keep) per image of the whole batch in the unsharded order.  Every rank must
        be given the same number of batches (the gather is collective)."""
        for dets, keep in self.pred.stream((self.shard(b) for b in batches), return_idxs=True):
            yield self._gather(dets, keep)

    def close(self):
        self.pred.close()
