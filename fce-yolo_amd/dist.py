"""Multi-GPU batch sharding for inference: one process per GPU, images are independent.

* `shard_range` restates the reference's `ContiguousDistributedSampler._get_rank_indices`
  (ultralytics/data/build.py:115-215): contiguous batch-aligned chunks, the remainder batches to the
  lowest ranks, and a batch size >= the dataset degenerating to batch size 1.
* `broadcast_module` sends rank 0's weights to every rank once per model load (RCCL over xGMI on the
  GPU box, gloo on CPU).
* `gather_detections` collects every rank's post-NMS detections on all ranks (outside the timed loop).
No collective is on the per-step data path: the bench scales weakly.
"""

from __future__ import annotations

import math

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
