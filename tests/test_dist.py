"""CPU (gloo, world size 2): the multi-GPU path's sharding rule, weight broadcast and detection gather."""

import os
import socket
import sys
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402  (spawned workers import this module fresh)

fce_pkg.load()
from fce_yolo_amd.dist import broadcast_module, gather_detections, shard_range, shard_sizes, unpack_gathered  # noqa: E402
from fce_yolo_amd.engine import NMS  # noqa: E402


def _ref_rule(total, world, rank, bs):
    """ContiguousDistributedSampler (data/build.py:115-215), written out independently."""
    bs = 1 if bs >= total else bs
    nb = -(-total // bs)
    per = [nb // world + (1 if r < nb % world else 0) for r in range(world)]
    start = sum(per[:rank])
    return start * bs, min((start + per[rank]) * bs, total)


@pytest.mark.parametrize("total,world,bs", [(256, 8, 32), (250, 8, 32), (7, 2, 32), (1000, 3, 16), (33, 4, 1)])
def test_shard_range_matches_reference_rule(total, world, bs):
    got = [shard_range(total, world, r, bs) for r in range(world)]
    assert got == [_ref_rule(total, world, r, bs) for r in range(world)]
    covered = [i for s, e in got for i in range(s, e)]
    assert covered == list(range(total))  # contiguous, disjoint, complete


def test_l256_eight_way_is_eight_by_32():
    assert [shard_range(256, 8, r, 32) for r in range(8)] == [(32 * r, 32 * r + 32) for r in range(8)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fce_yolo_amd.parser import DetectionModel

        torch.manual_seed(100 + rank)  # different init per rank
        m = DetectionModel("yolo11n-fce.yaml")
        broadcast_module(m)
        digest = float(sum(p.double().sum() for p in m.state_dict().values() if p.is_floating_point()))
        # uneven shards: rank 0 has 3 images, rank 1 has 2
        b = 3 if rank == 0 else 2
        dets = torch.full((b, 5, 6), float(rank))
        keep = torch.arange(b * 5, dtype=torch.int64).reshape(b, 5) + 100 * rank
        counts = torch.tensor([1 + i for i in range(b)], dtype=torch.int32)
        d, k = gather_detections(dets, keep, counts)
        q.put((rank, digest, [tuple(t.shape) for t in d], [t.tolist() for t in k]))
    finally:
        dist.destroy_process_group()


def test_broadcast_and_gather_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, d0, s0, k0), (_, d1, s1, k1) = res
    assert d0 == d1  # rank 1 now holds rank 0's weights
    assert s0 == s1 == [(1, 6), (2, 6), (3, 6), (1, 6), (2, 6)]
    assert k0 == k1 == [[0], [5, 6], [10, 11, 12], [100], [105, 106]]


def _packed_shard(rank, n, bmax, max_det, first):
    """This rank's NMS outputs in the packed engine.NMS layout (padded to bmax images); image i of the
    global batch keeps 1 + i % 4 boxes whose anchor indices encode (image, j)."""
    buf = torch.zeros(NMS.packed_bytes(bmax, max_det), dtype=torch.uint8)
    keep, dets, counts = NMS.unpack(buf, bmax, max_det)
    for i in range(n):
        g = first + i
        c = 1 + g % 4
        counts[i] = c
        keep[i, :c] = torch.arange(c) + 1000 * g
        dets[i, :c] = float(g)
    return buf


def _sharded_worker(rank, world, port, q, total, bs, max_det):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sizes = shard_sizes(total, world, bs)
        s, e = shard_range(total, world, rank, bs)
        buf = _packed_shard(rank, e - s, max(sizes), max_det, s)
        out = torch.empty(world * buf.numel(), dtype=torch.uint8)
        dist.all_gather_into_tensor(out, buf)  # the ShardedPredictor collective
        dets, keep = unpack_gathered(out, sizes, max_det)
        q.put((rank, [k.tolist() for k in keep], [float(d[0, 0]) if len(d) else None for d in dets]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total,bs", [(7, 2), (5, 3), (8, 4)])
def test_sharded_gather_restores_unsharded_order_gloo_world2(total, bs):
    """Uneven (remainder-rule) shards: the gathered per-image results come back in the global order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, 2, port, q, total, bs, 6)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [[1000 * g + j for j in range(1 + g % 4)] for g in range(total)]
    for _, keep, first in res:
        assert keep == want
        assert first == [float(g) for g in range(total)]


def _empty_shard_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fce_yolo_amd.dist import ShardedPredictor

        try:  # 1 image over 2 ranks: rank 1's shard is empty; BOTH ranks must refuse (no one reaches a collective)
            ShardedPredictor(None, 1, 320, "cpu", batch_size=1)
            q.put((rank, "no error"))
        except ValueError as e:
            q.put((rank, "ValueError" if "empty shard" in str(e) else str(e)))
    finally:
        dist.destroy_process_group()


def test_sharded_predictor_empty_shard_raises_on_every_rank_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_empty_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(0, "ValueError"), (1, "ValueError")]
