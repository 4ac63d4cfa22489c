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


class _StubPredictor:
    """Host stand-in for predict.Predictor (no GPU here): per image a deterministic function of the image's pixels
    -> (k, 6) rows and k anchor indices, k = 1 + (first pixel % 4); `stream` keeps Predictor's contract (one
    (dets, keep) pair of per-image lists per batch, in order)."""

    def __init__(self, batch):
        self.batch = batch

    @staticmethod
    def one(im):
        t = torch.from_numpy(im.astype("float32"))
        k = 1 + int(im.flat[0]) % 4
        d = torch.stack([t.mean() + j + torch.arange(6, dtype=torch.float32) for j in range(k)])
        return d, torch.arange(k, dtype=torch.int64) * 7 + int(im.flat[1])

    def stream(self, batches, return_idxs=True):
        for b in batches:
            assert 0 < len(b) <= self.batch
            r = [self.one(im) for im in b]
            yield [x[0] for x in r], [x[1] for x in r]

    def close(self):
        pass


def _host_batches(total, nb):
    import numpy as np

    rng = np.random.default_rng(5)
    return [[rng.integers(0, 256, (6 + i % 3, 5 + i % 2, 3), dtype=np.uint8) for i in range(total)] for _ in range(nb)]


def _host_worker(rank, world, port, q, total, bs):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fce_yolo_amd.dist import ShardedHostPredictor

        sp = ShardedHostPredictor(None, total, 640, "cpu", batch_size=bs, predictor=_StubPredictor)
        batches = _host_batches(total, 3)
        # rank 0 is handed whole global batches, rank 1 only its own shards ("each rank loads its own shard")
        feed = batches if rank == 0 else [b[sp.start:sp.end] for b in batches]
        out = [([d.tolist() for d in ds], [k.tolist() for k in ks]) for ds, ks in sp.stream(feed)]
        q.put((rank, (sp.start, sp.end), out))
        sp.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total,bs", [(7, 4), (6, 32)])
def test_sharded_host_predictor_matches_one_rank_gloo_world2(total, bs):
    """dist.ShardedHostPredictor over two gloo ranks: each rank predicts only its contiguous shard (uneven at 7
    images), and the all-gathered per-image results equal one predictor over every whole batch, in order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_worker, args=(r, 2, port, q, total, bs)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    one = _StubPredictor(total)
    want = []
    for b in _host_batches(total, 3):
        ds, ks = next(one.stream([b]))
        want.append(([d.tolist() for d in ds], [k.tolist() for k in ks]))
    (r0, rng0, out0), (r1, rng1, out1) = res
    assert rng0 == shard_range(total, 2, 0, bs) and rng1 == shard_range(total, 2, 1, bs)
    assert out0 == want and out1 == want
