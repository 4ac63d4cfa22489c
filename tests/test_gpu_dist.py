"""GPU, two processes: the sharded host-image predict path (dist.ShardedHostPredictor) with the real
predict.Predictor on each rank, both ranks on cuda:0 over gloo (the one-GPU box rehearsal of the multi-GPU path;
RCCL replaces gloo on an 8-GPU node), against one Predictor over the whole batches."""

import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fce_pkg  # noqa: E402  (spawned workers import this module fresh)

fce_pkg.load()

pytestmark = pytest.mark.gpu
TOTAL, BS, S = 7, 4, 256


def _model():
    from fce_yolo_amd.parser import DetectionModel
    from fce_yolo_amd.weights import seeded_state_dict

    m = DetectionModel("yolo11n-fce.yaml")
    m.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in m.state_dict().items()], 0, gain=1.45))
    return m.eval().to("cuda:0")


def _batches(nb=3):
    rng = np.random.default_rng(11)
    return [[rng.integers(0, 256, (200 + 17 * i, 300 - 9 * i, 3), dtype=np.uint8) for i in range(TOTAL)]
            for _ in range(nb)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fce_yolo_amd.dist import ShardedHostPredictor

        torch.cuda.set_device(0)
        sp = ShardedHostPredictor(_model(), TOTAL, S, "cuda:0", batch_size=BS, lanes=2, conf=0.05)
        out = [([d.numpy() for d in ds], [k.numpy() for k in ks]) for ds, ks in sp.stream(_batches())]
        q.put((rank, out))
        sp.close()
    finally:
        dist.destroy_process_group()


def test_sharded_host_predictor_two_ranks_match_one_predictor():
    from fce_yolo_amd.predict import Predictor

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    import queue
    import time

    res, t0 = [], time.time()
    while len(res) < len(procs):  # a rank that dies fails the test at once instead of leaving the others waiting
        try:
            res.append(q.get(timeout=2))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead and time.time() - t0 < 100, f"rank exit codes {[p.exitcode for p in procs]}"
    res.sort(key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pred = Predictor(_model(), TOTAL, S, "cuda:0", lanes=2, conf=0.05)
    want = list(pred.stream(_batches(), return_idxs=True))
    pred.close()
    assert sum(len(d) for ds, _ in want for d in ds) > 0  # the seeded head keeps some boxes
    for rank, out in res:
        assert len(out) == len(want)
        for (ds, ks), (wd, wk) in zip(out, want):
            assert len(ds) == TOTAL
            for d, k, d1, k1 in zip(ds, ks, wd, wk):
                assert np.array_equal(k, k1.numpy()), rank
                assert np.array_equal(d, d1.numpy()), rank


def _worker_resident(rank, world, port, q):
    """dist.ShardedPredictor over gloo with both ranks on cuda:0: grouped all-gathers (lanes 2 -> one collective per
    two batches, a partial group at flush), remainder shard in the largest shard's layout."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fce_yolo_amd.dist import ShardedPredictor

        torch.cuda.set_device(0)
        sp = ShardedPredictor(_model(), TOTAL, S, "cuda:0", batch_size=BS, lanes=2, gather=True, conf=0.05)
        assert sp.G == 2 and sp.bmax == BS
        xs = _resident_inputs()
        slots = [sp.submit(x[sp.start:sp.end].half().to("cuda:0")) for x in xs]
        sp.flush()
        out = []
        for k in slots[-sp.pipe.depth:]:
            ds, ks = sp.results(k)
            out.append(([d.cpu().numpy() for d in ds], [kk.cpu().numpy() for kk in ks]))
        q.put((rank, out))
        sp.close()
    finally:
        dist.destroy_process_group()


def _worker_midflush(rank, world, port, q):
    """dist.ShardedPredictor with lanes 3 (post groups of 3 aligned slot blocks, depth 6) and results read MID-STREAM:
    after batches 1 and 4 every batch submitted so far is read (results() flushes a partial group), then more batches
    are submitted into the rest of the flushed block; every batch's results are checked (a flushed partial
    group used to shift later groups across block boundaries, so some slots were never gathered)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fce_yolo_amd.dist import ShardedPredictor

        torch.cuda.set_device(0)
        sp = ShardedPredictor(_model(), TOTAL, S, "cuda:0", batch_size=BS, lanes=3, gather=True, conf=0.05)
        assert sp.G == 3 and sp.pipe.depth == 6
        xs = _resident_inputs(9)
        out, unread = [None] * len(xs), []
        for j, x in enumerate(xs):
            unread.append((j, sp.submit(x[sp.start:sp.end].half().to("cuda:0"))))
            if j in (1, 4) or j == len(xs) - 1:
                if j == len(xs) - 1:
                    sp.flush()
                for jj, k in unread:
                    ds, ks = sp.results(k)
                    out[jj] = ([d.cpu().numpy() for d in ds], [kk.cpu().numpy() for kk in ks])
                unread = []
        q.put((rank, out))
        sp.close()
    finally:
        dist.destroy_process_group()


def _resident_inputs(nb=5):
    g = torch.Generator().manual_seed(21)
    return [torch.rand(TOTAL, 3, S, S, generator=g) for _ in range(nb)]


def _run_ranks(worker):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    import queue
    import time

    res, t0 = [], time.time()
    while len(res) < len(procs):
        try:
            res.append(q.get(timeout=2))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead and time.time() - t0 < 100, f"rank exit codes {[p.exitcode for p in procs]}"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda t: t[0])
    return res


def _reference(model, xs, bounds):
    """per batch, per image (dets, keep) from one executor per [lo, hi) range of the batch"""
    from fce_yolo_amd.engine import NMS, Engine

    out = [([], []) for _ in xs]
    for lo, hi in bounds:
        eng = Engine(model, hi - lo, S, "cuda:0")
        nms = NMS(hi - lo, eng.anchors, eng.nc, "cuda:0", conf=0.05)
        for j, x in enumerate(xs):
            dets, keep, counts = nms(eng(x[lo:hi].half().to("cuda:0")).clone())
            c = counts.tolist()
            out[j][0].extend(dets[i, :c[i]].cpu().numpy() for i in range(hi - lo))
            out[j][1].extend(keep[i, :c[i]].cpu().numpy() for i in range(hi - lo))
        eng.close()
    return out


def _diff(out, want):
    return [(j, i) for j, ((ds, ks), (wd, wk)) in enumerate(zip(out, want)) for i, (d, k, d1, k1) in
            enumerate(zip(ds, ks, wd, wk)) if not (np.array_equal(k, k1) and np.array_equal(d, d1))]


def test_sharded_predictor_grouped_gather_two_ranks_match_one_engine():
    """Every rank gets every image's detections, bit-equal to one executor + NMS over the whole batch of 7."""
    res = _run_ranks(_worker_resident)
    model = _model()
    xs = _resident_inputs()
    per_shard = _reference(model, xs, [(0, BS), (BS, TOTAL)])[-len(res[0][1]):]  # what the gather must deliver
    assert sum(len(d) for ds, _ in per_shard for d in ds) > 0
    for rank, out in res:
        assert len(out) == len(per_shard) and all(len(ds) == TOTAL for ds, _ in out)
        assert not _diff(out, per_shard), (rank, _diff(out, per_shard))
    whole = _reference(model, xs, [(0, TOTAL)])[-len(res[0][1]):]  # one executor over all 7 images
    assert not _diff(res[0][1], whole), _diff(res[0][1], whole)


def test_sharded_predictor_results_mid_stream_two_ranks():
    """Results read mid-stream (partial post groups flushed, then more batches into the same slot blocks): every one of
    the nine batches bit-equal to the shards' own executors, on both ranks."""
    res = _run_ranks(_worker_midflush)
    per_shard = _reference(_model(), _resident_inputs(9), [(0, BS), (BS, TOTAL)])
    assert sum(len(d) for ds, _ in per_shard for d in ds) > 0
    for rank, out in res:
        assert len(out) == len(per_shard) and all(o is not None and len(o[0]) == TOTAL for o in out)
        assert not _diff(out, per_shard), (rank, _diff(out, per_shard))
