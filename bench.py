"""Benchmark: FCE-YOLOv11 detection inference (forward + decode + NMS) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model yolo11n-fce.yaml] [--batch 32] [--imgsz 640]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

`python bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment) launches the N ranks itself: before
torch is even imported, it runs the torch.distributed.run command above as a child process (one rank per
GPU, 127.0.0.1, a free port) and exits with its status -- the reference's trainer does the same with its
generated DDP command (engine/trainer.py:233-236, utils/dist.py:77-104).  The parent never touches the GPU.
A rank whose WORLD_SIZE differs from --gpus fails with a non-zero status.

A step = one global batch of B images per GPU through `dist.ShardedPredictor`: each rank's contiguous
shard (reference ContiguousDistributedSampler rule) of resident synthetic input (torch.rand fp16, seeded
per rank) runs the whole forward (a captured hipGraph replayed per lane; --graph 0 for direct launches) + the device NMS, and
with N > 1 the packed detections of every rank are all-gathered (one RCCL collective per batch).  By
default four batches are in flight per GPU on the n and s scales with one GPU and three otherwise (--lanes,
engine.Pipeline lanes): executors with their own arenas on their own streams, each running forward then NMS of every L-th batch, so one batch's
latency-bound coarse layers and NMS share the CUs with the next batches' full-width layers; the gather
runs on a side stream in batch order.  With four lanes the process asks HIP for 8 hardware queues
(GPU_MAX_HW_QUEUES, set before torch is imported; HIP's default 4 is shared by the lanes, the side stream and
the default stream): 4 lanes x 8 queues 29.3-29.6k against 28.7-28.8k images/s for 3 lanes x 4 queues,
interleaved on one box (profiles/r03w_lanes_queues.txt).  --lanes 1 keeps one executor (the NMS of batch i on a side stream
under the forward of batch i+1); --sequential runs forward and NMS back to back.  Weights are the portable seeded weights of the named
architecture (no checkpoints offline), broadcast from rank 0 over RCCL.  Per-GPU work is fixed as N
grows: scaling is weak.  Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time
from collections import defaultdict
from pathlib import Path


def launch_command(argv, env):
    """The torch.distributed.run command that starts `--gpus N` ranks of this script, or None when this
    process is already a rank (WORLD_SIZE set) or N == 1.  Pure: no torch import, no GPU call."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    a, _ = pre.parse_known_args(argv)
    if a.gpus <= 1 or "WORLD_SIZE" in env:
        return None
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *argv]


def default_lanes(model: str, env, gpus: int = 1) -> int:
    """Batches in flight per GPU when --lanes is not given: FCE_LANES, else 4 for the n and s scales (n32 29.3-29.6k
    vs 28.7-28.8k images/s with 3, s32 16.0-16.1k vs 15.8k, profiles/r03w_*) and, since round 4's faster kernels, the
    l scale (l32 5.64-5.65k vs 5.57-5.58k, profiles/r04aq_*); 3 on the m scale, whose four arenas overflow the MALL
    (m16-h8 1.83k vs 1.76k images/s with 4).  The same with or without a process group since round 5: the per-batch
    all-gather used to cost a four-lane step 17 % (a side-stream wait per batch on the device, 29.7-30.1k against
    36.0-36.4k, whatever the collective), so multi-GPU runs kept 3 lanes x 4 queues; the host-ordered poster with one
    collective per `lanes` batches (engine.Poster, dist.ShardedPredictor) measures 36.4-36.7k against 36.4-37.4k
    without a group (profiles/r05w_*)."""
    if env.get("FCE_LANES"):
        return int(env["FCE_LANES"])
    stem = Path(model).stem
    scale = stem[6:7] if stem.startswith("yolo11") else ""
    return 4 if scale in ("n", "s", "l") else 3


def hw_queues_env(argv, env):
    """HIP hardware queues for 4 or more lanes: at least 8 (the lanes' streams, the NMS / gather side stream and
    the default stream would share HIP's default 4).  Returns the value to export, or None to leave the
    environment alone.  Pure: runs before torch is imported (HIP reads it when it initialises)."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--model", default="yolo11n-fce.yaml")
    pre.add_argument("--lanes", type=int, default=None)
    pre.add_argument("--gpus", type=int, default=1)
    a, _ = pre.parse_known_args(argv)
    lanes = a.lanes if a.lanes is not None else default_lanes(a.model, env, a.gpus)
    have = int(env.get("GPU_MAX_HW_QUEUES", "4") or 4)
    return "8" if lanes >= 4 and have < 8 else None


_HWQ_GIVEN = os.environ.get("GPU_MAX_HW_QUEUES")  # as the caller set it (the N=1 line may raise it below)

if __name__ == "__main__":
    _q = hw_queues_env(sys.argv[1:], os.environ)
    if _q is not None:
        os.environ["GPU_MAX_HW_QUEUES"] = _q
    _cmd = launch_command(sys.argv[1:], os.environ)
    if _cmd is not None:  # launcher: start the ranks as a child process (never exec), exit with its status
        if os.environ.get("FCE_BENCH_DRY_LAUNCH") == "1":
            print(json.dumps({"launch": _cmd, "torch_imported": "torch" in sys.modules}), flush=True)
            sys.exit(0)
        import subprocess

        sys.exit(subprocess.call(_cmd))

import torch  # noqa: E402
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
import fce_pkg  # noqa: E402

fce_pkg.load()
from fce_yolo_amd.dist import ShardedPredictor, broadcast_module  # noqa: E402
from fce_yolo_amd.engine import NMS  # noqa: E402
from fce_yolo_amd.parser import DetectionModel, load_cfg  # noqa: E402
from fce_yolo_amd.weights import seeded_state_dict  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
MFMA_F16_PEAK_TFS = 2500.0  # dense fp16 MFMA (no sparsity)
RIDGE = MFMA_F16_PEAK_TFS * 1e12 / (HBM_PEAK_GBS * 1e9)
PROFILES = Path(__file__).resolve().parent / "profiles"


def _trace_marker():
    """One tiny torch spin kernel (never launched by the path itself): rocprofv3 traces are split at
    these dispatches into [setup+warmup | timed steps | forward-only | per-op profile] segments
    (scripts/trace_summary.py, scripts/pmc_summary.py)."""
    torch.cuda._sleep(64)


def pmc_path(model: str, batch: int, imgsz: int) -> Path:
    """The committed rocprofv3 PMC summary of THIS config (scripts/gpu_pmc.sh + pmc_summary.py)."""
    return PROFILES / f"pmc_{Path(model).stem}_b{batch}_s{imgsz}.json"


def _pmc_family(path: Path, family):
    """The PMC summary's per-launch entry for `family` (FETCH_SIZE x2 + WRITE_SIZE with the gfx950
    correction; MFMA counters when that pass was collected), or None."""
    try:
        return json.loads(path.read_text())["families"][family]
    except (OSError, KeyError, ValueError, TypeError):
        return None


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 timed steps (~0.2 s): the pipeline's fill and drain (lanes - 1 batches) are amortised; 50 steps read
    # ~1.2 % lower (profiles/r03ag_steps.txt)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", default="yolo11n-fce.yaml")
    ap.add_argument("--batch", type=int, default=32, help="images per GPU")
    ap.add_argument("--imgsz", type=int, default=640)
    ap.add_argument("--no-nms", action="store_true", help="time the forward only")
    ap.add_argument("--sequential", action="store_true", help="forward then NMS on one stream (no overlap)")
    ap.add_argument("--lanes", type=int, default=None,
                    help="batches in flight per GPU (engine.Pipeline lanes: one executor + stream each; default "
                         "FCE_LANES, else 4 for the n scale and 3 for the others)")
    ap.add_argument("--graph", type=int, default=-1, help="1: replay a captured hipGraph per lane; 0: direct "
                    "launches; -1 (default): replay when lanes > 1 (ties direct launches there, 28.2k both; with one "
                    "lane direct launches are faster, DESIGN.md)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--profile-json", default=None, help="write the per-op profile here")
    ap.add_argument("--profile-passes", type=int, default=10, help="per-op HIP-event passes averaged")
    ap.add_argument("--predict-lanes", type=int, default=None,
                    help="batches in flight in the host-image legs (default predict.default_lanes: 5 on n / s, 3 on m / l)")
    ap.add_argument("--predict-steps", type=int, default=100,
                    help="batches of the host-image predict path timed after the main line (0 = skip; 100: the "
                         "lanes' fill and drain are a few % of the window, 30 read ~25 %% low, profiles/r05aa_*)")
    ap.add_argument("--dist-config-steps", type=int, default=None,
                    help="N=1 only: also time this many steps in a child rank under the configuration `--gpus N` runs "
                         "(a one-rank RCCL process group, its lanes and hardware queues, the per-batch all-gather) -> "
                         "`value_dist_config` (default --steps; 0 = skip)")
    ap.add_argument("--inputs", type=int, default=None,
                    help="distinct resident input batches cycled through the timed steps (default lanes + 1, so no "
                         "lane reads an input another lane has just pulled into the MALL)")
    ap.add_argument("--source", choices=("device", "host"), default="device",
                    help="device (default, the contract line): resident fp16 inputs; host: every rank predicts its "
                         "contiguous shard of decoded uint8 host images (dist.ShardedHostPredictor: H2D, letterbox, "
                         "forward, NMS, scale_boxes, per-batch gather of the detections) -- PCIe inclusive, not `value` "
                         "of the contract line")
    a = ap.parse_args()
    a.lanes_given = a.lanes
    if a.lanes is None:
        a.lanes = default_lanes(a.model, os.environ, a.gpus)
    if a.graph < 0:
        a.graph = 1 if a.lanes > 1 else 0
    if a.dist_config_steps is None:
        a.dist_config_steps = a.steps
    if a.inputs is None:
        a.inputs = a.lanes + 1
    if a.predict_lanes is None:
        stem = Path(a.model).stem
        a.predict_lanes = 5 if (stem[6:7] if stem.startswith("yolo11") else "n") in ("n", "s") else 3
    return a


def model_cfg(name: str):
    """'yolo11m-fce-h8.yaml' = yolo11m-fce with the YAML's BiCoordCrossAtt args [512, 8, 8] (config 4)."""
    stem = Path(name).stem
    if not stem.endswith("-h8"):
        return name
    d = load_cfg(stem[:-3] + ".yaml")
    for row in d["backbone"]:
        if row[2] == "BiCoordCrossAtt":
            row[3] = [512, 8, 8]
    return d


def predict_rate(model, B: int, S: int, dev, steps: int, lanes: int = 3):
    """Whole predict path from HOST images (not `value`): B decoded 480x640 uint8 BGR numpy images per
    step -> H2D copy -> device letterbox -> forward -> NMS -> scale_boxes -> per-image results on host."""
    import numpy as np

    from fce_yolo_amd.predict import Predictor

    pred = Predictor(model, B, S, dev, lanes=lanes, workers=4)
    rng = np.random.default_rng(0)
    batches = [[rng.integers(0, 256, (480, 640, 3), dtype=np.uint8) for _ in range(B)] for _ in range(2)]
    for _ in pred.stream([batches[i % 2] for i in range(2 * lanes)]):
        pass
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    for d in pred.stream(batches[i % 2] for i in range(steps)):
        n += len(d)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    assert n == B * steps
    pred.close()
    return {"images_per_sec": round(B * steps / el, 2), "ms_per_batch": round(el / steps * 1e3, 3),
            "batches_in_flight": lanes,
            "source": f"{B} x 480x640 uint8 BGR host numpy images per batch, packed into pinned staging by 4 host "
                      f"threads, one async H2D per batch on a copy stream, device letterbox to {S}x{S} + forward (hipGraph lane) + NMS + "
                      f"scale_boxes, one async D2H of the detections, per-image results as host tensors; {steps} "
                      f"batches, predict.Predictor.stream"}


def cpu_baseline(model_name: str, imgsz: int, seconds: float, batch: int = 32):
    """The oracle (PyTorch-CPU fp32 restatement of the reference forward) on the host cores, with the
    BASELINE.md §2 protocol's batch (bs=32 on the headline config): one bs=1 warm-up, then whole bs=`batch`
    forwards until `seconds` have passed (at least one), images/s from the median batch time; a bs=1
    rate from the remaining time is reported beside it."""
    import statistics

    from oracle import fce_oracle as O
    from oracle.parse import parse

    cpu_model = DetectionModel(model_cfg(model_name))
    cpu_model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in cpu_model.state_dict().items()], 0))
    layers, save, _ = parse(cpu_model.yaml)
    sd = O.cast_sd(O.fuse_state_dict(cpu_model.state_dict()), torch.float32)
    g = torch.Generator().manual_seed(0)
    x1 = torch.rand(1, 3, imgsz, imgsz, generator=g)
    xb = torch.rand(batch, 3, imgsz, imgsz, generator=g)
    with torch.inference_mode():
        O.forward(layers, save, sd, x1)  # warm-up
        t_start = time.perf_counter()
        times = []
        while not times or (time.perf_counter() - t_start < seconds * 0.75 and len(times) < 5):
            t0 = time.perf_counter()
            O.forward(layers, save, sd, xb)
            times.append(time.perf_counter() - t0)
        n1, t1 = 0, time.perf_counter()
        while time.perf_counter() - t_start < seconds and n1 < 200:
            O.forward(layers, save, sd, x1)
            n1 += 1
        el1 = time.perf_counter() - t1
    med = statistics.median(times)
    return {
        "value": round(batch / med, 3),
        "unit": "images/sec",
        "cores": torch.get_num_threads(),
        "kind": "port",
        "sample": f"oracle fp32 forward of {model_name} @ {imgsz}x{imgsz}, bs={batch}: {len(times)} batch(es), "
        f"median {med:.2f} s/batch (1 bs=1 warm-up), torch {torch.__version__} CPU",
        "bs1_images_per_sec": round(n1 / el1, 3) if n1 else None,
    }


def dist_config_line(a):
    """`value_dist_config`: this N=1 workload timed again in a child process under exactly the configuration
    `bench.py --gpus N` runs for N > 1 -- a one-rank RCCL process group (FCE_DIST_FORCE=1 under torch.distributed.run:
    the weight broadcast, the per-batch packed all-gather on the side stream, max-over-ranks timing) with that
    path's lanes and hardware queues (default_lanes / hw_queues_env decide them in the child as for any rank).  A
    scaling ratio value(N) / (N x value(1)) otherwise folds the configuration change into "scaling" (DESIGN.md
    §Multi-GPU).  The parent has released its lanes first; the child runs alone on the GPU."""
    import subprocess

    env = dict(os.environ, FCE_DIST_FORCE="1")
    if _HWQ_GIVEN is None:
        env.pop("GPU_MAX_HW_QUEUES", None)
    else:
        env["GPU_MAX_HW_QUEUES"] = _HWQ_GIVEN
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), "--gpus", "1",
           "--steps", str(a.dist_config_steps), "--warmup", str(a.warmup), "--model", a.model, "--batch", str(a.batch),
           "--imgsz", str(a.imgsz), "--cpu-seconds", "0", "--predict-steps", "0", "--profile-passes", "1",
           "--dist-config-steps", "0"]
    if a.lanes_given is not None:  # an explicit --lanes is what the --gpus N ranks would run too
        cmd += ["--lanes", str(a.lanes_given)]
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    line = next((ln for ln in reversed(r.stdout.splitlines()) if ln.startswith("{")), None)
    if r.returncode != 0 or line is None:
        return {"error": f"rc {r.returncode}: {r.stderr.strip()[-300:]}"}
    d = json.loads(line)
    c = d["config"]
    return {"value": d["value"], "ms_per_step": d["ms_per_step"], "steps": d["steps"],
            "batches_in_flight": c["batches_in_flight"], "hw_queues": c["hw_queues"],
            "process_group": d["process_group"],
            "note": "N=1 under the --gpus N configuration (one-rank RCCL group, per-batch all-gather); the 1-GPU point "
                    "of a scaling curve compares like with like against this value"}


def host_source_line(a, model, rank, world, use_dist, dev):
    """--source host: the sharded host-image path, one JSON line (PCIe inclusive)."""
    import numpy as np

    from fce_yolo_amd.dist import ShardedHostPredictor

    B, S = a.batch, a.imgsz
    sp = ShardedHostPredictor(model, B * world, S, dev, batch_size=B, lanes=a.predict_lanes, workers=4,
                              gather=use_dist)
    # each rank decodes (synthesises) only its own shard: image i of a global batch is seeded by i
    shard = [np.random.default_rng(i).integers(0, 256, (480, 640, 3), dtype=np.uint8) for i in range(sp.start, sp.end)]

    def run(n):
        k = 0
        for dets, _ in sp.stream(shard for _ in range(n)):
            k += len(dets)
        return k

    run(max(2, a.warmup))
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = run(a.steps)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if use_dist and dist.get_backend() == "nccl":
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elif use_dist:
        t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    assert n == B * world * a.steps
    sp.close()
    stem = Path(a.model).stem
    return {
        "metric": "images/sec/GPU @ 640x640 bs=32, yolo11n-fce; fraction of fp16 MFMA roofline",
        "value": round(B * world * a.steps / el, 2), "unit": "images/sec", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp16",
        "data": "synthetic decoded 480x640 uint8 BGR host images, each rank generating only its own shard",
        "config": {"workload": f"{stem} detection predict from host images (H2D + letterbox + forward + NMS + "
                               f"scale_boxes + gather) @ {S}x{S}, {B} images/GPU", "model": stem,
                   "global_batch": B * world, "imgsz": S, "parallelism": f"dp{world}", "source": "host",
                   "batches_in_flight": a.predict_lanes},
        "note": "PCIe-inclusive host-image path (--source host), not the resident-input contract line",
        "process_group": ({"backend": dist.get_backend(), "world_size": dist.get_world_size()} if use_dist
                          else None),
    }


def main():
    a = parse_args()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE {world}: one rank per GPU "
                         f"(run `python bench.py --gpus {a.gpus}` or torch.distributed.run --nproc-per-node {a.gpus})")
    backend = os.environ.get("FCE_DIST_BACKEND", "nccl")  # nccl = RCCL; gloo only for rehearsals
    # FCE_DIST_FORCE=1 (rehearsal, under torch.distributed.run): the process group, the weight broadcast, the
    # per-batch all-gather and the max-over-ranks timing run even with one rank
    force = os.environ.get("FCE_DIST_FORCE") == "1" and "MASTER_ADDR" in os.environ
    use_dist = world > 1 or force
    ndev = torch.cuda.device_count()
    if local >= ndev:
        if world > 1 and backend == "nccl":
            raise RuntimeError(f"LOCAL_RANK {local} but only {ndev} visible GPU(s): one RCCL rank per GPU")
        local = local % max(1, ndev)  # gloo rehearsal with more ranks than GPUs
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if use_dist:
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
        if dist.get_world_size() != world:
            raise SystemExit(f"bench.py: process group world size {dist.get_world_size()} != WORLD_SIZE {world}")

    model = DetectionModel(model_cfg(a.model))
    if rank == 0:
        model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in model.state_dict().items()], 0))
    model.eval().to(dev)
    if use_dist:  # weights broadcast once per model load (RCCL over xGMI)
        broadcast_module(model, src=0)

    B, S = a.batch, a.imgsz
    if a.source == "host":
        out = host_source_line(a, model, rank, world, use_dist, dev)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if use_dist:
            dist.barrier()
            dist.destroy_process_group()
        return
    # this rank's contiguous shard of a global batch of B * world images (dist.ShardedPredictor)
    sp = ShardedPredictor(model, B * world, S, dev, batch_size=B, depth=int(os.environ.get("FCE_PIPE_DEPTH", "2")),
                          lanes=a.lanes, gather=use_dist and os.environ.get("FCE_DIST_NO_GATHER") != "1")
    eng = sp.engine
    for e in sp.pipe.engs:
        e.graph = bool(a.graph)
    # a ring of distinct resident input batches (lanes + 1 by default), cycled by the steps: no lane re-reads an input
    # batch another lane has just pulled through the 256 MB MALL
    gen = torch.Generator().manual_seed(1000 + rank)
    xs = [torch.rand(B, 3, S, S, generator=gen).half().to(dev) for _ in range(max(1, a.inputs))]
    x = xs[0]
    nms = NMS(B, eng.anchors, eng.nc, dev)
    it = [0]

    def step():
        xi = xs[it[0] % len(xs)]
        it[0] += 1
        if a.no_nms:
            eng(xi)
        elif a.sequential:
            nms(eng(xi), eng.best)
        else:  # forward of this batch overlaps the NMS (+ multi-GPU gather) of the previous one
            sp.submit(xi)

    def barrier():
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()  # device-wide: includes the NMS side stream

    for _ in range(a.warmup):
        step()
    sp.flush()
    _trace_marker()
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    sp.flush()  # the last batch's NMS (+ gather) is inside the timed region
    barrier()
    el = time.perf_counter() - t0
    _trace_marker()
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if use_dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    ms_step = el / a.steps * 1e3
    total_imgs = world * B * a.steps
    value = total_imgs / el

    # forward-only time (graph replay) for reference
    barrier()
    t1 = time.perf_counter()
    for _ in range(a.steps):
        eng(x)
    barrier()
    fwd_ms = (time.perf_counter() - t1) / a.steps * 1e3

    # strictly one batch at a time: forward (direct launches, the faster mode with one batch in flight) then
    # NMS, host-synchronised after every batch -> the one-lane rate and the per-batch latency (submit ->
    # detections ready); max over ranks
    lat = []
    for _ in range(max(5, min(a.steps, 30))):
        t2 = time.perf_counter()
        pr = eng(x, graph=False)
        if not a.no_nms:
            nms(pr, eng.best)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t2)
    lat_t = torch.tensor([sum(lat) / len(lat), sorted(lat)[len(lat) // 2]], dtype=torch.float64, device=dev)
    if use_dist:
        dist.all_reduce(lat_t, op=dist.ReduceOp.MAX)
    lat_mean, lat_med = (float(v) for v in lat_t.tolist())

    # per-op HIP-event profile (events on the launching stream around every op of the same direct-launch
    # sequence, averaged over `steps` passes) -> dominant kernel family roofline
    _trace_marker()
    prof = None
    for _ in range(max(1, a.profile_passes)):
        p = eng.profile(x, launches=True)
        prof = p if prof is None else [(*q[:3], q[3] + r[3], q[4]) for q, r in zip(prof, p)]
    prof = [(q[0], q[1], q[2], q[3] / max(1, a.profile_passes), q[4]) for q in prof]
    fam = defaultdict(lambda: [0.0, 0.0, 0.0, 0])
    for name, nbytes, flops, ms, nl in prof:
        f = fam[name]
        f[0] += ms
        f[1] += nbytes
        f[2] += flops
        f[3] += nl
    if not a.no_nms:  # device NMS (2 kernels per batch), event-timed over `steps` back-to-back calls
        _trace_marker()
        pred = eng(x)
        barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            nms(pred)
        e1.record()
        barrier()
        fam["nms"] = [e0.elapsed_time(e1) / a.steps, 0.0, 0.0, 2]
    dom = max(((k, v) for k, v in fam.items() if v[1] > 0), key=lambda kv: kv[1][0])
    dname, (dms, dbytes, dflops, dn) = dom
    ai = dflops / max(dbytes, 1.0)
    if ai >= RIDGE:
        ach = dflops / (dms / dn * 1e-3) / dn / 1e12
        roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": MFMA_F16_PEAK_TFS, "unit": "TFLOP/s"}
    else:
        ach = dbytes / dn / (dms / dn * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
    pp = pmc_path(a.model, B, S)
    pf = _pmc_family(pp, dname)
    roof["traffic"] = None if pf is None else round(float(pf["hbm_bytes"]) / 1e6, 3)
    roof["traffic_unit"] = f"MB/launch (rocprofv3 FETCH_SIZE*2 + WRITE_SIZE, {pp.relative_to(ROOT)})"
    if pf is not None and "mfma_tflops" in pf:  # MFMA counter pass of the same config (profiled clocks)
        roof["mfma_counter"] = {"tflops": pf["mfma_tflops"], "frac": pf["mfma_frac"],
                                "source": "SQ_INSTS_VALU_MFMA_MOPS_F16 x 512 / kernel time, rocprofv3 pass"}
    roof["kernel"] = dname
    roof["launches_per_step"] = dn
    roof["kernel_ms_per_step"] = round(dms, 4)
    kernel_ms = sum(p[3] for p in prof)
    stem = Path(a.model).stem
    batch_flops = sum(p[2] for p in prof)  # 2*MAC of every conv / matmul of one batch (op_cost)
    batch_bytes = sum(p[1] for p in prof)  # algorithmic bytes of every op of one batch (op_cost)
    # whole-forward roofline: achieved = img/s x GFLOP/img against min(MFMA peak, AI x HBM peak)
    ai_fwd = batch_flops / max(batch_bytes, 1.0)
    roof_tfs = min(MFMA_F16_PEAK_TFS, ai_fwd * HBM_PEAK_GBS / 1e3)
    ach_tfs = value / world * batch_flops / B / 1e12
    out = {
        "metric": "images/sec/GPU @ 640x640 bs=32, yolo11n-fce; fraction of fp16 MFMA roofline",
        "value": round(value, 2),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp16",
        "data": "synthetic torch.rand(B,3,S,S) fp16 per rank; seeded random-init weights of the architecture",
        "config": {"workload": f"{stem} detection inference (forward + decode + NMS) @ {S}x{S}, {B} images/GPU",
                   "model": stem, "global_batch": B * world, "imgsz": S, "parallelism": f"dp{world}",
                   "batches_in_flight": 1 if (a.no_nms or a.sequential) else a.lanes,
                   "distinct_inputs": len(xs),
                   "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4),
                   "forward_launch": "hipgraph" if a.graph else "direct"},
        "roofline": roof,
        "roofline_forward": {"achieved": round(ach_tfs, 3), "peak": round(roof_tfs, 2), "unit": "TFLOP/s",
                             "frac": round(ach_tfs / roof_tfs, 4), "ai_flop_per_byte": round(ai_fwd, 2),
                             "bound": "mfma" if ai_fwd >= RIDGE else "hbm",
                             "source": "img/s x algorithmic flop/img over min(2.5 PF, AI x 8 TB/s), AI = op_cost flops "
                                       "/ op_cost bytes of the whole forward (BASELINE.md §3)"},
        "value_1lane": round(B * world / lat_mean, 2),
        "latency_ms_per_batch": {"mean": round(lat_mean * 1e3, 4), "median": round(lat_med * 1e3, 4),
                                 "mode": "one batch at a time: forward (direct launches) + NMS, host sync per batch"},
        "forward_ms_per_batch": round(fwd_ms, 4),
        "forward_kernel_busy_ms": round(kernel_ms, 4),
        "profile_passes": max(1, a.profile_passes),
        "gflop_per_img": round(batch_flops / B / 1e9, 3),
        "model_tflops": round(value / world * batch_flops / B / 1e12, 3),
        "forward_mfma_frac": round(value / world * batch_flops / B / 1e12 / MFMA_F16_PEAK_TFS, 4),
        "kernels": {k: {"ms": round(v[0], 4), "launches": v[3], "GB/s": round(v[1] / (v[0] * 1e-3) / 1e9, 1)
                        if v[0] else None, "TFLOP/s": round(v[2] / (v[0] * 1e-3) / 1e12, 2) if v[0] else None}
                    for k, v in sorted(fam.items(), key=lambda kv: -kv[1][0])},
    }
    if a.profile_json and rank == 0:
        Path(a.profile_json).write_text(json.dumps([list(p) for p in prof], indent=0))
    if rank == 0 and world == 1 and (a.predict_steps > 0 or a.dist_config_steps > 0):
        # the main line's lanes (executors, streams, arenas) are released first: the later legs bring their own
        sp.close()
        sp = eng = nms = None
        xs = x = None
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and a.dist_config_steps > 0 and not use_dist and not (a.no_nms or a.sequential):
        out["value_dist_config"] = dist_config_line(a)
    if rank == 0 and world == 1 and a.predict_steps > 0:
        out["predict_pcie_inclusive"] = predict_rate(model, B, S, dev, a.predict_steps, a.predict_lanes)
    if rank == 0 and world == 1 and a.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(a.model, S, a.cpu_seconds, B)
    elif rank == 0:
        out["cpu_baseline"] = None
    out["process_group"] = ({"backend": dist.get_backend(), "world_size": dist.get_world_size()} if use_dist
                            else None)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()
    if sp is not None:
        sp.close()


if __name__ == "__main__":
    main()
