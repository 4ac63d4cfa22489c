"""Generate golden vectors by running the REFERENCE (ShioMisaka/fce-yolo) in the build container.

Run here only (the reference never travels to the GPU box):

    python tests/golden/make_golden.py

Import recipe: the reference imports ``cv2`` at module top
(``ultralytics/utils/__init__.py:24``) and reads the torchvision version through
``importlib.metadata`` (``:54``); neither is used by the tensor path.  This script
installs an attribute-only ``cv2`` module object and a name/version-only
torchvision dist-info on a temp path *for the import to succeed*; no arithmetic
goes through them.  With torchvision absent the reference NMS takes the
``TorchNMS.nms`` path (Q10).  Outputs are data only (inputs + expected outputs +
small per-op state_dicts) written to ``tests/golden/``.
"""

from __future__ import annotations

import hashlib
import importlib.util
import io
import json
import logging
import os
import sys
import tempfile
import types
from contextlib import contextmanager
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
REF = Path("/root/reference")


def _load_pkg():
    spec = importlib.util.spec_from_file_location(
        "fce_yolo_amd", REPO / "fce-yolo_amd" / "__init__.py", submodule_search_locations=[str(REPO / "fce-yolo_amd")]
    )
    mod = importlib.util.module_from_spec(spec)
    sys.modules["fce_yolo_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def import_reference():
    tmp = Path(tempfile.mkdtemp(prefix="fceref_"))
    os.environ.setdefault("YOLO_CONFIG_DIR", str(tmp / "cfg"))
    os.environ.setdefault("YOLO_OFFLINE", "1")
    cv2 = types.ModuleType("cv2")
    cv2.setNumThreads = lambda n: None
    for i, name in enumerate(["IMREAD_COLOR", "IMREAD_GRAYSCALE", "IMREAD_UNCHANGED", "INTER_LINEAR", "INTER_AREA"]):
        setattr(cv2, name, i)

    def _missing(name):
        if name.startswith("__"):
            raise AttributeError(name)

        def _unavailable(*a, **k):
            raise RuntimeError(f"cv2 stub: cv2.{name} is not available in the build container")

        return _unavailable

    cv2.__getattr__ = _missing
    sys.modules["cv2"] = cv2
    dist = tmp / "site" / "torchvision-0.25.0.dist-info"
    dist.mkdir(parents=True)
    (dist / "METADATA").write_text("Metadata-Version: 2.1\nName: torchvision\nVersion: 0.25.0\n")
    sys.path.insert(0, str(tmp / "site"))
    sys.path.insert(0, str(REF))
    import ultralytics  # noqa: F401
    from ultralytics.nn import tasks

    return tasks


@contextmanager
def capture_parse_log():
    from ultralytics.utils import LOGGER

    buf = io.StringIO()
    h = logging.StreamHandler(buf)
    h.setLevel(logging.INFO)
    old = LOGGER.level
    LOGGER.setLevel(logging.INFO)
    LOGGER.addHandler(h)
    try:
        yield buf
    finally:
        LOGGER.removeHandler(h)
        LOGGER.setLevel(old)


def seed_module(mod, seed, bn_eps=1e-3, **kw):
    from fce_yolo_amd.weights import seeded_state_dict

    sd = mod.state_dict()
    new = seeded_state_dict([(k, v.shape) for k, v in sd.items()], seed, **kw)
    mod.load_state_dict(new)
    for m in mod.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.eps = bn_eps
    mod.eval()
    return mod


def sd_np(mod):
    return {f"sd::{k}": v.detach().cpu().numpy() for k, v in mod.state_dict().items()}


def layer_table(tasks, cfg_name: str, mutate=None):
    """Parse `cfg_name` through the reference parser; return layer rows and state_dict keys/shapes."""
    d = tasks.yaml_model_load(cfg_name)
    if mutate:
        mutate(d)
    with capture_parse_log() as buf:
        model, save = tasks.parse_model(dict(d), ch=3, verbose=True)
    rows = []
    for line in buf.getvalue().splitlines():
        s = line.strip()
        if not s or not s.split()[0].isdigit():
            continue
        i = int(s.split()[0])
        m = model[i]
        t = type(m).__name__ if not isinstance(m, torch.nn.Sequential) else type(m[0]).__name__
        # args string is everything after the module type column
        args = s.split(str(m.type), 1)[1].strip() if hasattr(m, "type") else ""
        rows.append({"i": i, "f": m.f, "type": t, "np": int(m.np), "args": args})
    keys = [[f"model.{k}", list(v.shape)] for k, v in model.state_dict().items()]
    return {"rows": rows, "save": save, "state_dict": keys, "legacy_detect": bool(type(model[-1]).legacy)}


def main():
    torch.set_num_threads(8)
    tasks = import_reference()
    _load_pkg()
    from ultralytics.nn.modules import C2PSA, SPPF, C3k2, Conv, Detect, DWConv
    from ultralytics.nn.modules.fce_block import BiCoordCrossAtt, BiFPN_Concat, CoordAtt, CoordCrossAtt
    from ultralytics.utils.nms import non_max_suppression

    cfgdir = REF / "ultralytics/cfg/models/11"
    g = torch.Generator().manual_seed(1234)

    # ------------------------------------------------------------------ 1. parser fixtures
    def heads8(d):
        for row in d["backbone"]:
            if row[2] == "BiCoordCrossAtt":
                row[3] = [512, 8, 8]

    tables = {}
    for name in ["yolo11n-fce", "yolo11s-fce", "yolo11m-fce", "yolo11l-fce", "yolo11x-fce",
                 "yolo11n-bifpn", "yolo11s-bifpn", "yolo11m-bifpn", "yolo11n", "yolo11m"]:
        tables[name] = layer_table(tasks, str(cfgdir / f"{name}.yaml"))
    tables["yolo11m-fce-h8"] = layer_table(tasks, str(cfgdir / "yolo11m-fce.yaml"), heads8)
    (HERE / "parser_tables.json").write_text(json.dumps(tables, indent=0))
    print("parser tables:", list(tables))

    # ------------------------------------------------------------------ 2. per-op fixtures
    ops = {}

    def op_case(name, mod, inputs, seed, **kw):
        seed_module(mod, seed, **kw)
        with torch.inference_mode():
            out = mod(inputs if not isinstance(inputs, list) else list(inputs))
        ent = {"out": out.numpy()}
        if isinstance(inputs, list):
            for i, x in enumerate(inputs):
                ent[f"in{i}"] = x.numpy()
        else:
            ent["in0"] = inputs.numpy()
        ent["seed"] = np.array(seed)  # weights = seeded_state_dict(module keys, seed) + bn eps 1e-3
        ops[name] = ent

    def rnd(*s):
        return torch.randn(*s, generator=g)

    op_case("bicoord_n", BiCoordCrossAtt(128, 128, 8, 4), rnd(2, 128, 24, 20), 11)
    op_case("bicoord_l_dh16", BiCoordCrossAtt(512, 512, 8, 4), rnd(2, 512, 10, 12), 12)
    op_case("bicoord_h8", BiCoordCrossAtt(512, 512, 8, 8), rnd(1, 512, 12, 9), 13)
    op_case("bicoord_oup", BiCoordCrossAtt(64, 96, 8, 2), rnd(2, 64, 16, 12), 14)
    op_case("bicoord_dh2", BiCoordCrossAtt(32, 32, 32, 4), rnd(2, 32, 7, 11), 15)
    op_case("bifpn_2", BiFPN_Concat([64, 32], 32), [rnd(2, 64, 16, 12), rnd(2, 32, 16, 12)], 21)
    op_case("bifpn_3", BiFPN_Concat([16, 32, 32], 16), [rnd(2, 16, 8, 10), rnd(2, 32, 8, 10), rnd(2, 32, 8, 10)], 22)
    op_case("bifpn_id", BiFPN_Concat([32, 32], 32), [rnd(2, 32, 8, 10), rnd(2, 32, 8, 10)], 23)
    m = BiFPN_Concat([24, 48, 24], 24)
    seed_module(m, 24)
    with torch.no_grad():
        m.w[1] = -0.5  # relu clamps it to 0
    xs = [rnd(2, 24, 6, 6), rnd(2, 48, 6, 6), rnd(2, 24, 6, 6)]
    with torch.inference_mode():
        ops["bifpn_negw"] = {"out": m(list(xs)).numpy(), **{f"in{i}": x.numpy() for i, x in enumerate(xs)}, **sd_np(m)}
    op_case("coordatt_same", CoordAtt(64, 64, 16), rnd(2, 64, 12, 10), 31)
    op_case("coordatt_oup", CoordAtt(32, 48, 4), rnd(2, 32, 9, 14), 32)
    op_case("coordcross", CoordCrossAtt(64, 64, 4, 2), rnd(2, 64, 10, 13), 41)
    op_case("coordcross_h1", CoordCrossAtt(32, 32, 8, 1), rnd(2, 32, 6, 5), 42)
    op_case("conv_k1", Conv(24, 40, 1, 1), rnd(2, 24, 9, 11), 51)
    op_case("conv_k3s1", Conv(16, 32, 3, 1), rnd(2, 16, 9, 11), 52)
    op_case("conv_k3s2", Conv(16, 24, 3, 2), rnd(2, 16, 13, 11), 53)
    op_case("conv_c3", Conv(3, 16, 3, 2), rnd(2, 3, 20, 18), 54)
    op_case("dwconv", DWConv(32, 32, 3), rnd(2, 32, 9, 7), 55)
    op_case("sppf", SPPF(64, 64, 5), rnd(2, 64, 10, 9), 61)
    op_case("c2psa", C2PSA(256, 256, 1), rnd(2, 256, 6, 7), 62)
    op_case("c3k2_b", C3k2(32, 64, 1, False, 0.25), rnd(2, 32, 10, 8), 63)
    op_case("c3k2_c3k", C3k2(64, 64, 2, True), rnd(2, 64, 8, 6), 64)
    det = Detect(80, (64, 128, 256))
    det.stride = torch.tensor([8.0, 16.0, 32.0])
    seed_module(det, 71)
    feats = [rnd(2, 64, 16, 12), rnd(2, 128, 8, 6), rnd(2, 256, 4, 3)]
    with torch.inference_mode():
        y, maps = det([f.clone() for f in feats])
    ops["detect"] = {"out": y.numpy(), **{f"in{i}": f.numpy() for i, f in enumerate(feats)},
                     **{f"map{i}": mm.numpy() for i, mm in enumerate(maps)}, "seed": np.array(71)}
    np.savez_compressed(HERE / "ops.npz", **{f"{k}/{kk}": vv for k, v in ops.items() for kk, vv in v.items()})
    print("per-op fixtures:", list(ops))

    # ------------------------------------------------------------------ 3. end-to-end fixtures
    e2e = {}

    def build(name, mutate=None):
        d = tasks.yaml_model_load(str(cfgdir / f"{name}.yaml"))
        if mutate:
            mutate(d)
        model = tasks.DetectionModel(d, ch=3, verbose=False)
        sd = model.state_dict()
        from fce_yolo_amd.weights import seeded_state_dict

        model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in sd.items()], seed=0))
        model.eval()
        model.fuse(verbose=False)
        return model

    def run(model, bs, s, seed):
        x = torch.rand(bs, 3, s, s, generator=torch.Generator().manual_seed(seed))
        with torch.inference_mode():
            y = model(x)[0]
        return x, y

    for name, mut, bs, s in [("yolo11n-fce", None, 2, 160), ("yolo11n-fce", None, 1, 320),
                             ("yolo11s-bifpn", None, 2, 160), ("yolo11m-fce-h8", heads8, 1, 128),
                             ("yolo11l-fce", None, 1, 128), ("yolo11n", None, 1, 160)]:
        base = name.replace("-h8", "")
        model = build(base, mut)
        x, y = run(model, bs, s, seed=s + bs)
        key = f"{name}_{s}_b{bs}"
        e2e[f"{key}/x_sha256"] = np.frombuffer(hashlib.sha256(x.numpy().tobytes()).digest(), np.uint8)
        e2e[f"{key}/x_seed"] = np.array(s + bs)  # x = torch.rand(bs,3,s,s, generator=manual_seed(x_seed))
        e2e[f"{key}/y"] = y.numpy()
        if name == "yolo11n-fce" and s == 160:
            dets, keep = non_max_suppression(y.clone(), 0.25, 0.7, max_det=300, return_idxs=True)
            for b in range(bs):
                e2e[f"{key}/nms_det{b}"] = dets[b].numpy()
                e2e[f"{key}/nms_keep{b}"] = keep[b].numpy()
        print("e2e", key, tuple(y.shape), float(y[:, 4:].max()))
    # 640 bs=1 : digest + slices only (full tensor would be 2.8 MB)
    model = build("yolo11n-fce")
    x, y = run(model, 1, 640, seed=640)
    yn = y.numpy()
    e2e["yolo11n-fce_640_b1/sha256"] = np.frombuffer(hashlib.sha256(yn.tobytes()).digest(), np.uint8)
    e2e["yolo11n-fce_640_b1/y_slice"] = yn[:, :, ::37].copy()
    e2e["yolo11n-fce_640_b1/y_sum"] = yn.astype(np.float64).sum(axis=2)
    np.savez_compressed(HERE / "e2e.npz", **e2e)

    # ------------------------------------------------------------------ 4. NMS fixtures
    nms = {}
    rng = np.random.Generator(np.random.PCG64(99))

    def designed_pred(bs, A, ncand, nc=80, spread=40.0):
        p = np.zeros((bs, 4 + nc, A), np.float32)
        p[:, 4:, :] = rng.random((bs, nc, A), dtype=np.float32) * 0.2  # below conf
        for b in range(bs):
            idx = rng.choice(A, ncand, replace=False)
            cx = rng.random(ncand) * 600 + 20
            cy = rng.random(ncand) * 600 + 20
            p[b, 0, :] = rng.random(A) * 640
            p[b, 1, :] = rng.random(A) * 640
            p[b, 2, :] = rng.random(A) * 60 + 4
            p[b, 3, :] = rng.random(A) * 60 + 4
            # clusters of overlapping boxes
            p[b, 0, idx] = np.round(cx / spread) * spread + rng.random(ncand) * 8
            p[b, 1, idx] = np.round(cy / spread) * spread + rng.random(ncand) * 8
            cls = rng.integers(0, 4, ncand)
            sc = 0.3 + 0.69 * rng.permutation(ncand) / max(ncand, 1)  # distinct scores (margin > 5e-3 when ncand<=138)
            p[b, 4 + cls, idx] = sc.astype(np.float32)
        return p

    cases = {"designed_small": designed_pred(3, 525, 120), "designed_many": designed_pred(2, 2100, 1200, spread=25.0),
             "none": np.zeros((2, 84, 300), np.float32)}
    sat = designed_pred(1, 4000, 3000, spread=15.0)
    cases["saturated_maxdet"] = sat
    for name, p in cases.items():
        t = torch.from_numpy(p.copy())
        dets, keep = non_max_suppression(t, 0.25, 0.7, max_det=300, return_idxs=True)
        nms[f"{name}/pred"] = p
        for b in range(p.shape[0]):
            nms[f"{name}/det{b}"] = dets[b].numpy()
            nms[f"{name}/keep{b}"] = keep[b].numpy()
        print("nms", name, [int(k.numel()) for k in keep])
    np.savez_compressed(HERE / "nms.npz", **nms)
    meta = {"torch": torch.__version__, "reference": "ShioMisaka/fce-yolo @ /root/reference (ultralytics 8.3.242)",
            "threads": torch.get_num_threads()}
    (HERE / "meta.json").write_text(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
