"""CPU: host-side logic of the product package — parser parity with the reference, state_dict
layout of the drop-in modules, and the C-ABI library (loads, exports every declared symbol,
host-only packing).  No GPU compute here."""

import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest
import torch

import cases
from fce_yolo_amd import _native as N
from fce_yolo_amd import modules as M
from fce_yolo_amd.parser import DetectionModel, load_cfg

ROOT = Path(__file__).resolve().parents[1]
CONFIGS = ["yolo11n-fce", "yolo11s-fce", "yolo11m-fce", "yolo11l-fce", "yolo11x-fce", "yolo11n-bifpn",
           "yolo11s-bifpn", "yolo11m-bifpn", "yolo11n", "yolo11m", "yolo11m-fce-h8"]


def _model(name):
    if name.endswith("-h8"):
        d = load_cfg(name[:-3] + ".yaml")
        cases.heads8(d)
        return DetectionModel(d)
    return DetectionModel(name + ".yaml")


@pytest.mark.parametrize("name", CONFIGS)
def test_state_dict_matches_reference(name, tables):
    """Same keys, same order, same shapes as the reference DetectionModel (drop-in checkpoint load)."""
    m = _model(name)
    ours = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    assert ours == tables[name]["state_dict"]


@pytest.mark.parametrize("name", CONFIGS)
def test_layer_table_matches_reference(name, tables):
    m = _model(name)
    rows = tables[name]["rows"]
    assert len(rows) == len(m.model)
    for layer, row in zip(m.model, rows):
        assert layer.f == row["f"] and layer.np == row["np"]
        assert type(layer).__name__ == row["type"]
        assert str(layer.args).replace("'", "") == row["args"].replace("'", "")
    assert m.save == tables[name]["save"]
    assert type(m.model[-1]).legacy == tables[name]["legacy_detect"]
    assert m.stride.tolist() == [8.0, 16.0, 32.0]


def test_yolo11n_fce_param_count():
    m = DetectionModel("yolo11n-fce.yaml")
    assert sum(p.numel() for p in m.parameters()) == 2568281  # SURVEY §3B, measured on the reference


def test_bifpn_double_width_quirk():
    """Q1: BiFPN_Concat output = make_divisible(max(c1) * width, 8) -> 64/32/32/64 at n scale."""
    m = DetectionModel("yolo11n-fce.yaml")
    assert [m.model[i].output_ch for i in (14, 17, 20, 23)] == [64, 32, 32, 64]


def test_coordcrossatt_oup_mismatch_raises():
    mod = M.CoordCrossAtt(128, 256, 16, 2)

    class Be:
        device = torch.device("cpu")

    with pytest.raises(RuntimeError, match="oup != inp"):
        mod.emit(Be(), cases.__dict__.get("View", None) or type("V", (), {"n": 1, "h": 4, "w": 4})())


def test_cpu_forward_is_shape_only_never_numeric():
    """A drop-in on a CPU tensor propagates shapes only (meta output, for the reference's stride probe);
    reading a value raises.  The package's own whole-model forward refuses CPU input outright."""
    y = M.Conv(8, 16, 3, 2)(torch.zeros(1, 8, 5, 4))
    assert y.device.type == "meta" and tuple(y.shape) == (1, 16, 3, 2)
    with pytest.raises((RuntimeError, NotImplementedError)):
        y.sum().item()
    det = DetectionModel("yolo11n-fce.yaml").model[-1]
    maps = det.train()([torch.zeros(1, c, s, s) for c, s in ((64, 8), (128, 4), (256, 2))])
    assert [tuple(m.shape) for m in maps] == [(1, 144, 8, 8), (1, 144, 4, 4), (1, 144, 2, 2)]
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        DetectionModel("yolo11n-fce.yaml")(torch.zeros(1, 3, 64, 64))


def test_library_exports_every_declared_symbol():
    header = (ROOT / "include" / "fce_yolo.h").read_text()
    declared = set(re.findall(r"\b(fce_[a-z0-9_]+)\s*\(", header))
    L = N.lib()
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    assert declared <= set(N.EXPORTED) | {"fce_net_create", "fce_net_destroy"}
    assert L.fce_abi_version() == 7


def test_device_count_without_gpu_is_safe():
    n = N.lib().fce_device_count()
    assert n >= 0


def _pack_ref(w, cin, cout, k):
    """Python statement of the dense MFMA fragment order (csrc/conv.hip conv_pack)."""
    cpt, taps = cin // 8, k * k
    nchunk = taps * cpt
    nsteps = (nchunk + 3) // 4
    nalloc = ((nsteps + 7) & ~7) + 8  # multiple of 8 + 8 zero fragments for the depth-D prefetch
    cot = (cout + 15) // 16
    out = np.zeros((cot, nalloc, 64, 8), np.float16)
    for ct in range(cot):
        for s in range(nsteps):
            for l in range(64):
                co = ct * 16 + (l & 15)
                if cin % 32 == 0:  # chunk-major: step = 32-channel chunk * k*k + tap
                    tap, ci = s % (k * k), (s // (k * k)) * 32 + (l >> 4) * 8
                    ok = True
                else:  # 8-channel chunks c = 4s + lane/16, tap-major
                    c = s * 4 + (l >> 4)
                    tap, ci, ok = c // cpt, (c % cpt) * 8, c < nchunk
                if co < cout and ok:
                    out[ct, s, l] = w[co, ci:ci + 8, tap // k, tap % k]
    return out


@pytest.mark.parametrize("cin,cout,k", [(8, 16, 3), (16, 8, 3), (32, 40, 1), (64, 80, 3), (24, 24, 1), (96, 32, 3)])
def test_dense_weight_packing(cin, cout, k):
    w = np.random.default_rng(0).standard_normal((cout, cin, k, k)).astype(np.float32)
    d = N.ConvDesc(cin, cout, k, 1, 1, 1, 0, 0, None, 0, 0)
    nb = N.lib().fce_conv_weight_bytes(C.byref(d))
    out = np.empty(nb, np.uint8)
    N.call("fce_conv_pack_weights", C.byref(d), w.ctypes.data, out.ctypes.data)
    assert np.array_equal(out.view(np.float16).reshape(-1), _pack_ref(w, cin, cout, k).reshape(-1))


def test_dw_and_stem_packing():
    w = np.random.default_rng(1).standard_normal((16, 1, 3, 3)).astype(np.float32)
    d = N.ConvDesc(16, 16, 3, 1, 16, 1, 0, 0, None, 0, 0)
    out = np.empty(N.lib().fce_conv_weight_bytes(C.byref(d)), np.uint8)
    N.call("fce_conv_pack_weights", C.byref(d), w.ctypes.data, out.ctypes.data)
    assert np.array_equal(out.view(np.float32).reshape(9, 16), w.reshape(16, 9).T)
    w = np.random.default_rng(2).standard_normal((16, 3, 3, 3)).astype(np.float32)
    d = N.ConvDesc(3, 16, 3, 2, 1, 1, 0, 0, None, 0, 0)
    out = np.empty(N.lib().fce_conv_weight_bytes(C.byref(d)), np.uint8)
    N.call("fce_conv_pack_weights", C.byref(d), w.ctypes.data, out.ctypes.data)
    assert out.size == 27 * 16 * 4 + 64 * 8 * 2  # fp32 table + one MFMA fragment (cout 16)
    assert np.array_equal(out[:27 * 16 * 4].view(np.float32).reshape(27, 16), w.reshape(16, 27).T)
    frag = out[27 * 16 * 4:].view(np.float16).reshape(64, 8)  # lane l: cout l & 15, k = 8 (l >> 4) + j
    ref = np.zeros((64, 8), np.float16)
    for lane in range(64):
        for j in range(8):
            k = 8 * (lane >> 4) + j
            ref[lane, j] = w[lane & 15].reshape(27)[k] if k < 27 else 0
    assert np.array_equal(frag, ref)


@pytest.mark.parametrize("cin,cout,k,stride,kinds_in,kinds_out", [
    (512, 512, 1, 1, {0x400, 0x700, 0xB00}, {0x800}),  # wide 1x1: LDS tile, big-tile pipelined, 256-wide tiles
    (256, 32, 1, 1, {0x400}, {0x700, 0xB00}),       # narrow cout: no 64-cout-per-wave tile
    (48, 128, 1, 1, {0x400}, {0x300, 0x700, 0xB00}),  # cin % 32 != 0: no streaming, cin < 64: no big tile
    (64, 64, 3, 1, {0x100, 0x600, 0x800, 0xC00, 0xD00}, {0x400, 0x700}),  # 3x3: halo tiles, rings, big tiles, GEMM
    (256, 256, 3, 2, {0x100, 0x800, 0xC00}, {0x600, 0x700, 0xB00, 0xD00}),  # wide stride-2 3x3: + LDS-DMA tiles, GEMM
    (256, 96, 3, 2, {0x100, 0xC00}, {0x800}),        # stride 2 needs 128 couts per LDS-DMA big-tile block
    (64, 32, 3, 1, {0x100}, {0xC00}),                # the implicit GEMM needs >= 64 couts
    (16, 32, 3, 2, {0x200}, {0x100, 0x700, 0x800, 0xC00}),  # small-cin 3x3
])
def test_conv_variant_enumeration(cin, cout, k, stride, kinds_in, kinds_out):
    """Host-side candidate lists (no GPU): every listed code decodes to a known kernel kind, the kinds
    each shape qualifies for are present, and the ones it does not are absent."""
    d = N.ConvDesc(cin, cout, k, stride, 1, 1, 0, 0, None, 0, 0)
    codes = (C.c_int * 128)()
    nv = N.lib().fce_conv_variants(C.byref(d), 80, codes, 128)
    kinds = {c & 0xF00 for c in codes[:nv]}
    assert nv >= 2 and len(set(codes[:nv])) == nv
    assert kinds <= {0x000, 0x100, 0x200, 0x300, 0x400, 0x500, 0x600, 0x700, 0x800, 0xA00, 0xB00, 0xC00, 0xD00}
    assert kinds_in <= kinds and not (kinds_out & kinds)


def test_error_path_reports_message():
    d = N.ConvDesc(8, 8, 5, 1, 1, 1, 0, 0, None, 0, 0)
    t = N.Tensor(None, N.F16, N.NHWC, 1, 8, 4, 4, 8, 0)
    with pytest.raises(N.FceError, match="kernel size"):
        N.call("fce_conv2d", C.byref(d), C.byref(t), 1, 1, None, C.byref(t), None)


def test_fold_bn_matches_reference_fuse():
    """modules.fold_bn == torch_utils.fuse_conv_and_bn restated in the oracle (eps 1e-3)."""
    from oracle import fce_oracle as O

    conv = M.Conv(16, 32, 3)
    sd = {k: v for k, v in cases.seeded_model("yolo11n-fce.yaml").model[1].state_dict().items()}
    conv.load_state_dict(sd)
    w, b = M.fold_bn(conv.conv, conv.bn)
    f = O.fuse_state_dict({"m." + k: v for k, v in conv.state_dict().items()})
    assert torch.equal(w, f["m.conv.weight"]) and torch.allclose(b, f["m.conv.bias"], atol=1e-7)


def test_library_has_no_undefined_internal_symbols():
    """Every fce:: function the translation units call is defined (a signature drift between a
    declaration and its definition links fine into a .so and only fails at load on the GPU box)."""
    import shutil
    import subprocess

    if not shutil.which("nm"):
        pytest.skip("nm not available")
    out = subprocess.run(["nm", "-uC", str(N.LIB_PATH)], capture_output=True, text=True, check=True).stdout
    bad = [l for l in out.splitlines() if "fce::" in l]
    assert not bad, bad


def _bench_env(**kw):
    import os

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_bench_gpus_n_launches_ranks_before_torch():
    """`python bench.py --gpus 2` (no WORLD_SIZE) starts torch.distributed.run with 2 ranks on 127.0.0.1 as a
    child process, decided before torch (let alone the GPU) is touched in the launcher."""
    import json
    import subprocess
    import sys

    root = Path(__file__).resolve().parents[1]
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--steps", "3"], capture_output=True,
                       text=True, timeout=120, env=_bench_env(FCE_BENCH_DRY_LAUNCH="1"))
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["torch_imported"] is False
    cmd = d["launch"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=2" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "2", "--steps", "3"] and cmd[-5].endswith("bench.py")
    # a rank (WORLD_SIZE set) or one GPU: no launcher
    sys.path.insert(0, str(root))
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", root / "bench.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    assert m.launch_command(["--gpus", "8"], {"WORLD_SIZE": "8"}) is None
    assert m.launch_command(["--gpus", "1"], {}) is None
    assert m.launch_command([], {}) is None
    # hardware queues: 8 for the default 4 lanes unless the environment already asks for >= 8; 3 lanes: untouched
    assert m.hw_queues_env([], {}) == "8" and m.hw_queues_env([], {"GPU_MAX_HW_QUEUES": "4"}) == "8"
    assert m.hw_queues_env([], {"GPU_MAX_HW_QUEUES": "16"}) is None
    assert m.hw_queues_env(["--lanes", "3"], {}) is None and m.hw_queues_env([], {"FCE_LANES": "2"}) is None
    # lanes default by scale: 4 for n / s / l, 3 for m at 1280 (its activation arenas overflow the MALL)
    assert m.default_lanes("yolo11n-fce.yaml", {}) == 4 and m.default_lanes("yolo11l-fce.yaml", {}) == 4
    assert m.default_lanes("yolo11m-fce-h8.yaml", {}) == 3 and m.default_lanes("yolo11s-bifpn.yaml", {}) == 4
    assert m.hw_queues_env(["--model", "yolo11l-fce.yaml"], {}) == "8"
    assert m.hw_queues_env(["--model", "yolo11m-fce-h8.yaml"], {}) is None
    # with a process group (N > 1, a rank, or the one-rank RCCL rehearsal): the same lanes and queues as one GPU
    # (round 5: the grouped, host-ordered gather no longer costs a four-lane step)
    assert m.default_lanes("yolo11n-fce.yaml", {}, 8) == 4 and m.default_lanes("yolo11n-fce.yaml", {"WORLD_SIZE": "8"}) == 4
    assert m.hw_queues_env(["--gpus", "8"], {}) == "8" and m.hw_queues_env([], {"WORLD_SIZE": "2"}) == "8"
    assert m.hw_queues_env([], {"FCE_DIST_FORCE": "1"}) == "8"
    assert m.default_lanes("yolo11m-fce-h8.yaml", {}, 8) == 3


def test_bench_world_size_mismatch_fails():
    import subprocess
    import sys

    root = Path(__file__).resolve().parents[1]
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "4"], capture_output=True, text=True,
                       timeout=300, env=_bench_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0 and "WORLD_SIZE 2" in r.stderr, (r.returncode, r.stderr[-500:])


def _lowered(cfg, monkeypatch, **env):
    """A model lowered into a NetBackend on the CPU (ops recorded, never planned or run): [(name, alt_form)]."""
    from fce_yolo_amd.backend import NetBackend

    for k in ("FCE_FUSE_STEM", "FCE_FUSE_DCLS", "FCE_FUSE_C3K2", "FCE_FUSE_BNECK", "FCE_FUSE_PW2"):
        if k in env:
            monkeypatch.setenv(k, env[k])
        else:
            monkeypatch.delenv(k, raising=False)
    model = cases.seeded_model(cfg, 0)
    be = NetBackend(640, 640, torch.device("cpu"))
    try:
        with torch.no_grad():
            model.emit(be, be.input_view(1, 3))
        L = N.lib()
        out = []
        for i in range(L.fce_net_num_ops(be.net)):
            name = C.create_string_buffer(64)
            nb, fl = C.c_double(), C.c_double()
            N.call("fce_net_op_info", be.net, i, name, 64, C.byref(nb), C.byref(fl))
            out.append((name.value.decode(), L.fce_net_alt_form(be.net, i)))
        return out
    finally:
        be.close()


def test_lowering_records_the_fused_alternatives(monkeypatch):
    """Graph lowering (no GPU): the n scale records the one-kernel stem pair after its two convs, the fused C3k2 after
    each qualifying block's four convs, and per Detect level P3 / P4 the box tail before the cls chain, whose five ops
    are followed by their one-kernel alternative; every alternative starts in its fused form (the plan decides).  The
    FCE_FUSE_* switches drop them; the s scale gets the stem pair but not the cls branch (c3 128), the l scale
    neither."""
    ops = _lowered("yolo11n-fce.yaml", monkeypatch)
    names = [n for n, _ in ops]
    alts = [(i, n) for i, (n, f) in enumerate(ops) if f >= 0]
    assert all(ops[i][1] == 1 for i, _ in alts)
    # stem; C3k2 L2, L4; L7 [pair, chain, pair]; L10 [pair, chain, pair]; C2PSA L12 three pairs; L14 -> L15 [BiFPN
    # realign -> cv1 pair, chain]; C3k2 L18; L20 -> L21 [pair, chain]; L24 [pair, chain, pair]; Detect cls P3, P4
    assert [n for _, n in alts] == (["stem_fused"] + ["c3k2_fused"] * 2 + ["pw2_fused", "bneck_fused", "pw2_fused"] * 2 +
                                    ["pw2_fused"] * 3 + ["pw2_fused", "bneck_fused", "c3k2_fused", "pw2_fused",
                                                         "bneck_fused"] +
                                    ["pw2_fused", "bneck_fused", "pw2_fused"] + ["detect_cls_fused"] * 2)
    assert names[:3] == ["conv_stem", "conv3x3_mfma", "stem_fused"]
    # the Bottleneck chains: C3k pairs (L7, L10, L24: four 3x3s) and the 40^2 neck blocks' single Bottleneck (L15, L21)
    assert [sum(1 for n in names[i - 4:i] if n == "conv3x3_mfma") for i, n in alts if n == "bneck_fused"] == [4, 4, 2, 2, 4]
    # every 1x1 pair replaces the two 1x1 convs right before it
    assert all(names[i - 2:i] == ["conv1x1_mfma"] * 2 for i, n in alts if n == "pw2_fused")
    for i, n in alts:
        if n == "detect_cls_fused":
            assert names[i - 5:i] == ["dwconv3x3", "conv1x1_mfma", "dwconv3x3", "conv1x1_mfma", "conv1x1_detect_cls"]
            assert names[i - 6] == "conv1x1_detect_box"
        if n == "c3k2_fused":
            assert names[i - 4:i] == ["conv1x1_mfma", "conv3x3_mfma", "conv3x3_mfma", "conv1x1_mfma"]
    plain = _lowered("yolo11n-fce.yaml", monkeypatch, FCE_FUSE_STEM="0", FCE_FUSE_DCLS="0", FCE_FUSE_C3K2="0",
                     FCE_FUSE_BNECK="0", FCE_FUSE_PW2="0")
    assert all(f < 0 for _, f in plain) and len(plain) == len(ops) - len(alts)
    # without the whole-block C3k2 alternative, the n L2 / L4 / L18 Bottlenecks get the chain kernel's instead (their
    # (c, c_mid) are not instantiated: 16 / 8, 32 / 16), so only the five chains above remain
    noc3 = [n for n, f in _lowered("yolo11n-fce.yaml", monkeypatch, FCE_FUSE_C3K2="0") if f >= 0]
    assert noc3.count("bneck_fused") == 5 and "c3k2_fused" not in noc3
    s_ops = [n for n, f in _lowered("yolo11s-bifpn.yaml", monkeypatch) if f >= 0]
    assert "stem_fused" in s_ops and "detect_cls_fused" not in s_ops
    l_ops = [n for n, f in _lowered("yolo11l-fce.yaml", monkeypatch) if f >= 0]
    assert "stem_fused" not in l_ops and "detect_cls_fused" not in l_ops
