"""GPU parity tests (MI355X): every op through the C-ABI vs the reference's golden vectors and the
oracle; end-to-end detection outputs; bit-exact NMS indices; graph/eager/batch invariance.

Tolerances (fp16 storage, fp32 accumulate, fp32 decode — Q11):
  * per op:        max|ours - ref| <= OP_TOL * max|ref|           (OP_TOL = 1e-3: every op fixture, the full-size
                   BiCoord / C2PSA fixtures included, measures 2.9e-4 .. 8.0e-4 on MI355X; fp16 storage rounds
                   at 2^-11 = 4.9e-4 of max|ref|, so 1e-3 is two fp16 half-ulps of headroom)
  * end-to-end:    boxes  max|d xywh| <= 1e-3 * max|xywh|   (north-star "1e-3 fp16 tolerance", relative)
                   scores max|d sigmoid| <= 1e-3               (absolute, scores in [0, 1])
  * NMS:           kept anchor indices and (k, 6) rows bit-exact vs the reference on the same preds.
"""

import ctypes as C
import hashlib

import numpy as np
import pytest
import torch

import cases
from conftest import NMS_OPT_CASES, nms_opt_case
from fce_yolo_amd import _native as N
from fce_yolo_amd import modules as M
from fce_yolo_amd.engine import NMS, Engine, Pipeline, non_max_suppression
from oracle import nms_oracle

pytestmark = pytest.mark.gpu
OP_TOL = 1e-3
BOX_TOL = 1e-3
CLS_TOL = 1e-3


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def test_native_library_sees_the_gpu(device):
    assert N.lib().fce_device_count() >= 1


def test_mfma_conv_exact_integer(device):
    """A = weights, B = activations fragment maps: exact small-integer GEMM (asymmetric operands)."""
    torch.manual_seed(0)
    for cin, cout, k in [(32, 16, 1), (16, 48, 3), (8, 8, 3), (64, 24, 1)]:
        conv = M.Conv(cin, cout, k, act=False)
        with torch.no_grad():
            conv.conv.weight.copy_(torch.randint(-3, 4, conv.conv.weight.shape).float())
            conv.bn.weight.fill_(1.0)
            conv.bn.bias.zero_()
            conv.bn.running_mean.zero_()
            conv.bn.running_var.fill_(1.0 - 1e-3)  # scale exactly 1
        x = torch.randint(-2, 3, (2, cin, 7, 9)).half()
        ref = torch.nn.functional.conv2d(x.double(), conv.conv.weight.double(), None, 1, k // 2)
        conv = conv.to(device)
        y = conv(x.to(device).contiguous(memory_format=torch.channels_last))
        assert torch.equal(y.double().cpu(), ref), (cin, cout, k)


@pytest.mark.parametrize("cin,cout,H,W", [(3, 16, 64, 96), (3, 32, 40, 48), (1, 16, 34, 72), (2, 48, 30, 40),
                                            (3, 64, 66, 64)])
def test_stem_mfma_parity(cin, cout, H, W, device):
    """The MFMA stem (first Conv, 3x3 s2 on the NCHW network input, k = ci * 9 + tap zero-padded to one 32-deep
    K-step: the padded k slots re-read a real tap, their weights are zero) against a plain torch fp32 Conv + BN +
    SiLU on the same fp16 input, for 1-3 input channels, 16-64 outputs, odd / ragged maps."""
    torch.manual_seed(cin * 100 + cout)
    conv = M.Conv(cin, cout, 3, 2)
    with torch.no_grad():
        conv.conv.weight.normal_(0, 0.3)
        conv.bn.weight.uniform_(0.5, 1.5)
        conv.bn.bias.normal_(0, 0.2)
        conv.bn.running_mean.normal_(0, 0.1)
        conv.bn.running_var.uniform_(0.5, 1.5)
    conv.eval()
    x = torch.rand(2, cin, H, W).half()
    with torch.no_grad():
        ref = torch.nn.functional.silu(conv.bn(conv.conv(x.float())))
        y = conv.to(device)(x.to(device))
    assert tuple(y.shape) == tuple(ref.shape)
    err = _rel(y.float(), ref)
    print(f"OPERR stem {cin}->{cout} {err:.3e}")
    assert err <= OP_TOL, err


@pytest.mark.parametrize("name", list(cases.OPS))
def test_op_parity(name, ops_fx, device):
    fx = ops_fx.group(name)
    mod = cases.build_op(name, fx).to(device)
    ins = [t.to(device) for t in cases.op_inputs(fx)]
    with torch.no_grad():
        y = mod(ins if len(ins) > 1 else ins[0].half())
    ref = torch.from_numpy(fx["out"])
    assert tuple(y.shape) == tuple(ref.shape)
    assert torch.isfinite(y).all()
    err = _rel(y.float(), ref)
    print(f"OPERR {name} {err:.3e}")
    assert err <= OP_TOL, err


@pytest.mark.parametrize("name", ["bicoord_n", "bicoord_l_dh16", "bicoord_h8", "bicoord_oup", "bicoord_dh2"])
def test_bicoord_fused_core_and_split_paths(name, ops_fx, device, monkeypatch):
    """The one-launch middle (coord_core_kernel) and the split projection / attention / projection path
    both against the reference fixture, and against each other."""
    fx = ops_fx.group(name)
    mod = cases.build_op(name, fx).to(device)
    x = cases.op_inputs(fx)[0].to(device).half()
    ref = torch.from_numpy(fx["out"])
    with torch.no_grad():
        yc = mod(x).float()
        monkeypatch.setenv("FCE_COORD_NO_CORE", "1")
        ys = mod(x).float()
        monkeypatch.setenv("FCE_COORD_PROJ1", "1")  # scalar projection kernel: same k order
        y1 = mod(x).float()
    assert _rel(yc, ref) <= OP_TOL and _rel(ys, ref) <= OP_TOL
    assert _rel(yc, ys) <= 2e-3
    assert _rel(ys, y1) <= 1e-3, _rel(ys, y1)  # fp32 gate differences flip fp16 output roundings


def test_op_fp32_dropin_keeps_dtype(ops_fx, device):
    fx = ops_fx.group("conv_k3s1")
    mod = cases.build_op("conv_k3s1", fx).to(device)
    x = cases.op_inputs(fx)[0].to(device)
    y = mod(x)
    assert y.dtype == torch.float32 and y.shape == (2, 32, 9, 11)
    assert _rel(y, torch.from_numpy(fx["out"])) <= OP_TOL


def test_detect_parity(ops_fx, device):
    fx = ops_fx.group("detect")
    det = cases.build_detect(fx).to(device)
    feats = [torch.from_numpy(fx[f"in{i}"]).to(device).half() for i in range(3)]
    y, maps = det(feats)
    ref = torch.from_numpy(fx["out"])
    assert _rel(y[:, :4], ref[:, :4]) <= BOX_TOL * 3
    assert (y[:, 4:].cpu() - ref[:, 4:]).abs().max().item() <= CLS_TOL * 3
    for i in range(3):
        assert _rel(maps[i], torch.from_numpy(fx[f"map{i}"])) <= OP_TOL
    # the standalone decode kernel (fce_detect_decode) on the reference's own fp32 maps
    from fce_yolo_amd.backend import EagerBackend, View

    be = EagerBackend(device)
    views = []
    for i in range(3):
        m = torch.from_numpy(fx[f"map{i}"]).to(device).contiguous(memory_format=torch.channels_last)
        views.append(View(m, m.shape[0], m.shape[1], m.shape[2], m.shape[3], m.shape[1], 0, N.F32))
    yd = be.detect(views, [8.0, 16.0, 32.0], 16)
    assert _rel(yd[:, :4], ref[:, :4]) <= 1e-6
    assert (yd[:, 4:].cpu() - ref[:, 4:]).abs().max().item() <= 1e-6


def _engine_run(key, fx, device, graph=True):
    cfg, mut = cases.E2E[key]
    model = cases.seeded_model(cfg, 0, mut).to(device)
    x = cases.e2e_input(key, fx)
    eng = Engine(model, x.shape[0], x.shape[2], device)
    y = eng(x.to(device).half(), graph=graph).clone()
    torch.cuda.synchronize()
    return model, eng, x, y


@pytest.mark.parametrize("key", list(cases.E2E))
def test_end_to_end_parity(key, e2e_fx, device):
    fx = e2e_fx.group(key)
    model, eng, x, y = _engine_run(key, fx, device)
    ref = torch.from_numpy(fx["y"])
    assert torch.isfinite(y).all()
    box = _rel(y[:, :4], ref[:, :4])
    cls = (y[:, 4:].cpu() - ref[:, 4:]).abs().max().item()
    print(f"{key}: box rel {box:.2e} cls abs {cls:.2e}")
    assert box <= BOX_TOL and cls <= CLS_TOL, (box, cls)


def test_graph_eager_and_module_forward_agree_bitwise(e2e_fx, device, monkeypatch):
    """Captured hipGraph, direct launches (1 and 4 streams over the op DAG) and the module forward."""
    key = "yolo11n-fce_160_b2"
    fx = e2e_fx.group(key)
    model, eng, x, yg = _engine_run(key, fx, device, graph=True)
    ye = eng(x.to(device).half(), graph=False).clone()
    yg2 = eng(x.to(device).half(), graph=True).clone()  # replay
    monkeypatch.setenv("FCE_STREAMS", "4")
    ys = eng(x.to(device).half(), graph=False).clone()
    monkeypatch.delenv("FCE_STREAMS")
    ym, _ = model(x.to(device).half())
    torch.cuda.synchronize()
    assert torch.equal(yg, ye) and torch.equal(yg, yg2) and torch.equal(yg, ym) and torch.equal(yg, ys)


def _predict_once(model, x):
    """tasks.py:160-188 as the reference runs it with the drop-ins bound: module by
    module through ``forward``; ``nn.Upsample`` is torch's own there, so it runs as torch's here."""
    y = []
    for m in model.model:
        if m.f != -1:
            x = y[m.f] if isinstance(m.f, int) else [x if j == -1 else y[j] for j in m.f]
        x = torch.nn.Upsample.forward(m, x) if isinstance(m, M.Upsample) else m(x)
        y.append(x if m.i in model.save else None)
    return x


@pytest.mark.parametrize("key", list(cases.E2E))
def test_dropin_predict_once_parity(key, e2e_fx, device):
    """The eager drop-in path the reference drives: fuse() (tasks.py:223-252, restated by
    DetectionModel.fuse and checked against the reference in test_reference_dropin.py), .half().to(cuda),
    eval, per-module forward -> (y, maps); y against the reference's fused fp32 output."""
    fx = e2e_fx.group(key)
    cfg, mut = cases.E2E[key]
    model = cases.seeded_model(cfg, 0, mut).fuse().half().to(device).eval()
    x = cases.e2e_input(key, fx)
    with torch.inference_mode():
        y, maps = _predict_once(model, x.half().to(device))
    ref = torch.from_numpy(fx["y"])
    assert y.shape == ref.shape and len(maps) == 3 and torch.isfinite(y).all()
    box = _rel(y[:, :4], ref[:, :4])
    cls = (y[:, 4:].cpu() - ref[:, 4:]).abs().max().item()
    print(f"{key}: drop-in box rel {box:.2e} cls abs {cls:.2e}")
    assert box <= BOX_TOL and cls <= CLS_TOL, (box, cls)


@pytest.mark.parametrize("key", list(cases.FULL))
def test_full_size_parity(key, full_fx, device):
    """BASELINE configs at their real sizes (m-h8 @1280: C2PSA over 1600 keys, BiCoord L5 at 160x160 on the
    >64 KiB LDS path; l / s @640; n @640 bs2): the whole output against the oracle (fp32, run on this
    host) and the reference's slices / row sums (golden/full.npz)."""
    fx = full_fx.group(key)
    cfg, mut, b, s = cases.FULL[key]
    model = cases.seeded_model(cfg, 0, mut)
    x = cases.full_input(key, fx)
    y = Engine(model.to(device), b, s, device)(x.half().to(device)).cpu()
    assert torch.isfinite(y).all()
    ref = cases.oracle_model(model.cpu(), x, torch.float32)
    box = _rel(y[:, :4], ref[:, :4])
    cls = (y[:, 4:] - ref[:, 4:]).abs().max().item()
    e_slice, e_sum = cases.compare_full(y, fx)
    print(f"{key}: box rel {box:.2e} cls abs {cls:.2e} | ref slice {e_slice:.2e} row sums {e_sum:.2e}")
    assert box <= BOX_TOL and cls <= CLS_TOL, (box, cls)
    assert e_slice <= BOX_TOL and e_sum <= BOX_TOL, (e_slice, e_sum)


@pytest.mark.parametrize("key", list(cases.OPS_FULL))
def test_full_size_op_parity(key, full_fx, device):
    """BiCoordCrossAtt at 80x80 / 160x160 and C2PSA at 20x20 / 40x40 (1600 keys), drop-in forward in fp16
    against the oracle's full tensor and the reference's slices / channel sums."""
    fx = full_fx.group(key)
    mod, x = cases.full_op(key, fx)
    ref = cases.full_op_oracle(key, mod, x)
    with torch.inference_mode():
        y = mod.to(device)(x.half().to(device)).float().cpu()
    assert y.shape == ref.shape and torch.isfinite(y).all()
    err = _rel(y, ref)
    e_slice, e_sum = cases.compare_full(y, fx, anchors=False)
    print(f"{key}: rel {err:.2e} | ref slice {e_slice:.2e} channel sums {e_sum:.2e}")
    assert err <= OP_TOL and e_slice <= OP_TOL and e_sum <= OP_TOL, (err, e_slice, e_sum)


@pytest.mark.parametrize("cfg,batch,imgsz", [("yolo11n-fce.yaml", 2, 320), ("yolo11l-fce.yaml", 1, 256),
                                              ("yolo11m-fce.yaml", 1, 192)])
def test_c3_concatenated_cv1_cv2_bitwise(cfg, batch, imgsz, device, monkeypatch):
    """C3 / C3k's cv1 and cv2 (both 1x1 over x) as ONE conv with concatenated weights (modules.C3.emit, the
    default) give the forward bit for bit what the two convs give (FCE_C3_CAT=0), whole-graph (with the dense copy
    of the bottlenecks' input below 64 channels) and per module (eager drop-in)."""
    model = cases.seeded_model(cfg, 0).to(device)
    x = torch.rand(batch, 3, imgsz, imgsz, generator=torch.Generator().manual_seed(4)).half().to(device)
    monkeypatch.setenv("FCE_FUSE_PW2", "0")  # the fused 1x1 pairs start from the merged conv: op counts would differ
    monkeypatch.setenv("FCE_C3_CAT", "0")
    e0 = Engine(model, batch, imgsz, device)
    y0 = e0(x).clone()
    n0 = e0.num_ops()
    monkeypatch.setenv("FCE_C3_CAT", "1")
    e1 = Engine(model, batch, imgsz, device)
    y1 = e1(x).clone()
    torch.cuda.synchronize()
    n_c3k = sum(1 for m in model.modules() if isinstance(m, M.C3k))
    assert n_c3k > 0 and e1.num_ops() == n0 - n_c3k
    assert torch.equal(y0, y1)
    c3 = next(m for m in model.modules() if isinstance(m, M.C3k))
    xi = torch.randn(batch, c3.cv1.conv.in_channels, 24, 20, device=device).half().contiguous(
        memory_format=torch.channels_last)
    with torch.no_grad():
        u1 = c3(xi)
        monkeypatch.setenv("FCE_C3_CAT", "0")
        u0 = c3(xi)
    torch.cuda.synchronize()
    assert torch.equal(u0, u1)


def test_fused_c3k2_unknown_tile_is_an_error(device, monkeypatch):
    """FCE_C3K2_TILE names one of the two instantiated tiles; anything else fails loudly instead of running the
    tile chosen by map width."""
    model = cases.seeded_model("yolo11n-fce.yaml", 0).to(device)
    x = torch.rand(1, 3, 160, 160, generator=torch.Generator().manual_seed(9)).half().to(device)
    monkeypatch.setenv("FCE_FUSE_C3K2", "1")
    monkeypatch.setenv("FCE_C3K2_TILE", "2,16,8")
    with pytest.raises(RuntimeError, match="FCE_C3K2_TILE"):
        eng = Engine(model, 1, 160, device)
        eng(x)
        torch.cuda.synchronize()
    monkeypatch.delenv("FCE_C3K2_TILE")
    monkeypatch.setenv("FCE_C3K2_YSTORE", "lds")
    with pytest.raises(RuntimeError, match="FCE_C3K2_YSTORE"):
        eng = Engine(model, 1, 160, device)
        eng(x)
        torch.cuda.synchronize()


@pytest.mark.parametrize("cfg,batch,imgsz,tile,ystore", [
    ("yolo11n-fce.yaml", 2, 320, None, None), ("yolo11s-bifpn.yaml", 2, 256, None, None),
    ("yolo11n-fce.yaml", 1, 640, None, None), ("yolo11n-fce.yaml", 1, 224, None, None),
    ("yolo11n-fce.yaml", 1, 224, "8,16,4", None), ("yolo11n-fce.yaml", 1, 224, "4,40,8", None),
    ("yolo11n-fce.yaml", 2, 160, "4,40,8", None), ("yolo11n-fce.yaml", 1, 224, None, "buf"),
    ("yolo11n-fce.yaml", 1, 224, None, "global"), ("yolo11s-bifpn.yaml", 1, 224, "4,40,8", "buf")])
def test_fused_c3k2_bitwise_equal_to_four_convs(cfg, batch, imgsz, tile, ystore, device, monkeypatch):
    """The fused C3k2 kernel (csrc/fused.hip) gives the forward bit for bit what its four convs give, whole-graph
    and per-module; every tile shape the planner picks (8 x 16 on 160^2 maps, 4 x 40 below), both tiles forced
    on every block (FCE_C3K2_TILE), both y store forms forced on every block (FCE_C3K2_YSTORE: buffer stores
    whose dropped lanes are the partial tiles' outside pixels, or branched global stores) and partial edge tiles
    (224: 56 = 3.5 x 16 = 1.4 x 40).  FCE_FUSE_C3K2=1 forces the fused
    form, =0 records the convs only; the default records both and the plan keeps the faster (auto), and every
    combination of forms the auto plan can pick is bitwise the same forward."""
    if tile:
        monkeypatch.setenv("FCE_C3K2_TILE", tile)
    if ystore:
        monkeypatch.setenv("FCE_C3K2_YSTORE", ystore)
    model = cases.seeded_model(cfg, 0).to(device)
    x = torch.rand(batch, 3, imgsz, imgsz, generator=torch.Generator().manual_seed(9)).half().to(device)
    monkeypatch.setenv("FCE_FUSE_C3K2", "1")
    eng = Engine(model, batch, imgsz, device)
    names = [eng.op_info(i)[0] for i in range(eng.num_ops())]
    assert "c3k2_fused" in names
    yf = eng(x).clone()
    monkeypatch.setenv("FCE_FUSE_C3K2", "0")
    eng2 = Engine(model, batch, imgsz, device)
    assert "c3k2_fused" not in [eng2.op_info(i)[0] for i in range(eng2.num_ops())]
    yu = eng2(x).clone()
    torch.cuda.synchronize()
    assert torch.equal(yf, yu)
    monkeypatch.delenv("FCE_FUSE_C3K2")
    ea = Engine(model, batch, imgsz, device)  # auto: both forms recorded, the plan's choice per block
    alts = [i for i in range(ea.num_ops()) if ea.c3k2_form(i) >= 0]
    assert alts and ea.num_ops() == eng2.num_ops() + len(alts)
    assert torch.equal(ea(x).clone(), yu)
    for fused in (False, True):  # every block in each form (graph replay after the switch re-captures)
        for i in alts:
            ea.set_c3k2_form(i, fused)
        assert all(ea.skipped(j) == fused for i in alts for j in range(i - 4, i)) and all(ea.skipped(i) != fused
                                                                                          for i in alts)
        assert torch.equal(ea(x, graph=True).clone(), yu) and torch.equal(ea(x, graph=False).clone(), yu)
    c3 = next(m for m in model.model if isinstance(m, M.C3k2) and not isinstance(m.m[0], M.C3k))
    xi = torch.randn(batch, c3.cv1.conv.in_channels, 48, 40, device=device).half().contiguous(
        memory_format=torch.channels_last)
    with torch.no_grad():
        u = c3(xi)
        monkeypatch.setenv("FCE_FUSE_C3K2", "1")
        f = c3(xi)
    assert torch.equal(u, f)


@pytest.mark.parametrize("batch,imgsz,tiles", [
    (2, 320, None), (1, 640, None), (1, 224, None), (2, 320, ("8,8,4", "8,8,4")), (1, 224, ("8,16,4", "8,8,4")),
    (1, 224, ("8,8,4", "8,8,8"))])
def test_fused_detect_cls_bitwise_equal_to_five_ops(batch, imgsz, tiles, device, monkeypatch):
    """The one-kernel Detect cls branch (csrc/detect_cls.hip) writes bit for bit the scores and best-class keys its five
    ops write (dw 3x3, 1x1, dw 3x3, 1x1, cls 1x1 + sigmoid), whole-graph, on both instantiated levels (n P3 / P4),
    every tile (FCE_DCLS_TILE_64 / _128) and partial edge tiles (224: 28^2 / 14^2 maps).  FCE_FUSE_DCLS=1 forces the
    fused form, =0 records the five ops only, the default records both and the plan keeps the faster; every
    combination of forms is bitwise the same forward."""
    if tiles:
        monkeypatch.setenv("FCE_DCLS_TILE_64", tiles[0])
        monkeypatch.setenv("FCE_DCLS_TILE_128", tiles[1])
    model = cases.seeded_model("yolo11n-fce.yaml", 0).to(device)
    x = torch.rand(batch, 3, imgsz, imgsz, generator=torch.Generator().manual_seed(13)).half().to(device)
    monkeypatch.setenv("FCE_FUSE_DCLS", "1")
    eng = Engine(model, batch, imgsz, device)
    assert [eng.op_info(i)[0] for i in range(eng.num_ops())].count("detect_cls_fused") == 2
    yf, bf = eng(x).clone(), eng.best.clone()
    monkeypatch.setenv("FCE_FUSE_DCLS", "0")
    eng2 = Engine(model, batch, imgsz, device)
    assert "detect_cls_fused" not in [eng2.op_info(i)[0] for i in range(eng2.num_ops())]
    yu, bu = eng2(x).clone(), eng2.best.clone()
    torch.cuda.synchronize()
    assert torch.equal(yf, yu) and torch.equal(bf, bu)
    monkeypatch.delenv("FCE_FUSE_DCLS")
    ea = Engine(model, batch, imgsz, device)
    alts = [i for i in range(ea.num_ops()) if ea.alt_form(i) >= 0 and ea.op_info(i)[0] == "detect_cls_fused"]
    assert len(alts) == 2 and ea.num_ops() == eng2.num_ops() + 2
    assert torch.equal(ea(x).clone(), yu)
    for fused in (False, True):
        for i in alts:
            ea.set_alt_form(i, fused)
        assert all(ea.skipped(j) == fused for i in alts for j in range(i - 5, i)) and all(ea.skipped(i) != fused
                                                                                          for i in alts)
        assert torch.equal(ea(x, graph=True).clone(), yu) and torch.equal(ea.best, bu)
        assert torch.equal(ea(x, graph=False).clone(), yu)


@pytest.mark.parametrize("cfg,batch,imgsz,dtype,sr,nw", [
    ("yolo11n-fce.yaml", 2, 320, torch.float16, None, None), ("yolo11n-fce.yaml", 1, 640, torch.float16, "2", "8"),
    ("yolo11n-fce.yaml", 1, 224, torch.float32, "2", None), ("yolo11n-fce.yaml", 2, 224, torch.uint8, "1", "8"),
    ("yolo11n-fce.yaml", 1, 224, torch.uint8, None, None), ("yolo11n-fce.yaml", 3, 160, torch.float32, "1", "4"),
    ("yolo11s-bifpn.yaml", 2, 256, torch.float16, None, None), ("yolo11s-bifpn.yaml", 1, 224, torch.uint8, "1", "8")])
def test_fused_stem_bitwise_equal_to_two_convs(cfg, batch, imgsz, dtype, sr, nw, device, monkeypatch):
    """The one-kernel stem pair (csrc/stem_fused.hip: Conv(3, 16, 3, 2) -> Conv(16, 32, 3, 2) of the n scale, 3 -> 32 ->
    64 of the s scale with the chunk-major K order, the stem's output in LDS) gives the forward bit for bit what the
    two convs give, for f16 / f32 / u8 network inputs, both group heights
    (FCE_STEM2_SR), both block sizes (FCE_STEM2_NW) and partial fragments (224: 56-wide output rows, 160: 40);
    FCE_FUSE_STEM=1 / 0 / auto as the other
    alternatives, every form of the auto plan the same forward."""
    if sr:
        monkeypatch.setenv("FCE_STEM2_SR", sr)
    if nw:
        monkeypatch.setenv("FCE_STEM2_NW", nw)
    model = cases.seeded_model(cfg, 0).to(device)
    x = torch.rand(batch, 3, imgsz, imgsz, generator=torch.Generator().manual_seed(17))
    x = (x * 255).to(torch.uint8) if dtype == torch.uint8 else x.to(dtype)
    x = x.to(device)
    monkeypatch.setenv("FCE_FUSE_STEM", "1")
    eng = Engine(model, batch, imgsz, device)
    assert [eng.op_info(i)[0] for i in range(eng.num_ops())].count("stem_fused") == 1
    yf = eng(x).clone()
    monkeypatch.setenv("FCE_FUSE_STEM", "0")
    eng2 = Engine(model, batch, imgsz, device)
    assert "stem_fused" not in [eng2.op_info(i)[0] for i in range(eng2.num_ops())]
    yu = eng2(x).clone()
    torch.cuda.synchronize()
    assert torch.equal(yf, yu)
    monkeypatch.delenv("FCE_FUSE_STEM")
    ea = Engine(model, batch, imgsz, device)
    i = [k for k in range(ea.num_ops()) if ea.op_info(k)[0] == "stem_fused"]
    assert i == [2] and ea.alt_form(2) >= 0
    for fused in (False, True):
        ea.set_alt_form(2, fused)
        assert ea.skipped(0) == ea.skipped(1) == fused != ea.skipped(2)
        assert torch.equal(ea(x, graph=True).clone(), yu) and torch.equal(ea(x, graph=False).clone(), yu)
    # the l scale's stem pair (3 -> 64 -> 128) has no instantiation: its two convs only
    ml = cases.seeded_model("yolo11l-fce.yaml", 0).to(device)
    el = Engine(ml, 1, 160, device)
    assert "stem_fused" not in [el.op_info(k)[0] for k in range(el.num_ops())]


@pytest.mark.parametrize("batch,imgsz,nfused", [(2, 640, 5), (1, (608, 640), 5), (3, 320, 3), (1, (320, 640), 5),
                                                  (2, 256, 0)])
def test_fused_bneck_bitwise_equal_to_convs(batch, imgsz, nfused, device, monkeypatch):
    """The one-kernel Bottleneck chain (csrc/bneck.hip: the n scale's C3k pairs L7 / L10 / L24 and the 40^2 neck
    Bottlenecks L15 / L21) gives the forward bit for bit what its 3x3 convs give: full-width bands at 40 and 20 columns,
    partial last bands (608: 38 and 19 rows), the maps without an instantiation (320: L10 / L24 at 10^2; 256: all)
    locked to the convs at plan time even under FCE_FUSE_BNECK=1, and every form the auto plan can pick."""
    model = cases.seeded_model("yolo11n-fce.yaml", 0).to(device)
    hw = (imgsz, imgsz) if isinstance(imgsz, int) else imgsz
    x = torch.rand(batch, 3, *hw, generator=torch.Generator().manual_seed(19)).half().to(device)
    monkeypatch.setenv("FCE_FUSE_BNECK", "1")
    eng = Engine(model, batch, imgsz, device)
    alts = [i for i in range(eng.num_ops()) if eng.op_info(i)[0] == "bneck_fused"]
    assert len(alts) == 5 and sum(eng.alt_form(i) for i in alts) == nfused
    yf = eng(x).clone()
    monkeypatch.setenv("FCE_FUSE_BNECK", "0")
    eng2 = Engine(model, batch, imgsz, device)
    assert "bneck_fused" not in [eng2.op_info(i)[0] for i in range(eng2.num_ops())]
    yu = eng2(x).clone()
    torch.cuda.synchronize()
    assert torch.equal(yf, yu)
    monkeypatch.delenv("FCE_FUSE_BNECK")
    ea = Engine(model, batch, imgsz, device)
    alts = [i for i in range(ea.num_ops()) if ea.op_info(i)[0] == "bneck_fused" and ea.alt_form(i) >= 0]
    assert torch.equal(ea(x).clone(), yu)
    for fused in (False, True):
        for i in alts:
            if fused and nfused < 5:
                try:
                    ea.set_alt_form(i, True)
                except RuntimeError:  # locked: no instantiation for this map width
                    continue
            else:
                ea.set_alt_form(i, fused)
        assert torch.equal(ea(x, graph=True).clone(), yu) and torch.equal(ea(x, graph=False).clone(), yu)


@pytest.mark.parametrize("c,cm,nb,H,W", [(32, 32, 2, 23, 40), (64, 64, 2, 13, 20), (64, 32, 1, 29, 40),
                                         (64, 32, 1, 3, 20), (32, 32, 2, 1, 20)])
def test_fused_bneck_c_abi_views_and_parity(c, cm, nb, H, W, device):
    """fce_bneck_fused through the C-ABI on channel-slice views (in: c of c + 40 channels at offset 24; out: c of c + 16
    at offset 8) with partial bands and maps shorter than a band: equal to the 2 nb fce_conv2d calls (each odd one with
    its Bottleneck's input as the residual) bit for bit, the other output channels untouched, and within the op
    tolerance of an fp64 torch restatement."""
    n = 2
    g = torch.Generator().manual_seed(78)
    specs = [(c, cm), (cm, c)] * nb
    ws, bs, descs, packed = [], [], [], []
    for cin, cout in specs:
        w = torch.randn(cout, cin, 3, 3, generator=g) * (1.5 / (cin * 9) ** 0.5)
        b = torch.randn(cout, generator=g) * 0.2
        d = N.ConvDesc(cin, cout, 3, 1, 1, N.ACT_SILU, 0, N.EPI_STORE, None, 0, 0)
        ws.append(w), bs.append(b.float().to(device)), descs.append(d), packed.append(M.pack_conv(d, w, device))
    xbuf = torch.randn(n, H, W, c + 40, generator=g).half().to(device)
    xt = N.Tensor(xbuf.data_ptr(), N.F16, N.NHWC, n, c, H, W, c + 40, 24)
    stream = torch.cuda.current_stream(device).cuda_stream

    def run(fused):
        ybuf = torch.full((n, H, W, c + 16), float("nan"), dtype=torch.float16, device=device)
        yt = N.Tensor(ybuf.data_ptr(), N.F16, N.NHWC, n, c, H, W, c + 16, 8)
        if fused:
            d = N.BneckDesc()
            d.c, d.c_mid, d.n, d.shortcut = c, cm, nb, 1
            for j in range(2 * nb):
                d.w[j], d.b[j] = packed[j].data_ptr(), bs[j].data_ptr()
            assert N.lib().fce_bneck_supported(C.byref(d)) == 1
            N.call("fce_bneck_fused", C.byref(d), C.byref(xt), C.byref(yt), stream)
        else:
            cur, keep = xt, []
            for j, (cin, cout) in enumerate(specs):
                last = j == 2 * nb - 1
                if last:
                    ot = yt
                else:
                    o = torch.empty(n, H, W, cout, dtype=torch.float16, device=device)
                    keep.append(o)
                    ot = N.Tensor(o.data_ptr(), N.F16, N.NHWC, n, cout, H, W, cout, 0)
                if j % 2 == 0:
                    inp = cur  # this Bottleneck's input: the residual of its second conv
                N.call("fce_conv2d", C.byref(descs[j]), C.byref(cur), packed[j].data_ptr(), bs[j].data_ptr(),
                       C.byref(inp) if j % 2 == 1 else None, C.byref(ot), stream)
                cur = ot
        torch.cuda.synchronize()
        return ybuf.cpu()

    yf, yu = run(True), run(False)
    assert torch.equal(yf[..., 8:8 + c], yu[..., 8:8 + c])
    assert torch.isnan(yf[..., :8]).all() and torch.isnan(yf[..., 8 + c:]).all()
    F = torch.nn.functional
    t = xbuf[..., 24:24 + c].permute(0, 3, 1, 2).double().cpu()
    for b in range(nb):
        h = F.silu(F.conv2d(t, ws[2 * b].double(), bs[2 * b].double().cpu(), padding=1)).half().double()
        t = (F.silu(F.conv2d(h, ws[2 * b + 1].double(), bs[2 * b + 1].double().cpu(), padding=1)) + t).half().double()
    err = _rel(yf[..., 8:8 + c].permute(0, 3, 1, 2), t)
    print(f"OPERR bneck {err:.3e}")
    assert err <= OP_TOL, err
    # a map width without an instantiation fails loudly
    bad = N.Tensor(xbuf.data_ptr(), N.F16, N.NHWC, n, c, H, 24, c + 40, 24)
    d = N.BneckDesc()
    d.c, d.c_mid, d.n, d.shortcut = c, cm, nb, 1
    for j in range(2 * nb):
        d.w[j], d.b[j] = packed[j].data_ptr(), bs[j].data_ptr()
    with pytest.raises(RuntimeError, match="map width"):
        N.call("fce_bneck_fused", C.byref(d), C.byref(bad), C.byref(bad), stream)


@pytest.mark.parametrize("batch,imgsz", [(2, 640), (3, 320), (1, (352, 288))])
def test_fused_pw2_bitwise_equal_to_convs(batch, imgsz, device, monkeypatch):
    """The one-kernel 1x1 pair (csrc/pw2.hip: the n scale's C3k2 cv1 -> C3k cv1 / cv2 and C3k cv3 -> cv2 pairs,
    C2PSA's cv1 -> qkv, proj (+ b) -> ffn[0], ffn[1] (+ x1) -> cv2, and the neck's BiFPN realign (accumulate) -> C3k2
    cv1 pairs) gives the forward bit for bit what the two convs give: partial last pixel tiles (320, 352 x 288), op 1's
    output stored or not as the plan decides, and every form the auto plan can pick."""
    model = cases.seeded_model("yolo11n-fce.yaml", 0).to(device)
    hw = (imgsz, imgsz) if isinstance(imgsz, int) else imgsz
    x = torch.rand(batch, 3, *hw, generator=torch.Generator().manual_seed(23)).half().to(device)
    monkeypatch.setenv("FCE_FUSE_PW2", "1")
    eng = Engine(model, batch, imgsz, device)
    alts = [i for i in range(eng.num_ops()) if eng.op_info(i)[0] == "pw2_fused"]
    assert len(alts) == 11 and all(eng.alt_form(i) == 1 for i in alts)
    yf = eng(x).clone()
    monkeypatch.setenv("FCE_FUSE_PW2", "0")
    eng2 = Engine(model, batch, imgsz, device)
    assert "pw2_fused" not in [eng2.op_info(i)[0] for i in range(eng2.num_ops())]
    yu = eng2(x).clone()
    torch.cuda.synchronize()
    assert torch.equal(yf, yu)
    monkeypatch.delenv("FCE_FUSE_PW2")
    ea = Engine(model, batch, imgsz, device)
    alts = [i for i in range(ea.num_ops()) if ea.op_info(i)[0] == "pw2_fused"]
    assert torch.equal(ea(x).clone(), yu)
    for fused in (False, True):
        for i in alts:
            ea.set_alt_form(i, fused)
        assert torch.equal(ea(x, graph=True).clone(), yu) and torch.equal(ea(x, graph=False).clone(), yu)


@pytest.mark.parametrize("cin1,cout1,cin2,cout2,mode", [(128, 128, 64, 64, "pre"), (64, 64, 192, 128, "post"),
                                                       (128, 128, 128, 256, "res"), (256, 128, 256, 256, "res_post"),
                                                       (128, 64, 64, 128, "accum"), (128, 32, 32, 128, "wstore")])
def test_fused_pw2_c_abi_views_and_parity(cin1, cout1, cin2, cout2, mode, device):
    """fce_pw2 through the C-ABI on channel-slice views of a 2 x 17 x 23 map (a partial 64-pixel tile): "pre" -- op 2
    reads the second half of op 1's output (with a duplicate store of its upper half), "post" -- op 2 reads [E | h] with
    E from HBM, "res" / "res_post" -- op 1 without activation plus a residual (Attention.proj, ffn[1]), "accum" /
    "wstore" -- op 1 a BiFPN realign conv (weighted accumulate into / weighted store of the sum op 2 reads whole); bit for
    bit the two fce_conv2d calls, the channels outside the views untouched, h stored or not, and within the op
    tolerance of an fp64 restatement."""
    n, H, W = 2, 17, 23
    g = torch.Generator().manual_seed(79)
    acts = (N.ACT_NONE if mode.startswith("res") else N.ACT_SILU, N.ACT_SILU)
    fw = torch.tensor([0.7, -0.2, 1.3])
    fwd = fw.to(device)
    epi1 = {"accum": N.EPI_ACCUM, "wstore": N.EPI_WSTORE}.get(mode, N.EPI_STORE)
    ws, bs, descs, packed = [], [], [], []
    for j, (cin, cout, act) in enumerate(((cin1, cout1, acts[0]), (cin2, cout2, acts[1]))):
        w = torch.randn(cout, cin, 1, 1, generator=g) * (1.5 / cin ** 0.5)
        b = torch.randn(cout, generator=g) * 0.2
        bifpn = j == 0 and epi1 != N.EPI_STORE
        d = N.ConvDesc(cin, cout, 1, 1, 1, act, 0, epi1 if j == 0 else N.EPI_STORE, fwd.data_ptr() if bifpn else None,
                       3 if bifpn else 0, 2 if bifpn else 0)
        ws.append(w), bs.append(b.float().to(device)), descs.append(d), packed.append(M.pack_conv(d, w, device))
    xbuf = torch.randn(n, H, W, cin1 + 32, generator=g).half().to(device)
    x1 = N.Tensor(xbuf.data_ptr(), N.F16, N.NHWC, n, cin1, H, W, cin1 + 32, 16)
    # the shared buffer: h at hoff, op 2's input x2 at x2off (overlapping h)
    if mode == "pre":
        width, hoff, x2off = cout1 + 16, 8, 8 + cout1 - cin2
    elif mode in ("post", "res_post"):
        width, x2off = cin2 + 24, 16
        hoff = x2off + cin2 - cout1
    else:
        width, hoff, x2off = cout1 + 8, 8, 8
    rbuf = torch.randn(n, H, W, cout1 + 8, generator=g).half().to(device)
    r1 = N.Tensor(rbuf.data_ptr(), N.F16, N.NHWC, n, cout1, H, W, cout1 + 8, 8) if mode.startswith("res") else None
    base = torch.randn(n, H, W, width, generator=g).half().to(device)
    stream = torch.cuda.current_stream(device).cuda_stream
    dup_c, dup_lo = (cout2 // 2, cout2 // 2) if mode == "pre" else (0, 0)

    def run(fused, h_store):
        buf = base.clone()
        ybuf = torch.full((n, H, W, cout2 + 8), float("nan"), dtype=torch.float16, device=device)
        dbuf = torch.full((n, H, W, max(dup_c, 8)), float("nan"), dtype=torch.float16, device=device)
        ht = N.Tensor(buf.data_ptr(), N.F16, N.NHWC, n, cout1, H, W, width, hoff)
        x2 = N.Tensor(buf.data_ptr(), N.F16, N.NHWC, n, cin2, H, W, width, x2off)
        yt = N.Tensor(ybuf.data_ptr(), N.F16, N.NHWC, n, cout2, H, W, cout2 + 8, 8)
        dt = N.Tensor(dbuf.data_ptr(), N.F16, N.NHWC, n, dup_c, H, W, max(dup_c, 8), 0) if dup_c else None
        if fused:
            d = N.Pw2Desc()
            d.cin1, d.cout1, d.cin2, d.cout2 = cin1, cout1, cin2, cout2
            for j in range(2):
                d.act[j], d.w[j], d.b[j] = acts[j], packed[j].data_ptr(), bs[j].data_ptr()
            if epi1 != N.EPI_STORE:
                d.epi1, d.fw, d.fn, d.fi = epi1, fwd.data_ptr(), 3, 2
            assert N.lib().fce_pw2_supported(C.byref(d)) == 1
            N.call("fce_pw2", C.byref(d), C.byref(x1), C.byref(r1) if r1 else None, C.byref(ht), int(h_store),
                   C.byref(x2), None, C.byref(yt), C.byref(dt) if dt else None, dup_lo, stream)
        else:
            N.call("fce_conv2d", C.byref(descs[0]), C.byref(x1), packed[0].data_ptr(), bs[0].data_ptr(),
                   C.byref(r1) if r1 else None, C.byref(ht), stream)
            if dt:
                N.call("fce_conv2d_variant_dup", C.byref(descs[1]), C.byref(x2), packed[1].data_ptr(), bs[1].data_ptr(),
                       None, C.byref(yt), -1, C.byref(dt), dup_lo, stream)
            else:
                N.call("fce_conv2d", C.byref(descs[1]), C.byref(x2), packed[1].data_ptr(), bs[1].data_ptr(), None,
                       C.byref(yt), stream)
        torch.cuda.synchronize()
        return buf.cpu(), ybuf.cpu(), dbuf.cpu()

    bu, yu, du = run(False, True)
    bf, yf, df = run(True, True)
    assert torch.equal(yf[..., 8:], yu[..., 8:]) and torch.equal(bf, bu)
    assert not dup_c or torch.equal(df[..., :dup_c], du[..., :dup_c])
    assert torch.isnan(yf[..., :8]).all()
    b0, y0, _ = run(True, False)  # h not stored: nothing is written into the shared buffer, y is the same
    assert torch.equal(y0[..., 8:], yu[..., 8:]) and torch.equal(b0, base.cpu())
    F = torch.nn.functional
    t = F.conv2d(xbuf[..., 16:16 + cin1].permute(0, 3, 1, 2).double().cpu(), ws[0].double(), bs[0].double().cpu())
    t = F.silu(t) if acts[0] == N.ACT_SILU else t
    if r1:
        t = t + rbuf[..., 8:8 + cout1].permute(0, 3, 1, 2).double().cpu()
    hb = base.cpu().permute(0, 3, 1, 2).double().clone()
    if epi1 != N.EPI_STORE:
        r = fw.clamp_min(0).double()
        t = r[2] / (r.sum() + 1e-4) * t + (hb[:, hoff:hoff + cout1] if epi1 == N.EPI_ACCUM else 0)
    hb[:, hoff:hoff + cout1] = t.half().double()
    ref = F.silu(F.conv2d(hb[:, x2off:x2off + cin2], ws[1].double(), bs[1].double().cpu()))
    err = _rel(yf[..., 8:8 + cout2].permute(0, 3, 1, 2), ref)
    print(f"OPERR pw2 {mode} {err:.3e}")
    assert err <= OP_TOL, err


def test_fused_stem_kept_out_where_it_does_not_fit(device, monkeypatch):
    """The fused stem pair is built for input widths <= 640: at 704 the plan keeps the two convs (locked: the fused form
    cannot be selected, not even with FCE_FUSE_STEM=1), and the forward equals the one without the alternative."""
    model = cases.seeded_model("yolo11n-fce.yaml", 0).to(device)
    x = torch.rand(1, 3, 704, 704, generator=torch.Generator().manual_seed(5)).half().to(device)
    monkeypatch.setenv("FCE_FUSE_STEM", "1")
    eng = Engine(model, 1, 704, device)
    assert eng.op_info(2)[0] == "stem_fused" and eng.alt_form(2) == 0 and not eng.skipped(0) and eng.skipped(2)
    with pytest.raises(RuntimeError, match="cannot run"):
        eng.set_alt_form(2, True)
    y = eng(x).clone()
    monkeypatch.setenv("FCE_FUSE_STEM", "0")
    y0 = Engine(model, 1, 704, device)(x).clone()
    torch.cuda.synchronize()
    assert torch.equal(y, y0)


def test_fused_stem_locked_when_another_layer_reads_the_stem(device, monkeypatch):
    """The fused stem pair skips writing the stem's output, so the plan locks it out when any op other than the second
    conv reads that output: here layer 2 is a second conv from layer 0 (a saved layer), concatenated with layer 1.
    Even FCE_FUSE_STEM=1 keeps the two convs, and the forward equals the one planned without the alternative."""
    from fce_yolo_amd.parser import DetectionModel
    from fce_yolo_amd.weights import seeded_state_dict

    d = {"nc": 80, "scales": {"n": [0.50, 0.25, 1024]}, "scale": "n",
         "backbone": [[-1, 1, "Conv", [64, 3, 2]], [-1, 1, "Conv", [128, 3, 2]], [0, 1, "Conv", [128, 3, 2]],
                      [[1, 2], 1, "Concat", [1]], [-1, 1, "Conv", [256, 3, 2]], [-1, 1, "Conv", [512, 3, 2]],
                      [-1, 1, "Conv", [1024, 3, 2]]],
         "head": [[[4, 5, 6], 1, "Detect", ["nc"]]]}
    model = DetectionModel(d)
    assert 0 in model.save
    model.load_state_dict(seeded_state_dict([(k, v.shape) for k, v in model.state_dict().items()], 0))
    model = model.eval().to(device)
    x = torch.rand(1, 3, 256, 256, generator=torch.Generator().manual_seed(6)).half().to(device)
    monkeypatch.setenv("FCE_FUSE_STEM", "1")
    # the lowering does not record the alternative when layer 0 is saved (modules.stem_alt) ...
    eng = Engine(model, 1, 256, device)
    assert "stem_fused" not in [eng.op_info(i)[0] for i in range(eng.num_ops())]
    y1 = eng(x).clone()
    # ... and if it were recorded, the plan-time access check (fce_net_plan) locks it out
    from fce_yolo_amd import modules as M

    real = M.stem_alt
    monkeypatch.setattr(M, "stem_alt", lambda be, m0, m1, first, saved: real(be, m0, m1, first, False))
    eng = Engine(model, 1, 256, device)
    names = [eng.op_info(i)[0] for i in range(eng.num_ops())]
    assert names.count("stem_fused") == 1
    i = names.index("stem_fused")
    assert eng.alt_form(i) == 0 and not eng.skipped(0) and not eng.skipped(1) and eng.skipped(i)
    with pytest.raises(RuntimeError, match="cannot run"):
        eng.set_alt_form(i, True)
    y = eng(x).clone()
    monkeypatch.setenv("FCE_FUSE_STEM", "0")
    y0 = Engine(model, 1, 256, device)(x).clone()
    torch.cuda.synchronize()
    assert torch.equal(y, y0) and torch.equal(y1, y0)


def test_fused_detect_cls_unknown_tile_is_an_error(device, monkeypatch):
    """FCE_DCLS_TILE_64 / _128 name a tile of that instantiation; anything else fails loudly."""
    model = cases.seeded_model("yolo11n-fce.yaml", 0).to(device)
    x = torch.rand(1, 3, 160, 160, generator=torch.Generator().manual_seed(9)).half().to(device)
    monkeypatch.setenv("FCE_FUSE_DCLS", "1")
    monkeypatch.setenv("FCE_DCLS_TILE_128", "8,16,8")
    with pytest.raises(RuntimeError, match="FCE_DCLS_TILE_128"):
        eng = Engine(model, 1, 160, device)
        eng(x)
        torch.cuda.synchronize()


def test_fused_detect_cls_c_abi_views_and_parity(device):
    """fce_detect_cls through the C-ABI on a channel-slice input view (64 of 96 channels at offset 16), a 19 x 37
    map (partial tiles both ways) and a level block inside a wider anchor range: equal to the five fce_conv2d /
    fce_conv2d_detect calls bit for bit (scores and keys), the other anchors untouched, and within the op tolerance
    of an fp64 torch restatement of the branch."""
    n, c0, c3, nc, H, W = 2, 64, 80, 80, 19, 37
    g = torch.Generator().manual_seed(77)
    specs = [(c0, c0, 3, c0, N.ACT_SILU), (c0, c3, 1, 1, N.ACT_SILU), (c3, c3, 3, c3, N.ACT_SILU),
             (c3, c3, 1, 1, N.ACT_SILU), (c3, nc, 1, 1, N.ACT_NONE)]
    ws, bs, descs, packed = [], [], [], []
    for cin, cout, k, grp, act in specs:
        w = torch.randn(cout, cin // grp, k, k, generator=g) * (1.5 / (cin // grp * k * k) ** 0.5)
        b = torch.randn(cout, generator=g) * 0.2
        d = N.ConvDesc(cin, cout, k, 1, grp, act, 0, N.EPI_STORE, None, 0, 0)
        ws.append(w), bs.append(b.float().to(device)), descs.append(d), packed.append(M.pack_conv(d, w, device))
    xbuf = torch.randn(n, H, W, 96, generator=g).half().to(device)
    xt = N.Tensor(xbuf.data_ptr(), N.F16, N.NHWC, n, c0, H, W, 96, 16)
    A, a0 = H * W + 50, 20
    stream = torch.cuda.current_stream(device).cuda_stream

    def run(fused):
        pred = torch.full((n, 4 + nc, A), float("nan"), device=device)
        best = torch.zeros(n, A, dtype=torch.int64, device=device)
        e = N.DetectEpi(pred.data_ptr(), A, a0, nc, 16, 1, 8.0, best.data_ptr())
        if fused:
            d = N.DclsDesc()
            d.c0, d.c3, d.nc = c0, c3, nc
            for j in range(5):
                d.w[j], d.b[j] = packed[j].data_ptr(), bs[j].data_ptr()
            N.call("fce_detect_cls", C.byref(d), C.byref(xt), C.byref(e), stream)
        else:
            cur = xt
            keep = []
            for j in range(4):
                y = torch.empty(n, H, W, specs[j][1], dtype=torch.float16, device=device)
                keep.append(y)
                yt = N.Tensor(y.data_ptr(), N.F16, N.NHWC, n, specs[j][1], H, W, specs[j][1], 0)
                N.call("fce_conv2d", C.byref(descs[j]), C.byref(cur), packed[j].data_ptr(), bs[j].data_ptr(), None,
                       C.byref(yt), stream)
                cur = yt
            N.call("fce_conv2d_detect", C.byref(descs[4]), C.byref(cur), packed[4].data_ptr(), bs[4].data_ptr(),
                   C.byref(e), stream)
        torch.cuda.synchronize()
        return pred.cpu(), best.cpu()

    pf, bf = run(True)
    pu, bu = run(False)
    assert torch.equal(pf[:, 4:, a0:a0 + H * W], pu[:, 4:, a0:a0 + H * W]) and torch.equal(bf, bu)
    assert torch.isnan(pf[:, :4]).all() and torch.isnan(pf[:, 4:, :a0]).all() and torch.isnan(pf[:, 4:, a0 + H * W:]).all()
    assert (bf[:, :a0] == 0).all() and (bf[:, a0 + H * W:] == 0).all() and (bf[:, a0:a0 + H * W] != 0).all()
    t = xbuf[..., 16:16 + c0].permute(0, 3, 1, 2).double().cpu()
    F = torch.nn.functional
    for j, (cin, cout, k, grp, act) in enumerate(specs):
        t = F.conv2d(t, ws[j].double(), bs[j].double().cpu(), padding=k // 2, groups=grp)
        t = F.silu(t) if act == N.ACT_SILU else torch.sigmoid(t)
        if j < 4:
            t = t.half().double()  # the unfused ops store fp16 intermediates
    ref = t.reshape(n, nc, H * W)
    err = (pf[:, 4:, a0:a0 + H * W].double() - ref).abs().max().item()
    print(f"OPERR detect_cls {err:.3e}")
    assert err <= 2e-3, err


@pytest.mark.parametrize("cfg,mut,batch,imgsz", [("yolo11n-fce.yaml", None, 2, 320), ("yolo11s-bifpn.yaml", None, 2, 256)])
def test_c2f_dense_chunk_copy_bitwise(cfg, mut, batch, imgsz, device, monkeypatch):
    """With FCE_DUP=1 whole-graph lowering stores the chunk a C2f / C3k2's first block reads densely from cv1's
    epilogue (fce_net_add_conv_dup); the forward is bitwise the one that reads it as a slice of the concat
    record (the default)."""
    model = cases.seeded_model(cfg, 0, mut).to(device)
    x = torch.rand(batch, 3, imgsz, imgsz, generator=torch.Generator().manual_seed(21)).half().to(device)
    monkeypatch.setenv("FCE_DUP", "1")
    e1 = Engine(model, batch, imgsz, device)
    y1 = e1(x).clone()
    monkeypatch.delenv("FCE_DUP")
    e0 = Engine(model, batch, imgsz, device)
    y0 = e0(x).clone()
    torch.cuda.synchronize()
    assert e1.num_ops() == e0.num_ops() and e1.arena_bytes() > e0.arena_bytes()
    assert torch.equal(y1, y0)


@pytest.mark.parametrize("cfg,mut,batch,imgsz,rows", [
    ("yolo11n-fce.yaml", None, 32, 640, (0, 17, 31)),
    ("yolo11s-bifpn.yaml", None, 32, 640, (0, 31)),
    ("yolo11l-fce.yaml", None, 32, 640, (0, 31)),
    ("yolo11m-fce.yaml", cases.heads8, 16, 1280, (0, 15)),
])
def test_batch_invariance(cfg, mut, batch, imgsz, rows, device):
    """Size-independent property at every BASELINE GPU config's bench batch (n32, s32, l32 = l256's per-GPU
    shard, m-h8 16 @1280): an image's outputs do not depend on its batch -- the autotuned bs-B executor's
    rows equal a bs-1 executor's bit for bit (bs-1 parity is pinned by the full-size reference fixtures)."""
    model = cases.seeded_model(cfg, 0, mut).to(device)
    g = torch.Generator().manual_seed(7)
    xb = torch.rand(batch, 3, imgsz, imgsz, generator=g).half().to(device)
    eb = Engine(model, batch, imgsz, device)
    yb = eb(xb).clone()
    eb.close()
    e1 = Engine(model, 1, imgsz, device)
    for i in rows:
        y1 = e1(xb[i:i + 1].contiguous()).clone()
        assert torch.equal(y1[0], yb[i]), i
    assert torch.isfinite(yb).all()
    e1.close()


def test_640_matches_reference_digest(e2e_fx, device):
    fx = e2e_fx.group("yolo11n-fce_640_b1")
    model = cases.seeded_model("yolo11n-fce.yaml", 0).to(device)
    x = torch.rand(1, 3, 640, 640, generator=torch.Generator().manual_seed(640))
    y = Engine(model, 1, 640, device)(x.half().to(device)).cpu().numpy()
    ref = fx["y_slice"]
    got = y[:, :, ::37]
    assert np.abs(got[:, :4] - ref[:, :4]).max() <= BOX_TOL * np.abs(ref[:, :4]).max()
    assert np.abs(got[:, 4:] - ref[:, 4:]).max() <= CLS_TOL


@pytest.fixture(params=["v1", "v2"])
def nms_path(request, monkeypatch):
    """Both device NMS paths: the one-workgroup kernel (default) and the multi-workgroup one (FCE_NMS_V2=1)."""
    if request.param == "v2":
        monkeypatch.setenv("FCE_NMS_V2", "1")
    return request.param


@pytest.mark.parametrize("name", ["designed_small", "designed_many", "none", "saturated_maxdet"])
def test_nms_bit_exact_vs_reference(name, nms_fx, device, nms_path):
    fx = nms_fx.group(name)
    pred = torch.from_numpy(fx["pred"]).to(device)
    dets, keep = non_max_suppression(pred, 0.25, 0.7, 300, return_idxs=True)
    for b in range(pred.shape[0]):
        assert np.array_equal(keep[b].cpu().numpy(), fx[f"keep{b}"].reshape(-1).astype(np.int64)), b
        assert np.array_equal(dets[b].cpu().numpy(), fx[f"det{b}"].reshape(-1, 6)), b


@pytest.mark.parametrize("name", NMS_OPT_CASES)
def test_nms_options_bit_exact_vs_reference(name, nms_opts_fx, device, nms_path):
    """fce_nms_ex (classes / agnostic / multi_label, nms.py:116-141): kept anchors and rows bit-exact against the
    reference's outputs; with best-class keys built like the Detect epilogue's too (ignored by multi_label)."""
    pred, opts, exp = nms_opt_case(nms_opts_fx, name)
    pt = torch.from_numpy(pred).to(device)
    dets, keep = non_max_suppression(pt, 0.25, 0.7, 300, return_idxs=True, **opts)
    for b, (d, k) in enumerate(exp):
        assert np.array_equal(keep[b].cpu().numpy(), k), b
        assert np.array_equal(dets[b].cpu().numpy(), d), b
    sc, cl = pt[:, 4:].max(1)  # first maximum, like the cls epilogue's keys
    best = ((sc.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF) << 32) | (0xFFFFFFFF - cl)
    b_, a_ = pred.shape[0], pred.shape[2]
    nms = NMS(b_, a_, pred.shape[1] - 4, device, 0.25, 0.7, 300, **opts)
    nms(pt, best.contiguous())
    d2, k2 = nms.results()
    for b, (d, k) in enumerate(exp):
        assert np.array_equal(k2[b].cpu().numpy(), k) and np.array_equal(d2[b].cpu().numpy(), d), b


def test_nms_on_reference_model_output(e2e_fx, device):
    fx = e2e_fx.group("yolo11n-fce_160_b2")
    dets, keep = non_max_suppression(torch.from_numpy(fx["y"]).to(device), return_idxs=True)
    for b in range(2):
        assert np.array_equal(keep[b].cpu().numpy(), fx[f"nms_keep{b}"].astype(np.int64))
        assert np.array_equal(dets[b].cpu().numpy(), fx[f"nms_det{b}"])


def test_nms_on_gpu_predictions_matches_oracle(e2e_fx, device, nms_path):
    key = "yolo11n-fce_320_b1"
    fx = e2e_fx.group(key)
    _, _, _, y = _engine_run(key, fx, device)
    for conf in (0.25, 0.2, 0.1):
        dets, keep = non_max_suppression(y, conf, 0.7, return_idxs=True)
        odets, okeep = nms_oracle.non_max_suppression(y.cpu().numpy(), conf, 0.7)
        assert np.array_equal(keep[0].cpu().numpy(), okeep[0])
        assert np.array_equal(dets[0].cpu().numpy(), odets[0])


def test_nms_large_candidate_set_global_sort(device, nms_path):
    """> 8192 candidates takes the workspace (global-memory) bitonic sort path; max_nms truncation."""
    rng = np.random.default_rng(3)
    A = 33600
    p = np.zeros((1, 84, A), np.float32)
    p[0, 0] = rng.random(A) * 1280
    p[0, 1] = rng.random(A) * 1280
    p[0, 2:4] = rng.random((2, A)) * 50 + 2
    p[0, 4 + rng.integers(0, 80, A), np.arange(A)] = (0.3 + 0.7 * rng.permutation(A) / A).astype(np.float32)
    for max_nms in (30000, 5000):
        dets, keep = non_max_suppression(torch.from_numpy(p).to(device), max_nms=max_nms, return_idxs=True)
        od, ok = nms_oracle.non_max_suppression(p, max_nms=max_nms)
        assert np.array_equal(keep[0].cpu().numpy(), ok[0]) and np.array_equal(dets[0].cpu().numpy(), od[0])



@pytest.mark.parametrize("case", ["group_done", "group_runs_out", "group_is_everything"])
def test_nms_equal_top_score_group(case, device, nms_path):
    """>= max_det candidates share the top score (saturated sigmoids): ties resolved by anchor order, whether the
    greedy stops inside the tied group, runs through it (one pile of near-identical boxes), or the whole candidate
    set is tied.  Bit-exact vs the oracle."""
    rng = np.random.default_rng({"group_done": 7, "group_runs_out": 8, "group_is_everything": 9}[case])
    A, nc = 6000, 4
    p = np.zeros((2, 4 + nc, A), np.float32)
    for b in range(2):
        p[b, 0:2] = rng.random((2, A)) * 600 + 20
        p[b, 2:4] = rng.random((2, A)) * 40 + 8
        cls = rng.integers(0, nc, A)
        sc = (0.3 + 0.6 * rng.random(A)).astype(np.float32)
        top = rng.choice(A, {"group_done": 2000, "group_runs_out": 700, "group_is_everything": A}[case], replace=False)
        sc[top] = 1.0
        if case == "group_runs_out":  # the top group is one pile of near-identical boxes: almost all suppressed
            p[b, 0, top], p[b, 1, top] = 300 + rng.random(len(top)), 300 + rng.random(len(top))
            p[b, 2, top], p[b, 3, top] = 50, 50
            cls[top] = 0
        p[b, 4 + cls, np.arange(A)] = sc
    pt = torch.from_numpy(p).to(device)
    for max_det in (300, 100):
        dets, keep = non_max_suppression(pt, 0.25, 0.7, max_det, return_idxs=True)
        od, ok = nms_oracle.non_max_suppression(p, 0.25, 0.7, max_det)
        for b in range(2):
            assert np.array_equal(keep[b].cpu().numpy(), ok[b]), (b, max_det)
            assert np.array_equal(dets[b].cpu().numpy(), od[b]), (b, max_det)


def _iou_fp32(b1, b2):
    """The reference's IoU (nms.py:276-291) in fp32 on xywh pairs (xywh2xyxy as ops.py:224-240), vectorised."""
    f = np.float32
    x1 = [b1[0] - b1[2] / f(2), b1[1] - b1[3] / f(2), b1[0] + b1[2] / f(2), b1[1] + b1[3] / f(2)]
    x2 = [b2[0] - b2[2] / f(2), b2[1] - b2[3] / f(2), b2[0] + b2[2] / f(2), b2[1] + b2[3] / f(2)]
    a1 = (x1[2] - x1[0]) * (x1[3] - x1[1])
    a2 = (x2[2] - x2[0]) * (x2[3] - x2[1])
    ww = np.maximum(np.minimum(x1[2], x2[2]) - np.maximum(x1[0], x2[0]), f(0))
    hh = np.maximum(np.minimum(x1[3], x2[3]) - np.maximum(x1[1], x2[1]), f(0))
    inter = ww * hh
    return inter / ((a1 + a2) - inter)


@pytest.mark.parametrize("thr", [0.7, 0.45])
def test_nms_iou_at_the_threshold(thr, device, nms_path):
    """Box pairs whose fp32 IoU lies within a few ulps of iou_thres, on both sides (2e5 random pairs per slot, the
    closest kept; measured ~8 ulps at 0.7): the kernel
    decides `IoU > thr` without the IEEE division unless inter is within 2^-20 of thr * union (nms.py:276-291
    computes the quotient), so these pairs take the exact fallback.  Kept indices and rows bit-exact vs the oracle."""
    rng = np.random.default_rng(int(thr * 100))
    f = np.float32
    slots, tries = 64, 200_000
    A = 2 * slots
    p = np.zeros((1, 5, A), f)
    got = []
    for s_ in range(slots):
        cx, cy = f(30 + 90 * (s_ % 8)), f(30 + 90 * (s_ // 8))
        w1, h1 = rng.uniform(20, 40, tries).astype(f), rng.uniform(20, 40, tries).astype(f)
        w2, h2 = (w1 * rng.uniform(0.8, 1.2, tries)).astype(f), (h1 * rng.uniform(0.8, 1.2, tries)).astype(f)
        dx, dy = rng.uniform(-8, 8, tries).astype(f), rng.uniform(-8, 8, tries).astype(f)
        b1 = [np.full(tries, cx, f), np.full(tries, cy, f), w1, h1]
        b2 = [cx + dx, cy + dy, w2, h2]
        iou = _iou_fp32(b1, b2)
        want = [-1, 0, 1][s_ % 3]  # just below, as close as possible, just above
        d = (iou.astype(np.float64) - thr) * [1, 1, -1][s_ % 3]
        d = np.where((d <= 0) if want != 0 else np.ones_like(d, bool), np.abs(d), np.inf)
        k = int(np.argmin(d))
        got.append(float(iou[k]))
        for j, b in enumerate((b1, b2)):
            p[0, :4, 2 * s_ + j] = [b[0][k], b[1][k], b[2][k], b[3][k]]
        p[0, 4, 2 * s_] = f(0.9)
        p[0, 4, 2 * s_ + 1] = f(0.8)
    got = np.array(got)
    assert np.abs(got - thr).max() < 1e-5 and (got > f(thr)).any() and (got <= f(thr)).any()
    pt = torch.from_numpy(p).to(device)
    dets, keep = non_max_suppression(pt, 0.25, thr, 300, return_idxs=True)
    od, ok = nms_oracle.non_max_suppression(p, 0.25, thr)
    assert np.array_equal(keep[0].cpu().numpy(), ok[0]) and np.array_equal(dets[0].cpu().numpy(), od[0])
    assert len(ok[0]) == slots + int((got <= f(thr)).sum())  # every pair: the second box survives iff IoU <= thr


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_nms_clustered_suppression_chains(seed, device, nms_path):
    """Heavy, chained suppression: jittered boxes around a few centres, few classes, tied (quantised)
    scores; several IoU thresholds and max_det values.  Kept indices and rows bit-exact vs the oracle."""
    rng = np.random.default_rng(100 + seed)
    B, A, nc = 4, (4000, 1500, 900)[seed], 3  # full sort / 2048-slot / 1024-slot small-set sort
    p = np.zeros((B, 4 + nc, A), np.float32)
    for b in range(B):
        centres = rng.random((12, 2)) * 600 + 20
        k = rng.integers(0, 12, A)
        p[b, 0:2] = (centres[k] + rng.normal(0, 6, (A, 2))).T
        p[b, 2:4] = (rng.random((A, 2)) * 30 + 40).T
        cls = rng.integers(0, nc, A)
        p[b, 4 + cls, np.arange(A)] = np.round(rng.random(A) * 64) / 64  # ties on purpose
    pt = torch.from_numpy(p).to(device)
    for iou, max_det in ((0.7, 300), (0.5, 300), (0.3, 50), (0.9, 1000), (0.7, 7)):
        dets, keep = non_max_suppression(pt, 0.25, iou, max_det, return_idxs=True)
        od, ok = nms_oracle.non_max_suppression(p, 0.25, iou, max_det=max_det)
        for b in range(B):
            assert np.array_equal(keep[b].cpu().numpy(), ok[b]), (iou, max_det, b)
            assert np.array_equal(dets[b].cpu().numpy(), od[b]), (iou, max_det, b)


@pytest.mark.parametrize("max_nms,max_det", [(1500, 300), (3000, 300), (30000, 3000), (30000, 40)])
def test_nms_sorted_prefix_select(max_nms, max_det, device, nms_path):
    """2049..8192 candidates: the first 2048 of the order (score desc, position asc) are selected and sorted
    alone -- a radix select over the score bits gives the 2048-th score T, every candidate above T is taken and
    of those scoring exactly T the first `need` in position order (a ballot scan over the candidates' chunk /
    wave order) -- with the full sort when the greedy runs out of the prefix (max_det 3000; heavy suppression
    with max_det 40) or max_nms truncates inside it (1500).  Most scores tied, the tied group straddling the
    2048-th position.  Bit-exact vs the oracle."""
    rng = np.random.default_rng(21)
    B, A, nc = 2, 7000, 5
    p = np.zeros((B, 4 + nc, A), np.float32)
    tight = max_det == 40  # one class, 24 piles: the 40th kept box at sorted depth 2324 / 1463 (past / inside 2048)
    for b in range(B):
        c = rng.random((24 if tight else 60, 2)) * 600 + 20
        k = rng.integers(0, len(c), A)
        p[b, 0:2] = (c[k] + rng.normal(0, 1.5 if tight else 12, (A, 2))).T
        p[b, 2:4] = (rng.random((A, 2)) * (2 if tight else 10) + 40).T
        sc = np.where(rng.random(A) < 0.6, np.float32(0.875), 0.3 + 0.69 * rng.random(A)).astype(np.float32)
        p[b, 4 + rng.integers(0, 1 if tight else nc, A), np.arange(A)] = sc
    pt = torch.from_numpy(p).to(device)
    dets, keep = non_max_suppression(pt, 0.25, 0.7, max_det, max_nms=max_nms, return_idxs=True)
    od, ok = nms_oracle.non_max_suppression(p, 0.25, 0.7, max_det=max_det, max_nms=max_nms)
    for b in range(B):
        assert np.array_equal(keep[b].cpu().numpy(), ok[b]), b
        assert np.array_equal(dets[b].cpu().numpy(), od[b]), b


@pytest.mark.parametrize("n1", [0, 1, 2048, 2049, 5000])
def test_nms_empty_and_small_images_beside_a_large_one(n1, device, nms_path):
    """Images with no candidate, one, exactly 2048 (the sorted-head capacity) and just past it, in one batch with a
    5000-candidate image: the empty image takes no select / sort path at all (an empty set once ran the 2048-prefix
    radix select over stale LDS), and every image is bit-exact vs the oracle."""
    rng = np.random.default_rng(5)
    B, A, nc = 3, 6000, 4
    p = np.zeros((B, 4 + nc, A), np.float32)
    for b, n in enumerate((0, n1, 5000)):
        p[b, 0:2] = rng.random((2, A)) * 600
        p[b, 2:4] = rng.random((2, A)) * 30 + 4
        idx = rng.permutation(A)[:n]
        p[b, 4 + rng.integers(0, nc, n), idx] = np.where(rng.random(n) < 0.5, np.float32(0.75),
                                                         0.3 + 0.6 * rng.random(n)).astype(np.float32)
    pt = torch.from_numpy(p).to(device)
    dets, keep = non_max_suppression(pt, 0.25, 0.7, 300, return_idxs=True)
    od, ok = nms_oracle.non_max_suppression(p, 0.25, 0.7, max_det=300)
    assert len(ok[0]) == 0 and keep[0].numel() == 0
    for b in range(B):
        assert np.array_equal(keep[b].cpu().numpy(), ok[b]), b
        assert np.array_equal(dets[b].cpu().numpy(), od[b]), b


@pytest.mark.parametrize("case", ["bench_like", "unbanded", "one_class_heavy"])
def test_nms_top_selection_and_class_buckets(case, device, nms_path):
    """The large-candidate-set paths against the oracle: top-1024 selection (MSB radix select on tied
    scores) with the full-sort fallback, and the class-bucketed kept lists (exact only inside the class
    bands; `unbanded` breaks the band condition with max_wh below the box extent)."""
    rng = np.random.default_rng(11)
    B, A, nc = 3, 8400, 80
    p = np.zeros((B, 4 + nc, A), np.float32)
    for b in range(B):
        p[b, 0:2] = rng.random((2, A)) * 640
        p[b, 2:4] = rng.random((2, A)) * 120 + 8
        if case == "one_class_heavy":  # 2 classes, clustered: heavy suppression, long class lists
            cls = rng.integers(0, 2, A)
            c = rng.random((20, 2)) * 600 + 20
            k = rng.integers(0, 20, A)
            p[b, 0:2] = (c[k] + rng.normal(0, 8, (A, 2))).T
        else:
            cls = rng.integers(0, nc, A)
        sc = np.where(rng.random(A) < 0.7, 1.0, rng.random(A)).astype(np.float32)  # saturated, like the bench
        p[b, 4 + cls, np.arange(A)] = sc
    max_wh = 64.0 if case == "unbanded" else 7680.0
    pt = torch.from_numpy(p).to(device)
    for iou, max_det in ((0.7, 300), (0.45, 300), (0.7, 1000)):
        dets, keep = non_max_suppression(pt, 0.25, iou, max_det, max_wh=max_wh, return_idxs=True)
        od, ok = nms_oracle.non_max_suppression(p, 0.25, iou, max_det=max_det, max_wh=max_wh)
        for b in range(B):
            assert np.array_equal(keep[b].cpu().numpy(), ok[b]), (case, iou, max_det, b)
            assert np.array_equal(dets[b].cpu().numpy(), od[b]), (case, iou, max_det, b)


def test_fused_best_class_keys_match_pred_and_nms(device):
    """The cls epilogue's per-anchor best-class keys (atomic max, box epilogue zeroes) equal torch.max over
    the pred rows (first maximum), and the NMS fed with them equals the NMS that does its own arg-max."""
    model = cases.seeded_model("yolo11n-fce.yaml", 0).to(device)
    B, S = 4, 320
    eng = Engine(model, B, S, device)
    x = torch.rand(B, 3, S, S, generator=torch.Generator().manual_seed(77)).half().to(device)
    for graph in (False, True):
        best = eng.new_best().fill_(-1)
        pred = eng(x, out=torch.empty_like(eng.pred), best=best, graph=graph)
        torch.cuda.synchronize()
        sc, cl = pred[:, 4:].max(1)
        kb = best.cpu().numpy().view(np.uint64)
        assert np.array_equal((kb >> np.uint64(32)).astype(np.uint32), sc.cpu().numpy().view(np.uint32))
        assert np.array_equal((np.uint64(0xFFFFFFFF) - (kb & np.uint64(0xFFFFFFFF))).astype(np.int64), cl.cpu().numpy())
        n1, n2 = NMS(B, eng.anchors, eng.nc, device), NMS(B, eng.anchors, eng.nc, device)
        n1(pred)
        n2(pred, best)
        torch.cuda.synchronize()
        assert torch.equal(n1.buf, n2.buf)


@pytest.mark.parametrize("defer,lanes,graph", [(True, 1, False), (False, 1, False), (False, 2, False), (False, 3, True),
                                               (False, 4, True)])
def test_pipeline_overlap_matches_sequential(defer, lanes, graph, device):
    """engine.Pipeline (forward i+1 overlapping NMS i, double-buffered; deferred to the next forward's
    fork point or right after the forward; or 2-3 lanes = executors on their own streams with batches
    in flight) gives every batch exactly the sequential forward + NMS result; so does
    dist.ShardedPredictor on one rank.  (False, 3, True) is the bench's shipped mode: three lanes, each
    replaying its own captured hipGraph (bench.py)."""
    model = cases.seeded_model("yolo11n-fce.yaml", 0).to(device)
    B, S = 4, 320
    eng = Engine(model, B, S, device)
    xs = [torch.rand(B, 3, S, S, generator=torch.Generator().manual_seed(500 + i)).half().to(device) for i in range(7)]
    seq = []
    nms = NMS(B, eng.anchors, eng.nc, device)
    for x in xs:
        nms(eng(x))
        d, k = nms.results()
        seq.append(([t.clone() for t in d], [t.clone() for t in k]))

    def check(i, d, k):
        for b in range(B):
            assert torch.equal(d[b], seq[i][0][b]) and torch.equal(k[b], seq[i][1][b]), (i, b)

    pipe = Pipeline(eng, depth=2, defer=defer, lanes=lanes)
    for e in pipe.engs:
        e.graph = graph
    got = [pipe.submit(x) for x in xs]  # back to back; only the last `depth` batches remain in their slots
    for i in range(len(xs) - pipe.depth, len(xs)):
        check(i, *pipe.results(got[i]))
    # and every batch, by draining after each submit
    pipe2 = Pipeline(eng, depth=2, defer=defer, lanes=lanes)
    for e in pipe2.engs:
        e.graph = graph
    for i, x in enumerate(xs):
        check(i, *pipe2.results(pipe2.submit(x)))
    if lanes > 1:
        # fresh input tensors dropped right after submit (the caching allocator may hand their blocks to the
        # next batch's H2D copy while a lane still reads them unless the lane holds them: Pipeline records
        # them on the lane stream)
        pipe3 = Pipeline(eng, depth=lanes, lanes=lanes)
        for e in pipe3.engs:
            e.graph = graph
        slots = []
        for x in xs:
            slots.append(pipe3.submit(x.cpu().to(device)))  # the only reference is dropped here
        for i in range(len(xs) - pipe3.depth, len(xs)):
            check(i, *pipe3.results(slots[i]))
    if defer or lanes > 1:
        from fce_yolo_amd.dist import ShardedPredictor

        sp = ShardedPredictor(model, B, S, device, lanes=lanes)
        for e in sp.pipe.engs:
            e.graph = graph
        slots = [sp.submit(x) for x in xs]
        for i in range(len(xs) - sp.pipe.depth, len(xs)):
            check(i, *sp.results(slots[i]))
        sp.close()


@pytest.mark.parametrize("key", list(cases.E2E_NMS))
def test_end_to_end_nms_indices_bit_exact_vs_reference(key, e2e_nms_fx, device):
    """North star "bit-exact box indices after NMS": the HIP fp16 forward + device NMS, on a margin-designed
    case (make_golden_e2e_nms.py: score gaps, conf distance and IoU distance from 0.7 far above the fp16
    error), keeps exactly the anchors the reference's fp32 forward + non_max_suppression kept, in the same
    order; boxes within the end-to-end tolerance, scores within the fixture's designed margin (the designed
    head scales its logits by K / s_c, so an fp16 score error, measured up to 7.4e-3, is larger than the
    plain models' 1e-3; the margins, >= 1e-2 and checked on the reference's fp32 output, are what keep
    every decision fixed, and the kept indices are asserted exactly).  Graph replay and direct launches, NMS with and
    without the Detect epilogue's best-class keys."""
    fx = e2e_nms_fx.group(key)
    model, x = cases.designed_model(key, fx)
    _, B, S = cases.E2E_NMS[key]
    eng = Engine(model.to(device), B, S, device)
    xd = x.half().to(device)
    for graph in (True, False):
        best = eng.new_best()
        pred = eng(xd, out=torch.empty_like(eng.pred), best=best, graph=graph)
        torch.cuda.synchronize()
        ys = pred.cpu().numpy()[:, :, ::7]
        ref = fx["y_slice"]
        print(f"{key}: score err {np.abs(ys[:, 4:] - ref[:, 4:]).max():.2e}, box rel "
              f"{np.abs(ys[:, :4] - ref[:, :4]).max() / np.abs(ref[:, :4]).max():.2e}, kept "
              f"{[len(fx[f'keep{b}']) for b in range(B)]}")
        for use_best in (False, True):
            nms = NMS(B, eng.anchors, eng.nc, device)
            nms(pred, best if use_best else None)
            dets, keep = nms.results()
            for b in range(B):
                k, d, r = keep[b].cpu().numpy(), dets[b].cpu().numpy(), fx[f"det{b}"]
                assert np.array_equal(k, fx[f"keep{b}"]), (graph, use_best, b, k, fx[f"keep{b}"])
                assert np.array_equal(d[:, 5], r[:, 5])
                assert np.abs(d[:, :4] - r[:, :4]).max() <= BOX_TOL * np.abs(r[:, :4]).max()
                assert np.abs(d[:, 4] - r[:, 4]).max() <= float(fx["score_margin"])


@pytest.mark.parametrize("key", list(cases.E2E_NMS640))
def test_end_to_end_nms_indices_640_in_the_shipped_modes(key, e2e_nms640_fx, device):
    """Kept anchor indices bit-equal to the reference's at the HEADLINE size (make_golden_e2e_nms640.py: yolo11n-fce
    640 x 640 with the bench's batch of 32, yolo11s-bifpn 640 batch 4; the 20 x 20 level's 8 designed classes, per
    image margins), through every way the bench and the multi-GPU path run the forward: one executor (graph replay
    and direct launches, NMS with and without the epilogue's best-class keys), engine.Pipeline with four lanes each
    replaying its own captured hipGraph (bench.py's default on one GPU) with fresh inputs dropped after submit, and
    dist.ShardedPredictor on one rank (the bench's step object)."""
    from fce_yolo_amd.dist import ShardedPredictor

    fx = e2e_nms640_fx.group(key)
    model, x = cases.designed_model640(key, fx)
    _, B, S = cases.E2E_NMS640[key]
    a0, ref_y = int(fx["anchor0"]), fx["y_level"]
    model = model.to(device)
    xd = x.half().to(device)

    def check(tag, dets, keep):
        for b in range(B):
            k, d, r = keep[b].cpu().numpy(), dets[b].cpu().numpy(), fx[f"det{b}"]
            assert np.array_equal(k, fx[f"keep{b}"]), (tag, b, k, fx[f"keep{b}"])
            assert np.array_equal(d[:, 5], r[:, 5]), (tag, b)
            assert np.abs(d[:, :4] - r[:, :4]).max() <= BOX_TOL * np.abs(r[:, :4]).max(), (tag, b)
            assert np.abs(d[:, 4] - r[:, 4]).max() <= float(fx["score_margin"]), (tag, b)

    eng = Engine(model, B, S, device)
    for graph in (True, False):
        best = eng.new_best()
        pred = eng(xd, out=torch.empty_like(eng.pred), best=best, graph=graph)
        torch.cuda.synchronize()
        yl = pred[:, :ref_y.shape[1], a0:a0 + ref_y.shape[2]].cpu().numpy()
        print(f"{key} graph={graph}: score err {np.abs(yl[:, 4:] - ref_y[:, 4:]).max():.2e}, box rel "
              f"{np.abs(yl[:, :4] - ref_y[:, :4]).max() / np.abs(ref_y[:, :4]).max():.2e}, kept "
              f"{[len(fx[f'keep{b}']) for b in range(B)]}")
        for use_best in (False, True):
            nms = NMS(B, eng.anchors, eng.nc, device)
            nms(pred, best if use_best else None)
            check(f"engine graph={graph} best={use_best}", *nms.results())
    pipe = Pipeline(eng, depth=4, lanes=4)
    for e in pipe.engs:
        e.graph = True
    slots = [pipe.submit(x.half().to(device)) for _ in range(6)]  # fresh inputs, dropped right after submit
    for i in range(len(slots) - pipe.depth, len(slots)):
        check(f"pipeline slot {i}", *pipe.results(slots[i]))
    eng.close()
    sp = ShardedPredictor(model, B, S, device, lanes=4)
    for e in sp.pipe.engs:
        e.graph = True
    slots = [sp.submit(xd) for _ in range(5)]
    for i in range(len(slots) - sp.pipe.depth, len(slots)):
        check(f"sharded slot {i}", *sp.results(slots[i]))
    sp.close()


@pytest.mark.parametrize("key", list(cases.E2E_NMS_ML))
def test_end_to_end_nms_indices_all_levels_and_scales(key, e2e_nms_ml_fx, device):
    """Kept anchor indices bit-equal to the reference's with designed candidates on several Detect levels of every
    image: all three at n 640 (batch 8: P3 / P4 / P5 outputs of the HIP forward all reach the NMS), P3 and P4 at the
    l (640, batch 2: the scale of the 8-GPU l256 config's per-rank shard) and m-h8 (1280, batch 2: config 4) scales
    (make_golden_e2e_nms_ml.py).  Through one executor (graph replay and direct launches, NMS with and without the
    epilogue's best-class keys), engine.Pipeline with three lanes replaying captured hipGraphs, and
    dist.ShardedPredictor; scores within the fixture's margin and boxes within BOX_TOL at every candidate anchor."""
    from fce_yolo_amd.dist import ShardedPredictor

    fx = e2e_nms_ml_fx.group(key)
    model, x = cases.designed_model_ml(key, fx)
    _, _, B, S = cases.E2E_NMS_ML[key]
    model = model.to(device)
    xd = x.half().to(device)

    def check(tag, dets, keep):
        for b in range(B):
            k, d, r = keep[b].cpu().numpy(), dets[b].cpu().numpy(), fx[f"det{b}"]
            assert np.array_equal(k, fx[f"keep{b}"]), (tag, b, k, fx[f"keep{b}"])
            assert np.array_equal(d[:, 5], r[:, 5]), (tag, b)
            assert np.abs(d[:, :4] - r[:, :4]).max() <= BOX_TOL * np.abs(r[:, :4]).max(), (tag, b)
            assert np.abs(d[:, 4] - r[:, 4]).max() <= float(fx["score_margin"]), (tag, b)

    eng = Engine(model, B, S, device)
    for graph in (True, False):
        best = eng.new_best()
        pred = eng(xd, out=torch.empty_like(eng.pred), best=best, graph=graph)
        torch.cuda.synchronize()
        yc = [pred[b][:fx[f"y_cand{b}"].shape[1]][:, torch.from_numpy(fx[f"cand{b}"]).to(device)].cpu().numpy().T
              for b in range(B)]  # (candidates, 4 + designed classes), as stored
        es = max(np.abs(yc[b][:, 4:] - fx[f"y_cand{b}"][:, 4:]).max() for b in range(B))
        eb = max(np.abs(yc[b][:, :4] - fx[f"y_cand{b}"][:, :4]).max() / np.abs(fx[f"y_cand{b}"][:, :4]).max()
                 for b in range(B))
        print(f"{key} graph={graph}: candidate score err {es:.2e}, box rel {eb:.2e}, kept "
              f"{[len(fx[f'keep{b}']) for b in range(B)]}")
        # the designed cls convs scale a principal direction by K / its std (x10-x25): the fp16 forward's feature
        # rounding reaches the designed scores amplified by that much (2.6e-3 / 2.8e-3 / 9.3e-4 measured, n / l / m),
        # so scores are held to the fixture's margin, as in the other e2e cases; the forward's own 1e-3 bar is
        # test_full_size_parity / test_op_parity on the undesigned weights
        assert es <= float(fx["score_margin"]) and eb <= BOX_TOL, (es, eb)
        for use_best in (False, True):
            nms = NMS(B, eng.anchors, eng.nc, device)
            nms(pred, best if use_best else None)
            check(f"engine graph={graph} best={use_best}", *nms.results())
    pipe = Pipeline(eng, depth=3, lanes=3)
    for e in pipe.engs:
        e.graph = True
    slots = [pipe.submit(x.half().to(device)) for _ in range(4)]  # fresh inputs, dropped right after submit
    for i in range(len(slots) - pipe.depth, len(slots)):
        check(f"pipeline slot {i}", *pipe.results(slots[i]))
    eng.close()
    sp = ShardedPredictor(model, B, S, device, lanes=3)
    for e in sp.pipe.engs:
        e.graph = True
    slots = [sp.submit(xd) for _ in range(4)]
    for i in range(len(slots) - sp.pipe.depth, len(slots)):
        check(f"sharded slot {i}", *sp.results(slots[i]))
    sp.close()


CONV_VARIANT_CASES = [  # cin, cout, k, stride, H, W, residual
    (8, 8, 3, 1, 37, 45, True), (16, 32, 3, 2, 40, 50, False), (8, 16, 3, 1, 33, 20, False),
    (48, 64, 3, 1, 21, 35, False), (24, 40, 3, 2, 19, 31, False), (64, 64, 3, 1, 40, 40, True),
    (32, 16, 1, 1, 30, 30, False), (96, 80, 3, 2, 23, 29, False), (128, 64, 3, 1, 20, 20, False),
    (128, 64, 1, 1, 25, 27, True), (256, 40, 1, 1, 16, 24, False), (96, 48, 1, 1, 41, 17, False),
    (64, 128, 1, 1, 30, 40, False), (384, 64, 1, 1, 13, 17, True), (264, 48, 1, 1, 9, 11, False),
    (576, 256, 1, 1, 5, 7, False), (32, 32, 1, 1, 256, 256, False), (64, 48, 1, 1, 200, 200, True),
    (192, 128, 1, 1, 128, 160, False), (32, 64, 3, 2, 90, 100, False), (64, 48, 3, 1, 130, 70, True),
    (64, 80, 3, 2, 41, 37, False),
    # wide 1x1s of the m/l scales (big-tile K-pipelined kernel, 0x7xx; 256-wide tiles, 0xBxx): odd K-step counts,
    # partial cout tiles / groups, partial pixel tiles, cin % 32 != 0
    (512, 256, 1, 1, 40, 40, True), (96, 256, 1, 1, 33, 35, False), (136, 72, 1, 1, 19, 23, True),
    (200, 144, 1, 1, 17, 29, True), (1024, 512, 1, 1, 20, 20, False), (72, 384, 1, 1, 31, 9, False),
    # m/l 3x3s (A-in-LDS tile kernel, 0x81xx): partial cout groups, odd chunk counts, stride 2, residual
    (256, 256, 3, 1, 40, 40, True), (128, 80, 3, 2, 41, 37, False), (192, 128, 3, 1, 37, 29, True),
    (160, 48, 3, 1, 21, 19, False),
    # big-tile LDS-DMA 3x3 (0x8x0): stride 2 with partial cout groups / edge tiles, residual
    (128, 136, 3, 2, 41, 37, False), (96, 192, 3, 2, 33, 47, True), (64, 96, 3, 1, 19, 35, True),
    # 256-wide implicit-GEMM 3x3 (0xCx0): stride 2 over odd maps with partial pixel tiles, residual, 512 couts
    (512, 256, 3, 2, 21, 19, True), (64, 512, 3, 1, 13, 11, False),
    # persistent 32x32x16 ring 3x3 (0x9x0): cin 32 / 64, stride 1 / 2, partial row / column tiles, residual, 32 couts
    (32, 32, 3, 1, 9, 50, True), (64, 128, 3, 2, 19, 33, True), (64, 64, 3, 2, 21, 37, False),
    (32, 96, 3, 1, 23, 17, False),
]


@pytest.mark.parametrize("cin,cout,up,xpad,ypad,epi", [
    (64, 32, 1, 16, 8, N.EPI_STORE), (96, 128, 1, 0, 32, N.EPI_STORE), (48, 24, 0, 24, 16, N.EPI_STORE),
    (256, 64, 2, 8, 0, N.EPI_STORE), (256, 64, 1, 0, 64, N.EPI_WSTORE), (128, 64, 0, 0, 0, N.EPI_WSTORE),
    (256, 64, 1, 0, 64, N.EPI_ACCUM), (64, 128, 0, 32, 0, N.EPI_ACCUM)])
def test_conv1x1_variants_views_and_upsampling(cin, cout, up, xpad, ypad, epi, device):
    """1x1 variants on channel-slice views (input and output inside wider NHWC buffers), with fused
    nearest upsampling of the input and the BiFPN weighted-store / accumulate epilogues: bitwise equal
    across variants, fp64-reference parity, and the output buffer's other channels untouched."""
    H, W = 20, 20
    g = torch.Generator().manual_seed(cin + 7 * cout + up + 100 * epi)
    w = torch.randn(cout, cin, 1, 1, generator=g) * (1.0 / cin ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    x = torch.randn(2, cin, H, W, generator=g).half()
    fw = torch.tensor([0.7, -0.2, 1.3])
    fwd = fw.to(device)
    desc = N.ConvDesc(cin, cout, 1, 1, 1, N.ACT_SILU, up, epi, fwd.data_ptr() if epi else None, 3 if epi else 0,
                      2 if epi else 0)
    wp = M.pack_conv(desc, w, device)
    bd = b.float().to(device)
    xbuf = torch.randn(2, H, W, cin + xpad, generator=g).half().to(device)
    xbuf[..., xpad:] = x.to(device).permute(0, 2, 3, 1)
    Ho, Wo = H << up, W << up
    xu = x.double().repeat_interleave(1 << up, 2).repeat_interleave(1 << up, 3)
    ref = torch.nn.functional.silu(torch.nn.functional.conv2d(xu, w.double(), b.double()))
    y0 = torch.randn(2, Ho, Wo, cout, generator=g).half()
    if epi:
        r = fw.clamp_min(0).double()
        alpha = r[2] / (r.sum() + 1e-4)
        ref = alpha * ref + (y0.permute(0, 3, 1, 2).double() if epi == N.EPI_ACCUM else 0)
    xt = N.Tensor(xbuf.data_ptr(), N.F16, N.NHWC, 2, cin, H, W, cin + xpad, xpad)
    codes = (C.c_int * 128)()
    nv = N.lib().fce_conv_variants(C.byref(desc), W, codes, 128)
    assert any((codes[i] & 0xF00) == 0x400 for i in range(nv))
    assert any((codes[i] & 0xF00) == 0x700 for i in range(nv)) == (cin >= 64 and cout >= 64)
    assert any((codes[i] & 0xF00) == 0xB00 for i in range(nv)) == (cin >= 64 and cout >= 64)
    outs = {}
    for code in [-1] + list(codes[:nv]):
        y = torch.full((2, Ho, Wo, cout + ypad), float("nan"), dtype=torch.float16, device=device)
        y[..., ypad:] = y0.to(device)
        yt = N.Tensor(y.data_ptr(), N.F16, N.NHWC, 2, cout, Ho, Wo, cout + ypad, ypad)
        N.call("fce_conv2d_variant", C.byref(desc), C.byref(xt), wp.data_ptr(), bd.data_ptr(), None, C.byref(yt),
               code, None)
        yc = y.cpu()
        assert torch.isnan(yc[..., :ypad]).all(), hex(code)
        outs[code] = yc[..., ypad:].permute(0, 3, 1, 2)
    base = outs[-1]
    for code, y in outs.items():
        assert torch.equal(y, base), (hex(code), (y.float() - base.float()).abs().max().item())
    err = _rel(base, ref)
    print(f"OPERR variants {err:.3e}")
    assert err <= OP_TOL, err
    if epi != N.EPI_STORE:
        return
    # the duplicate store (C2f / C3k2 cv1, fce_net_add_conv_dup) through every variant's store path: the dense
    # copy equals the output's channels [lo, lo + dc) and the output itself is unchanged
    lo, dc = 8, min(16, cout - 8)
    for code in [-1] + list(codes[:nv]):
        y = torch.full((2, Ho, Wo, cout + ypad), float("nan"), dtype=torch.float16, device=device)
        dup = torch.full((2, Ho, Wo, dc), float("nan"), dtype=torch.float16, device=device)
        yt = N.Tensor(y.data_ptr(), N.F16, N.NHWC, 2, cout, Ho, Wo, cout + ypad, ypad)
        dt = N.Tensor(dup.data_ptr(), N.F16, N.NHWC, 2, dc, Ho, Wo, dc, 0)
        N.call("fce_conv2d_variant_dup", C.byref(desc), C.byref(xt), wp.data_ptr(), bd.data_ptr(), None, C.byref(yt),
               code, C.byref(dt), lo, None)
        yc = y.cpu()
        assert torch.equal(yc[..., ypad:].permute(0, 3, 1, 2), base), hex(code)
        assert torch.equal(dup.cpu(), yc[..., ypad + lo:ypad + lo + dc]), hex(code)


@pytest.mark.parametrize("case", CONV_VARIANT_CASES)
def test_conv_every_variant_bitwise_and_parity(case, device, monkeypatch):
    """Every kernel variant the executor may autotune to (register tiles, LDS-tile kernels, the opt-in
    A-in-LDS and wide-tile 3x3 kernels) gives the bit-identical result, and that result matches the fp64 reference
    within the per-op tolerance."""
    monkeypatch.setenv("FCE_TILE3AL", "1")
    monkeypatch.setenv("FCE_WIDE3", "1")  # + the opt-in wide-tile 3x3 (0xA00)
    monkeypatch.setenv("FCE_RING32", "1")  # + the opt-in 32x32x16 ring 3x3 (0x900)
    cin, cout, k, stride, H, W, with_res = case
    g = torch.Generator().manual_seed(cin * 1000 + cout)
    w = torch.randn(cout, cin, k, k, generator=g) * (1.0 / (cin * k * k) ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    x = torch.randn(2, cin, H, W, generator=g).half()
    desc = N.ConvDesc(cin, cout, k, stride, 1, N.ACT_SILU, 0, 0, None, 0, 0)
    wp = M.pack_conv(desc, w, device)
    bd = b.float().to(device)
    xd = x.to(device).permute(0, 2, 3, 1).contiguous()
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    ref = torch.nn.functional.conv2d(x.double(), w.double(), b.double(), stride, k // 2)
    res = None
    if with_res:
        r = torch.randn(2, cout, Ho, Wo, generator=g).half()
        res = r.to(device).permute(0, 2, 3, 1).contiguous()
    ref = torch.nn.functional.silu(ref) + (r.double() if with_res else 0)
    xt = N.Tensor(xd.data_ptr(), N.F16, N.NHWC, 2, cin, H, W, cin, 0)
    rt = N.Tensor(res.data_ptr(), N.F16, N.NHWC, 2, cout, Ho, Wo, cout, 0) if with_res else None
    codes = (C.c_int * 128)()
    nv = N.lib().fce_conv_variants(C.byref(desc), W, codes, 128)
    assert nv >= 2
    # the 32x32x16 ring is offered exactly where one of its tiles applies (its sums are the 16x16x32 kernels', bit for
    # bit): cin 32 / 64, cout % 32 == 0, a double-buffered tile within 64 KiB of static LDS, more couts than half a group
    def ring32_fits(wc, rpw):
        ne = (((2 * rpw * (4 // wc) - 1) * stride + 3) * (15 * stride + 3) * 4 * (cin // 32) + 255) // 256 * 256
        return 2 * ne * 16 <= 64 * 1024

    offered = k == 3 and cin in (32, 64) and cout % 32 == 0 and any(
        ring32_fits(wc, rpw) and 16 * wc < cout for wc in (1, 2, 4) for rpw in (1, 2))
    assert any((codes[i] & 0xF00) == 0x900 for i in range(nv)) == offered
    outs = {}
    for code in [-1] + list(codes[:nv]):
        y = torch.full((2, Ho, Wo, cout), float("nan"), dtype=torch.float16, device=device)
        yt = N.Tensor(y.data_ptr(), N.F16, N.NHWC, 2, cout, Ho, Wo, cout, 0)
        N.call("fce_conv2d_variant", C.byref(desc), C.byref(xt), wp.data_ptr(), bd.data_ptr(),
               C.byref(rt) if rt is not None else None, C.byref(yt), code, None)
        outs[code] = y.permute(0, 3, 1, 2).cpu()
    base = outs[-1]
    for code, y in outs.items():
        assert torch.equal(y, base), hex(code)
    err = _rel(base, ref)
    print(f"OPERR variants {err:.3e}")
    assert err <= OP_TOL, err


@pytest.mark.parametrize("cin,cout,stride,H,W,xpad,ypad,with_res", [
    (64, 64, 1, 37, 41, 16, 8, True), (32, 32, 1, 45, 33, 32, 4, False), (64, 64, 2, 41, 37, 8, 24, True),
    (32, 64, 2, 50, 30, 0, 2, True), (64, 96, 1, 19, 23, 64, 6, False), (128, 128, 2, 41, 37, 16, 8, True),
    (128, 64, 2, 21, 19, 0, 2, False)])
def test_conv3x3_rings_on_channel_slice_views(cin, cout, stride, H, W, xpad, ypad, with_res, device):
    """The persistent 3x3 rings (register ring 0x6xx, LDS-DMA ring 0xDxx) on the views the graph hands them: input,
    output and residual as channel slices of wider NHWC buffers (ypad % 4 != 0: the LDS-DMA ring's unaligned-output
    fallback to the register ring, or at cin 128 to the implicit-GEMM kernel).  Bitwise equal to the default variant, the output buffer's other channels
    untouched, fp64 parity."""
    g = torch.Generator().manual_seed(cin * 31 + cout + stride + ypad)
    w = torch.randn(cout, cin, 3, 3, generator=g) * (1.0 / (cin * 9) ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    x = torch.randn(2, cin, H, W, generator=g).half()
    desc = N.ConvDesc(cin, cout, 3, stride, 1, N.ACT_SILU, 0, 0, None, 0, 0)
    wp = M.pack_conv(desc, w, device)
    bd = b.float().to(device)
    xbuf = torch.randn(2, H, W, cin + xpad, generator=g).half().to(device)
    xbuf[..., xpad:] = x.to(device).permute(0, 2, 3, 1)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    ref = torch.nn.functional.silu(torch.nn.functional.conv2d(x.double(), w.double(), b.double(), stride, 1))
    rt = None
    if with_res:
        r = torch.randn(2, cout, Ho, Wo, generator=g).half()
        rbuf = torch.randn(2, Ho, Wo, cout + 8, generator=g).half().to(device)
        rbuf[..., 8:] = r.to(device).permute(0, 2, 3, 1)
        rt = N.Tensor(rbuf.data_ptr(), N.F16, N.NHWC, 2, cout, Ho, Wo, cout + 8, 8)
        ref = ref + r.double()
    xt = N.Tensor(xbuf.data_ptr(), N.F16, N.NHWC, 2, cin, H, W, cin + xpad, xpad)
    codes = (C.c_int * 128)()
    nv = N.lib().fce_conv_variants(C.byref(desc), W, codes, 128)
    rings = [c for c in codes[:nv] if (c & 0xF00) in (0x600, 0xD00)]
    # cin 128: only the LDS-DMA ring's stride-2 one-row tiles (the register ring is cin 32 / 64)
    assert any((c & 0xF00) == 0xD00 for c in rings) and any((c & 0xF00) == 0x600 for c in rings) == (cin < 128)
    outs = {}
    for code in [-1] + rings:
        y = torch.full((2, Ho, Wo, cout + ypad), float("nan"), dtype=torch.float16, device=device)
        yt = N.Tensor(y.data_ptr(), N.F16, N.NHWC, 2, cout, Ho, Wo, cout + ypad, ypad)
        N.call("fce_conv2d_variant", C.byref(desc), C.byref(xt), wp.data_ptr(), bd.data_ptr(),
               C.byref(rt) if rt is not None else None, C.byref(yt), code, None)
        yc = y.cpu()
        assert torch.isnan(yc[..., :ypad]).all(), hex(code)
        outs[code] = yc[..., ypad:].permute(0, 3, 1, 2)
    base = outs[-1]
    for code, y in outs.items():
        assert torch.equal(y, base), (hex(code), (y.float() - base.float()).abs().max().item())
    err = _rel(base, ref)
    assert err <= OP_TOL, err


@pytest.mark.parametrize("c,stride,H,W,cpad", [
    (64, 1, 80, 80, 0), (80, 1, 37, 45, 0), (80, 2, 41, 37, 0), (128, 1, 19, 23, 16), (256, 2, 20, 20, 0),
    (24, 1, 11, 9, 8), (64, 2, 7, 5, 0),
])
def test_dwconv_every_variant_bitwise_and_parity(c, stride, H, W, cpad, device):
    """Every depthwise 3x3 variant (pixel quads, row-staged LDS, lane-contiguous, column runs of 2 / 4) gives the
    bit-identical result on channel-slice views, and matches the fp64 reference (Detect cls branch DWConv,
    reference ultralytics/nn/modules/conv.py DWConv)."""
    g = torch.Generator().manual_seed(c * 100 + H)
    w = torch.randn(c, 1, 3, 3, generator=g) * (1.0 / 3)
    b = torch.randn(c, generator=g) * 0.1
    x = torch.randn(2, c, H, W, generator=g).half()
    desc = N.ConvDesc(c, c, 3, stride, c, N.ACT_SILU, 0, 0, None, 0, 0)
    wp = M.pack_conv(desc, w, device)
    bd = b.float().to(device)
    xbuf = torch.randn(2, H, W, c + cpad, generator=g).half().to(device)
    xbuf[..., cpad:] = x.to(device).permute(0, 2, 3, 1)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    ref = torch.nn.functional.silu(torch.nn.functional.conv2d(x.double(), w.double(), b.double(), stride, 1, groups=c))
    xt = N.Tensor(xbuf.data_ptr(), N.F16, N.NHWC, 2, c, H, W, c + cpad, cpad)
    codes = (C.c_int * 128)()
    nv = N.lib().fce_conv_variants(C.byref(desc), W, codes, 128)
    assert set(codes[:nv]) >= {100, 102, 103, 104}
    outs = {}
    for code in [-1] + list(codes[:nv]):
        y = torch.full((2, Ho, Wo, c + cpad), float("nan"), dtype=torch.float16, device=device)
        yt = N.Tensor(y.data_ptr(), N.F16, N.NHWC, 2, c, Ho, Wo, c + cpad, cpad)
        N.call("fce_conv2d_variant", C.byref(desc), C.byref(xt), wp.data_ptr(), bd.data_ptr(), None, C.byref(yt),
               code, None)
        yc = y.cpu()
        assert torch.isnan(yc[..., :cpad]).all(), code
        outs[code] = yc[..., cpad:].permute(0, 3, 1, 2)
    base = outs[-1]
    for code, y in outs.items():
        assert torch.equal(y, base), (code, (y.float() - base.float()).abs().max().item())
    err = _rel(base, ref)
    print(f"OPERR variants {err:.3e}")
    assert err <= OP_TOL, err


@pytest.mark.parametrize("cfg,batch,imgsz", [("yolo11n-fce.yaml", 2, 320), ("yolo11s-bifpn.yaml", 2, 256),
                                             ("yolo11n-fce.yaml", 1, 640), ("yolo11m-fce.yaml", 1, 320)])
def test_every_op_variant_bitwise_in_model(cfg, batch, imgsz, device, monkeypatch):
    """Each conv op of a planned model, pinned in turn to every candidate kernel variant, leaves the
    whole forward bitwise unchanged (the model's own views, upsampling, BiFPN / Detect epilogues and
    partial tiles; this is what keeps batch invariance under plan-time autotuning)."""
    monkeypatch.setenv("FCE_AUTOTUNE", "0")
    model = cases.seeded_model(cfg, 0).to(device)
    x = torch.rand(batch, 3, imgsz, imgsz, generator=torch.Generator().manual_seed(3)).half().to(device)
    eng = Engine(model, batch, imgsz, device)
    base = eng(x).clone()
    bad, tried = [], 0
    for i in range(eng.num_ops()):
        codes = eng.variants(i)
        for code in codes:
            eng.set_variant(i, code)
            tried += 1
            if not torch.equal(eng(x), base):
                bad.append((i, hex(code)))
        if codes:
            eng.set_variant(i, -1)
    assert tried > 100 and not bad, bad


@pytest.mark.parametrize("hw", [(20, 23), (9, 7), (16, 16), (33, 20)])
def test_c2psa_multi_chunk_vs_oracle(hw, device):
    """C2PSA attention over more keys than one 256-key LDS chunk (and ragged 64-key tiles) vs the fp64
    oracle restatement (block.py:1247-1304)."""
    H, W = hw
    fx = {"seed": np.array(62)}
    mod = cases.build_op("c2psa", fx)
    x = torch.randn(2, 256, H, W, generator=torch.Generator().manual_seed(H * 100 + W)).half()
    ref = cases.oracle_op("c2psa", mod, [x.float()])
    with torch.no_grad():
        y = mod.to(device)(x.to(device))
    assert torch.isfinite(y).all()
    assert _rel(y.float(), ref) <= OP_TOL
