"""The drop-in boundary driven by the REFERENCE itself.

The reference's ``ultralytics.nn.tasks`` is imported from /root/reference (build container only; these
tests skip where it is absent, e.g. on the GPU box), the 14 class names of INTEGRATION.md §1 are rebound
to this package's modules, and the reference's own ``DetectionModel`` builds the BASELINE configs:
``parse_model`` (tasks.py:1489-1743), the CPU stride probe in train mode (tasks.py:396-411, served by
the shape-only path), ``bias_init`` (head.py:169-180), ``initialize_weights``, ``fuse`` (tasks.py:223-252)
and ``.half()`` (BaseModel._apply, tasks.py:276-293).  The resulting module tree is checked against this
package's parser (which the GPU tests run), so the GPU parity of the drop-in forward
(``test_gpu.py::test_dropin_predict_once_parity``) covers the reference-built tree.
"""

from __future__ import annotations

import sys
from pathlib import Path

import pytest
import torch

import cases
from fce_yolo_amd import integrate
from fce_yolo_amd import modules as fce
from fce_yolo_amd.parser import DetectionModel, load_cfg

REF = Path("/root/reference")
pytestmark = pytest.mark.skipif(not (REF / "ultralytics").is_dir(), reason="reference not present (GPU box)")

# the names tasks.py resolves (C3k, PSABlock and Attention are built inside C3k2 / C2PSA, not looked up)
NAMES = ("Conv", "DWConv", "Concat", "Bottleneck", "C2f", "C3", "C3k2", "SPPF", "C2PSA", "BiFPN_Concat", "CoordAtt",
         "CoordCrossAtt", "BiCoordCrossAtt", "Detect")
CFGS = {  # parser_tables key: (reference yaml, mutate)
    "yolo11n-fce": ("yolo11n-fce.yaml", None),
    "yolo11s-bifpn": ("yolo11s-bifpn.yaml", None),
    "yolo11m-fce-h8": ("yolo11m-fce.yaml", cases.heads8),
    "yolo11l-fce": ("yolo11l-fce.yaml", None),
}


@pytest.fixture(scope="module")
def T():
    """ultralytics.nn.tasks with the drop-ins bound; the names are restored after."""
    sys.path.insert(0, str(Path(__file__).parent / "golden"))
    import make_golden

    tasks = make_golden.import_reference()
    saved = {n: getattr(tasks, n) for n in NAMES}
    for n in NAMES:
        setattr(tasks, n, getattr(fce, n))
    yield tasks
    for n, v in saved.items():
        setattr(tasks, n, v)


def _build(T, key):
    name, mut = CFGS[key]
    d = T.yaml_model_load(str(REF / "ultralytics/cfg/models/11" / name))
    if mut:
        mut(d)
    return T.DetectionModel(d, verbose=False)


def _tree(seq):
    return [(type(m).__name__, m.i, m.f) for m in seq]


@pytest.mark.parametrize("key", list(CFGS))
def test_reference_builds_with_dropins(T, key, tables):
    model = _build(T, key)
    assert model.stride.tolist() == [8.0, 16.0, 32.0]
    det = model.model[-1]
    assert type(det) is fce.Detect and det.training  # the reference leaves the model in train mode
    got = [[f"{k}", list(v.shape)] for k, v in model.state_dict().items()]
    assert got == tables[key]["state_dict"]
    # every layer the drop-ins cover is one of ours (nn.Upsample stays torch's, as in the YAML)
    for m in model.model:
        assert type(m).__module__ in ("fce_yolo_amd.modules", "torch.nn.modules.upsampling"), type(m)
    # same tree and save list as this package's parser (the model the GPU tests run)
    name, mut = CFGS[key]
    d = load_cfg(name)
    if mut:
        mut(d)
    ours = DetectionModel(d)
    assert _tree(model.model) == _tree(ours.model)
    assert model.save == ours.save
    # bias_init (head.py:169-180) ran with the probed strides
    for a, b, s in zip(det.cv2, det.cv3, det.stride):
        assert torch.all(a[-1].bias == 1.0)
        assert torch.allclose(b[-1].bias, torch.full_like(b[-1].bias, torch.log(5 / det.nc / (640 / s) ** 2)))


def test_fuse_half_and_eval_forward_shapes(T):
    model = _build(T, "yolo11n-fce")
    n_bn = sum(isinstance(m, torch.nn.BatchNorm2d) for m in model.modules())
    model.fuse(verbose=False)
    assert n_bn > 0 and not any(isinstance(m, torch.nn.BatchNorm2d) for m in model.modules())
    model = model.half().eval()
    assert model.model[-1].stride.dtype == torch.float16  # BaseModel._apply moved stride/anchors/strides
    with torch.inference_mode():
        y, maps = model(torch.zeros(2, 3, 320, 256))
    # shape-only on CPU: meta tensors of the reference's shapes, no values to read
    assert y.device.type == "meta" and tuple(y.shape) == (2, 84, 40 * 32 + 20 * 16 + 10 * 8)
    assert [tuple(m.shape) for m in maps] == [(2, 144, 40, 32), (2, 144, 20, 16), (2, 144, 10, 8)]
    with pytest.raises((RuntimeError, NotImplementedError)):
        y.sum().item()


def test_from_reference_model_fused_source(T):
    """AutoBackend fuses (autobackend.py:203-207): a fused reference model converts, and its BN-folded
    weights equal the ones this package folds from the unfused state_dict."""
    ref = _build(T, "yolo11n-fce")
    ref.load_state_dict(cases.seeded_model("yolo11n-fce.yaml", 3).state_dict())
    unfused = integrate.from_reference_model(ref)
    ref.eval().fuse(verbose=False)
    fused = integrate.from_reference_model(ref)
    assert fused.is_fused() and not unfused.is_fused()
    a = {n: m for n, m in unfused.named_modules() if isinstance(m, fce.Conv)}
    b = {n: m for n, m in fused.named_modules() if isinstance(m, fce.Conv)}
    assert a.keys() == b.keys()
    for n in a:
        wa, ba = fce.fold_bn(a[n].conv, a[n].bn)
        wb, bb = fce.fold_bn(b[n].conv, None)
        assert torch.allclose(wa, wb, rtol=1e-6, atol=1e-7) and torch.allclose(ba, bb, rtol=1e-5, atol=1e-6), n


def test_device_postprocess_fallback_uses_reference_signature(T):
    """Argument combinations off the device path reach the reference NMS by keyword (utils/nms.py:13-29)."""
    import ultralytics.utils.nms as nms_mod

    orig = nms_mod.non_max_suppression

    class _P:
        pass

    try:
        integrate.device_postprocess(_P())
        p = torch.zeros(1, 84, 50)
        p[0, :4, :] = torch.tensor([100.0, 100.0, 20.0, 20.0])[:, None]
        p[0, 4 + 3, 7] = 0.9
        kw = dict(classes=[3], agnostic=True, max_det=10, return_idxs=True)
        out = nms_mod.non_max_suppression(p.clone(), 0.25, 0.7, **kw)  # the reference converts boxes in place
        ref = orig(p.clone(), 0.25, 0.7, **kw)
        assert torch.equal(out[0][0], ref[0][0]) and torch.equal(out[1][0], ref[1][0])
        assert out[1][0].tolist() == [7]
    finally:
        nms_mod.non_max_suppression = orig
