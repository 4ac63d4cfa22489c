"""CPU: pin the oracle restatement to the reference's golden vectors (tests/golden, made by
tests/golden/make_golden.py from the reference itself)."""

import hashlib
import json

import numpy as np
import pytest
import torch

import cases
from conftest import NMS_OPT_CASES, nms_opt_case
from oracle import nms_oracle
from oracle.parse import parse

torch.set_num_threads(8)


@pytest.mark.parametrize("name", list(cases.OPS))
def test_oracle_ops_match_reference(name, ops_fx):
    fx = ops_fx.group(name)
    mod = cases.build_op(name, fx)
    out = cases.oracle_op(name, mod, cases.op_inputs(fx), torch.float32)
    ref = torch.from_numpy(fx["out"])
    assert out.shape == ref.shape
    err = (out.float() - ref).abs().max().item()
    assert err <= 1e-4 * max(1.0, ref.abs().max().item()), err


def test_oracle_detect_matches_reference(ops_fx):
    from oracle import fce_oracle as O

    fx = ops_fx.group("detect")
    det = cases.build_detect(fx)
    sd = O.cast_sd(O.fuse_state_dict({"m." + k: v for k, v in det.state_dict().items()}), torch.float32)
    feats = [torch.from_numpy(fx[f"in{i}"]) for i in range(3)]
    maps = O.detect_head_maps(sd, "m", feats, 80)
    for i in range(3):
        assert torch.allclose(maps[i], torch.from_numpy(fx[f"map{i}"]), atol=1e-4, rtol=1e-4)
    y = O.detect_decode(maps, [8.0, 16.0, 32.0], 80)
    ref = torch.from_numpy(fx["out"])
    assert (y - ref).abs().max().item() <= 1e-3


@pytest.mark.parametrize("key", list(cases.E2E))
def test_oracle_end_to_end_matches_reference(key, e2e_fx):
    fx = e2e_fx.group(key)
    cfg, mut = cases.E2E[key]
    model = cases.seeded_model(cfg, 0, mut)
    x = cases.e2e_input(key, fx)
    assert hashlib.sha256(x.numpy().tobytes()).digest() == fx["x_sha256"].tobytes()
    y = cases.oracle_model(model, x, torch.float32)
    ref = torch.from_numpy(fx["y"])
    box_err = (y[:, :4] - ref[:, :4]).abs().max().item() / ref[:, :4].abs().max().item()
    cls_err = (y[:, 4:] - ref[:, 4:]).abs().max().item()
    assert box_err < 1e-5 and cls_err < 1e-5, (box_err, cls_err)


def test_oracle_640_digest(e2e_fx):
    fx = e2e_fx.group("yolo11n-fce_640_b1")
    model = cases.seeded_model("yolo11n-fce.yaml", 0)
    x = torch.rand(1, 3, 640, 640, generator=torch.Generator().manual_seed(640))
    y = cases.oracle_model(model, x, torch.float32).numpy()
    ref_slice = fx["y_slice"]
    assert np.abs(y[:, :, ::37] - ref_slice).max() <= 1e-3 * np.abs(ref_slice).max()
    assert np.allclose(y.astype(np.float64).sum(2), fx["y_sum"], rtol=1e-4)


@pytest.mark.parametrize("name", ["designed_small", "designed_many", "none", "saturated_maxdet"])
def test_oracle_nms_bit_exact(name, nms_fx):
    fx = nms_fx.group(name)
    dets, keeps = nms_oracle.non_max_suppression(fx["pred"])
    for b in range(fx["pred"].shape[0]):
        assert np.array_equal(keeps[b], fx[f"keep{b}"].reshape(-1).astype(np.int64)), b
        assert np.array_equal(dets[b], fx[f"det{b}"].reshape(-1, 6)), b


@pytest.mark.parametrize("name", NMS_OPT_CASES)
def test_oracle_nms_options_bit_exact(name, nms_opts_fx):
    """classes / agnostic / multi_label (nms.py:116-141) against the reference's outputs."""
    pred, opts, exp = nms_opt_case(nms_opts_fx, name)
    dets, keeps = nms_oracle.non_max_suppression(pred, **opts)
    for b, (d, k) in enumerate(exp):
        assert np.array_equal(keeps[b], k), b
        assert np.array_equal(dets[b], d), b


def test_oracle_nms_on_model_output(e2e_fx):
    fx = e2e_fx.group("yolo11n-fce_160_b2")
    dets, keeps = nms_oracle.non_max_suppression(fx["y"])
    for b in range(2):
        assert np.array_equal(keeps[b], fx[f"nms_keep{b}"].astype(np.int64))
        assert np.array_equal(dets[b], fx[f"nms_det{b}"])


@pytest.mark.parametrize("key", list(cases.E2E_NMS))
def test_oracle_designed_end_to_end_nms_matches_reference(key, e2e_nms_fx):
    """Margin-designed end-to-end case (make_golden_e2e_nms.py): the oracle's fp32 forward + oracle NMS keep
    exactly the anchors the reference's forward + non_max_suppression kept, with the same rows to 1e-4."""
    fx = e2e_nms_fx.group(key)
    model, x = cases.designed_model(key, fx)
    y = cases.oracle_model(model, x, torch.float32).numpy()
    assert np.abs(y[:, :, ::7] - fx["y_slice"]).max() <= 1e-4 * np.abs(fx["y_slice"]).max()
    dets, keeps = nms_oracle.non_max_suppression(y)
    for b in range(x.shape[0]):
        assert np.array_equal(keeps[b], fx[f"keep{b}"]), b
        assert np.abs(dets[b] - fx[f"det{b}"]).max() <= 1e-4 * max(1.0, np.abs(fx[f"det{b}"]).max()), b


@pytest.mark.parametrize("key", list(cases.E2E_NMS640))
def test_oracle_designed_end_to_end_nms_640_matches_reference(key, e2e_nms640_fx):
    """Headline-size margin-designed case (make_golden_e2e_nms640.py: n-fce 640 batch 32, s-bifpn 640 batch 4):
    the oracle's fp32 forward + oracle NMS keep exactly the reference's anchors, rows to 1e-4."""
    fx = e2e_nms640_fx.group(key)
    model, x = cases.designed_model640(key, fx)
    y = cases.oracle_model(model, x, torch.float32).numpy()
    a0, ref = int(fx["anchor0"]), fx["y_level"]
    yl = y[:, :ref.shape[1], a0:a0 + ref.shape[2]]
    assert np.abs(yl - ref).max() <= 1e-4 * np.abs(ref).max()
    dets, keeps = nms_oracle.non_max_suppression(y)
    for b in range(x.shape[0]):
        assert np.array_equal(keeps[b], fx[f"keep{b}"]), b
        assert np.abs(dets[b] - fx[f"det{b}"]).max() <= 1e-4 * max(1.0, np.abs(fx[f"det{b}"]).max()), b


@pytest.mark.parametrize("key", list(cases.E2E_NMS_ML))
def test_oracle_designed_end_to_end_nms_levels_and_scales_matches_reference(key, e2e_nms_ml_fx):
    """Several-level margin-designed cases (make_golden_e2e_nms_ml.py: n 640 on all three levels, l 640 and m-h8
    1280 on P3 / P4): the oracle's fp32 forward + oracle NMS keep exactly the reference's anchors, the candidates'
    rows and the kept rows to 1e-4."""
    fx = e2e_nms_ml_fx.group(key)
    model, x = cases.designed_model_ml(key, fx)
    y = cases.oracle_model(model, x, torch.float32).numpy()
    for b in range(x.shape[0]):
        ref = fx[f"y_cand{b}"]
        yc = y[b][:ref.shape[1]][:, fx[f"cand{b}"]].T
        assert np.abs(yc - ref).max() <= 1e-4 * np.abs(ref).max(), b
    dets, keeps = nms_oracle.non_max_suppression(y)
    for b in range(x.shape[0]):
        assert np.array_equal(keeps[b], fx[f"keep{b}"]), b
        assert np.abs(dets[b] - fx[f"det{b}"]).max() <= 1e-4 * max(1.0, np.abs(fx[f"det{b}"]).max()), b


def _cfg(name):
    """The built-in graph data of the product package (restated from the reference YAMLs)."""
    from fce_yolo_amd.parser import load_cfg

    if name.endswith("-h8"):
        d = load_cfg(name[:-3] + ".yaml")
        cases.heads8(d)
        return d
    return load_cfg(name + ".yaml")


@pytest.mark.parametrize("name", ["yolo11n-fce", "yolo11s-fce", "yolo11m-fce", "yolo11l-fce", "yolo11x-fce",
                                  "yolo11n-bifpn", "yolo11s-bifpn", "yolo11m-bifpn", "yolo11n", "yolo11m",
                                  "yolo11m-fce-h8"])
def test_oracle_parser_layer_table(name, tables):
    layers, save, legacy = parse(_cfg(name))
    t = tables[name]
    assert save == t["save"]
    assert legacy == t["legacy_detect"]
    for L, row in zip(layers, t["rows"]):
        assert L["i"] == row["i"] and L["f"] == row["f"]
        assert L["type"] == row["type"] or (L["type"] == "Upsample" and row["type"] == "Upsample")
        assert str(L["args"]).replace("'", "") == row["args"].replace("'", ""), (L, row)


@pytest.mark.parametrize("key", list(cases.FULL))
def test_oracle_full_size_matches_reference(key, full_fx):
    """The oracle at the BASELINE configs' real sizes (m-h8 @1280: C2PSA over 1600 keys, BiCoord at 160x160)
    against the reference's slices / row sums (golden/full.npz)."""
    fx = full_fx.group(key)
    cfg, mut, _, _ = cases.FULL[key]
    y = cases.oracle_model(cases.seeded_model(cfg, 0, mut), cases.full_input(key, fx), torch.float32)
    e_slice, e_sum = cases.compare_full(y, fx)
    assert e_slice < 2e-5 and e_sum < 1e-6, (e_slice, e_sum)


@pytest.mark.parametrize("key", list(cases.OPS_FULL))
def test_oracle_full_size_ops_match_reference(key, full_fx):
    fx = full_fx.group(key)
    mod, x = cases.full_op(key, fx)
    y = cases.full_op_oracle(key, mod, x)
    e_slice, e_sum = cases.compare_full(y, fx, anchors=False)
    assert e_slice < 2e-5 and e_sum < 1e-6, (e_slice, e_sum)
