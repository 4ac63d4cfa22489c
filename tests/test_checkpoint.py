"""Checkpoint adapter: safetensors + weights_only state_dicts round-trip into the
reference-keyed DetectionModel; pickled whole-module checkpoints are refused (never unpickled)."""

import pytest
import torch

import cases
from fce_yolo_amd import weights as Wt
from fce_yolo_amd.parser import DetectionModel


def _same(a, b):
    sa, sb = a.state_dict(), b.state_dict()
    return sa.keys() == sb.keys() and all(torch.equal(sa[k], sb[k]) for k in sa)


def test_safetensors_round_trip_with_architecture(tmp_path):
    m = cases.seeded_model("yolo11n-fce.yaml", 3)
    m.names = {i: f"c{i}" for i in range(80)}
    Wt.save_checkpoint(m, tmp_path / "w.safetensors")
    m2 = Wt.load_model(tmp_path / "w.safetensors")
    assert _same(m, m2) and m2.names == m.names
    assert m2.yaml["backbone"] == m.yaml["backbone"] and m2.yaml["head"] == m.yaml["head"]


@pytest.mark.parametrize("wrap", [None, "model", "ema", "state_dict"])
def test_weights_only_state_dict_forms(tmp_path, wrap):
    m = cases.seeded_model("yolo11s-bifpn.yaml", 4)
    sd = {k: v.half() if v.is_floating_point() else v for k, v in m.state_dict().items()}  # fp16 EMA-style
    obj = sd if wrap is None else {wrap: sd, "epoch": 3, "train_args": {"imgsz": 640}}
    torch.save(obj, tmp_path / "w.pt")
    m2 = Wt.load_model(tmp_path / "w.pt", cfg="yolo11s-bifpn.yaml")
    ref = {k: v.half().float() if v.is_floating_point() else v for k, v in m.state_dict().items()}
    assert all(torch.equal(m2.state_dict()[k], ref[k]) for k in ref)


def test_pickled_module_checkpoint_is_refused(tmp_path):
    torch.save({"model": torch.nn.Conv2d(3, 4, 1)}, tmp_path / "mod.pt")  # whole module, like the reference
    with pytest.raises(RuntimeError, match="convert once"):
        Wt.load_model(tmp_path / "mod.pt", cfg="yolo11n-fce.yaml")


def test_mismatched_architecture_raises(tmp_path):
    m = cases.seeded_model("yolo11n-fce.yaml", 0)
    torch.save(m.state_dict(), tmp_path / "n.pt")
    with pytest.raises(RuntimeError, match="mismatch"):
        Wt.load_model(tmp_path / "n.pt", cfg="yolo11s-fce.yaml")
    assert isinstance(Wt.load_model(tmp_path / "n.pt", cfg="yolo11n-fce.yaml"), DetectionModel)


def test_patch_autobackend_refuses_cpu():
    from fce_yolo_amd import integrate

    class _Backend:  # the attributes AutoBackend exposes for a PyTorch model
        def __init__(self, model):
            self.model, self.device = model, torch.device("cpu")

    with pytest.raises(RuntimeError, match="no CPU fallback"):
        integrate.patch_autobackend(_Backend(cases.seeded_model("yolo11n-fce.yaml", 0)))


def test_from_reference_model_keeps_keys_and_weights():
    from fce_yolo_amd import integrate

    ref = cases.seeded_model("yolo11n-fce.yaml", 5)  # same YAML / key layout as the reference model
    ref.names = {i: f"n{i}" for i in range(80)}
    m = integrate.from_reference_model(ref)
    assert _same(ref, m) and m.names == ref.names


@pytest.mark.gpu
def test_patched_autobackend_forward_is_the_engine(device):
    from fce_yolo_amd import integrate
    from fce_yolo_amd.engine import Engine

    class _Backend:
        def __init__(self, model):
            self.model, self.device = model, device

    ref = cases.seeded_model("yolo11n-fce.yaml", 0)
    be = _Backend(ref)
    integrate.patch_autobackend(be)
    x = torch.rand(2, 3, 160, 160, generator=torch.Generator().manual_seed(9)).half().to(device)
    y = be.forward(x).clone()
    eng = Engine(ref.to(device), 2, 160, device)
    assert torch.equal(y, eng(x)) and tuple(y.shape) == (2, 84, 525)
