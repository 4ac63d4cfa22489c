import json
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))

import fce_pkg  # noqa: E402

fce_pkg.load()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libfceyolo.so")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def tables():
    return json.loads((GOLDEN / "parser_tables.json").read_text())


class _Npz:
    def __init__(self, path):
        self.z = np.load(path, allow_pickle=False)

    def group(self, name):
        pre = name + "/"
        return {k[len(pre):]: self.z[k] for k in self.z.files if k.startswith(pre)}

    def names(self):
        return sorted({k.split("/")[0] for k in self.z.files})


@pytest.fixture(scope="session")
def ops_fx():
    return _Npz(GOLDEN / "ops.npz")


@pytest.fixture(scope="session")
def e2e_fx():
    return _Npz(GOLDEN / "e2e.npz")


@pytest.fixture(scope="session")
def full_fx():
    return _Npz(GOLDEN / "full.npz")


@pytest.fixture(scope="session")
def e2e_nms_fx():
    return _Npz(GOLDEN / "e2e_nms.npz")


@pytest.fixture(scope="session")
def e2e_nms640_fx():
    return _Npz(GOLDEN / "e2e_nms640.npz")


@pytest.fixture(scope="session")
def e2e_nms_ml_fx():
    return _Npz(GOLDEN / "e2e_nms_ml.npz")


@pytest.fixture(scope="session")
def nms_fx():
    return _Npz(GOLDEN / "nms.npz")


@pytest.fixture(scope="session")
def nms_opts_fx():
    return _Npz(GOLDEN / "nms_opts.npz")


NMS_OPT_CASES = ["agnostic", "classes", "classes_absent", "multi", "multi_classes", "multi_agnostic", "multi_small",
                 "multi_big"]


def nms_opt_case(fx_all, name):
    """(pred, options dict, [(det, keep) per image]) of one nms_opts.npz case (make_golden_nms_opts.py)."""
    fx = fx_all.group(name)
    opts = json.loads(bytes(fx["opts"]).decode())
    pred = fx_all.group("pred")[opts.pop("pred")]
    exp = [(fx[f"det{b}"].reshape(-1, 6), fx[f"keep{b}"].reshape(-1).astype(np.int64)) for b in range(pred.shape[0])]
    return pred, opts, exp


@pytest.fixture(scope="session")
def device():
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible ROCm device")
    return torch.device("cuda:0")
