"""Register the ``fce-yolo_amd/`` package directory under the importable name ``fce_yolo_amd``.

    import fce_pkg; fce = fce_pkg.load()
"""

from __future__ import annotations

import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG_DIR = ROOT / "fce-yolo_amd"


def load():
    if "fce_yolo_amd" in sys.modules:
        return sys.modules["fce_yolo_amd"]
    spec = importlib.util.spec_from_file_location(
        "fce_yolo_amd", PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)]
    )
    mod = importlib.util.module_from_spec(spec)
    sys.modules["fce_yolo_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
