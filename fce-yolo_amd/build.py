"""Build libfceyolo.so (gfx950) in-tree with hipcc.

    python fce-yolo_amd/build.py [--force] [--jobs N]

Each csrc/*.hip is compiled to an object with ``hipcc --offload-arch=gfx950`` and linked
into ``fce-yolo_amd/lib/libfceyolo.so`` (git-ignored, shipped to the GPU box with the
snapshot).  Objects are rebuilt only when a source or header is newer.
"""

from __future__ import annotations

import argparse
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
OBJ = PKG / "build"
LIB = PKG / "lib" / "libfceyolo.so"
INCLUDE = PKG.parent / "include"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("FCE_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result", f"-I{INCLUDE}"]


def _newest_header() -> float:
    hs = list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _compile(src: Path, force: bool) -> Path:
    obj = OBJ / (src.stem + ".o")
    if not force and obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, _newest_header()):
        return obj
    cmd = [HIPCC, *FLAGS, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int | None = None) -> Path:
    OBJ.mkdir(exist_ok=True)
    LIB.parent.mkdir(exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    jobs = jobs or min(8, len(srcs))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or not LIB.exists() or LIB.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        tmp = LIB.with_suffix(".so.tmp")  # linked aside, then renamed: the library is never seen half-written
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    a = ap.parse_args()
    print(build(a.force, a.jobs))
    sys.exit(0)
