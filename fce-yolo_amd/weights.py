"""Portable seeded weights for reference-architecture state_dicts.

There are no pretrained checkpoints offline, so benchmarks and parity fixtures use
random-init weights of the reference architecture.  The generator is a pure
function of the ordered (key, shape) list and a seed (numpy PCG64), so the
fixtures in ``tests/golden`` never need to store full model weights: the test
regenerates them.  Ranges keep activations O(1) through the folded-BN stack and
randomise the BN statistics so BN folding (eps = 1e-3) is exercised.
"""

from __future__ import annotations

import math

import numpy as np
import torch


def _is(key: str, suffix: str) -> bool:
    return key == suffix or key.endswith("." + suffix)


def _u(rng, shape, lo, hi):
    return (rng.random(shape, dtype=np.float64) * (hi - lo) + lo).astype(np.float32)


def seeded_state_dict(keys_shapes, seed: int = 0, cls_bias=(-2.6, -1.4), gain: float = 1.0):
    """Return {key: tensor} for an ordered iterable of (key, shape).

    * 4-D weights: N(0, 1) * gain * sqrt(1 / fan_in) (depthwise: fan_in = 9).  gain 1 (the default, every
      committed fixture and the bench) lets the signal decay with depth; gain ~1.6 keeps the outputs
      input-dependent (the margin-designed end-to-end NMS fixture, make_golden_e2e_nms.py).
    * BN: weight U(0.6,1.4), bias U(-0.3,0.3), running_mean U(-0.3,0.3), running_var U(0.5,1.5).
    * conv biases U(-0.2, 0.2); the final Detect cls conv bias U(cls_bias) so that only a
      fraction of anchors passes conf=0.25; BiFPN ``w`` U(0.3, 1.5).
    * ``dfl.conv.weight`` is the fixed arange(16) projection (block.py:58-80).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for key, shape in keys_shapes:
        shape = tuple(int(s) for s in shape)
        if _is(key, "num_batches_tracked"):
            out[key] = torch.tensor(0, dtype=torch.int64)
            continue
        if _is(key, "dfl.conv.weight"):
            out[key] = torch.arange(shape[1], dtype=torch.float32).view(shape)
            continue
        if _is(key, "bn.weight"):
            a = _u(rng, shape, 0.6, 1.4)
        elif _is(key, "bn.bias") or _is(key, "bn.running_mean"):
            a = _u(rng, shape, -0.3, 0.3)
        elif _is(key, "bn.running_var"):
            a = _u(rng, shape, 0.5, 1.5)
        elif len(shape) == 4:
            fan_in = shape[1] * shape[2] * shape[3]
            a = (rng.standard_normal(shape) * (gain * math.sqrt(1.0 / fan_in))).astype(np.float32)
        elif _is(key, "w") and len(shape) == 1:
            a = _u(rng, shape, 0.3, 1.5)
        elif _is(key, "bias"):
            parts = key.split(".")
            is_cls = len(parts) >= 4 and parts[-4] == "cv3" and parts[-2] == "2"
            a = _u(rng, shape, *cls_bias) if is_cls else _u(rng, shape, -0.2, 0.2)
        else:
            a = _u(rng, shape, -0.5, 0.5)
        out[key] = torch.from_numpy(a)
    return out


# ------------------------------------------------------------------------------------------------
# Checkpoint adapter.  Reference checkpoints (engine/trainer.py:588-611 save_model) are
# pickles of whole nn.Modules ({'ema': DetectionModel.half(), 'model': ..., 'train_args': ...}); the
# reference loads them with torch.load(weights_only=False) and its own classes (nn/tasks.py:1371-1486
# attempt_load_one_weight: ckpt.get('ema') or ckpt['model'], .float()).  This package never unpickles:
# it reads flat tensors only —
#   * a safetensors file written by scripts/convert_checkpoint.py (run once where the reference package
#     is importable), whose metadata carries the model's YAML dict and class names, or
#   * any torch.save'd state_dict / {'model' | 'ema' | 'state_dict': state_dict} loadable with
#     torch.load(weights_only=True).
# Keys and shapes are the reference's own (model.N.<...>), so they load unchanged.

META_YAML, META_NAMES = "fce_yolo.yaml", "fce_yolo.names"


def read_checkpoint(path):
    """(state_dict fp32, yaml dict | None, names dict | None) from a safetensors / weights_only file."""
    import json
    from pathlib import Path

    p = Path(path)
    if p.suffix == ".safetensors":
        from safetensors import safe_open
        from safetensors.torch import load_file

        with safe_open(str(p), framework="pt") as f:
            meta = f.metadata() or {}
        sd = load_file(str(p))
        yaml_d = json.loads(meta[META_YAML]) if META_YAML in meta else None
        names = {int(k): v for k, v in json.loads(meta[META_NAMES]).items()} if META_NAMES in meta else None
    else:
        try:
            obj = torch.load(str(p), map_location="cpu", weights_only=True)
        except Exception as e:  # a pickled reference checkpoint (whole modules)
            raise RuntimeError(
                f"{p}: not a tensors-only checkpoint ({type(e).__name__}). Reference .pt files pickle whole "
                "modules; convert once where the reference package is importable: "
                "python scripts/convert_checkpoint.py in.pt out.safetensors") from None
        yaml_d, names = None, None
        if isinstance(obj, dict):
            for k in ("ema", "model", "state_dict"):
                if isinstance(obj.get(k), dict):
                    obj = obj[k]
                    break
        if not isinstance(obj, dict) or not all(isinstance(v, torch.Tensor) for v in obj.values()):
            raise RuntimeError(f"{p}: expected a state_dict of tensors")
        sd = obj
    sd = {k: (v.float() if v.is_floating_point() else v) for k, v in sd.items()}
    return sd, yaml_d, names


def load_model(path, cfg=None, device=None):
    """DetectionModel built from the checkpoint's YAML (or `cfg`) with its weights loaded, eval mode."""
    from .parser import DetectionModel

    sd, yaml_d, names = read_checkpoint(path)
    arch = cfg if cfg is not None else yaml_d
    if arch is None:
        raise ValueError(f"{path}: no architecture in the checkpoint; pass cfg='yolo11n-fce.yaml' (or a YAML dict)")
    model = DetectionModel(arch)
    missing, unexpected = model.load_state_dict(sd, strict=False)
    if missing or unexpected:
        raise RuntimeError(f"{path}: state_dict mismatch: missing {missing[:5]}, unexpected {unexpected[:5]}")
    if names:
        model.names = names
    model.eval()
    return model.to(device) if device is not None else model


def save_checkpoint(model, path):
    """Write a model as this adapter's safetensors format (weights fp32 + YAML + names metadata)."""
    import json

    from safetensors.torch import save_file

    sd = {k: v.detach().float().contiguous().cpu() if v.is_floating_point() else v.detach().contiguous().cpu()
          for k, v in model.state_dict().items()}
    yaml_d = {k: v for k, v in model.yaml.items() if k not in ("yaml_file",)}
    meta = {META_YAML: json.dumps(yaml_d), META_NAMES: json.dumps({str(k): v for k, v in model.names.items()})}
    save_file(sd, str(path), metadata=meta)
