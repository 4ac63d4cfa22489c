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


def seeded_state_dict(keys_shapes, seed: int = 0, cls_bias=(-2.6, -1.4)):
    """Return {key: tensor} for an ordered iterable of (key, shape).

    * 4-D weights: N(0, 1) * sqrt(1 / fan_in) (depthwise: fan_in = 9).
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
            a = (rng.standard_normal(shape) * math.sqrt(1.0 / fan_in)).astype(np.float32)
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
