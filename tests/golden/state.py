"""Deterministic, non-trivial U-Net parameter/buffer values for the golden fixtures.

Shared by ``make_golden.py`` (which feeds them to the real reference) and the tests
(which feed them to the oracle and the HIP path), so 31 MB of weights never need to
be committed: only the seed.  numpy PCG64, independent of torch's RNG.
"""
from __future__ import annotations

import math
import os
import sys
from collections import OrderedDict

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from oracle.unet_ref import param_specs  # noqa: E402

GOLDEN_DIR = os.path.dirname(os.path.abspath(__file__))
SEED = 20250227


def fixture_state_np(seed: int = SEED):
    """name -> float32 ndarray (int64 for num_batches_tracked), reference key order."""
    rng = np.random.default_rng(seed)
    st = OrderedDict()
    for name, shape, kind in param_specs():
        if kind == "conv_w":
            fan_out = shape[0] * shape[2] * shape[3]
            v = rng.standard_normal(shape) * math.sqrt(2.0 / fan_out)
        elif kind == "conv_b":
            v = rng.uniform(-0.05, 0.05, shape)
        elif kind == "bn_w":
            v = rng.uniform(0.8, 1.2, shape)
        elif kind == "bn_b":
            v = rng.uniform(-0.1, 0.1, shape)
        elif kind == "bn_rm":
            v = rng.uniform(-0.1, 0.1, shape)
        elif kind == "bn_rv":
            v = rng.uniform(0.5, 1.5, shape)
        else:
            st[name] = np.zeros((), dtype=np.int64)
            continue
        st[name] = v.astype(np.float32)
    return st


def fixture_state_torch(dtype=None, device="cpu", seed: int = SEED):
    import torch
    out = OrderedDict()
    for k, v in fixture_state_np(seed).items():
        t = torch.from_numpy(np.array(v))
        if dtype is not None and t.is_floating_point():
            t = t.to(dtype)
        out[k] = t.to(device)
    return out


def fixture_inputs(batch: int = 4, seed: int = 7, hw: int = 40):
    """Model inputs as in SURVEY 8(d): ch0 ~ N(0,1), ch1 = 1 (constant theta), ch2 ~ N(0,1)."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((batch, 3, hw, hw)).astype(np.float32)
    x[:, 1] = 1.0
    t = rng.standard_normal((batch, 1, hw, hw)).astype(np.float32)
    return x, t


def sample_indices(numel: int, seed: int, k: int = 96):
    rng = np.random.default_rng(seed)
    head = np.arange(min(numel, 32))
    rand = rng.integers(0, numel, size=min(k, numel))
    return np.concatenate([head, rand]).astype(np.int64)
