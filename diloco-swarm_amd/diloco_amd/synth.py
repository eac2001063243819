"""Counter-based synthetic values, bit-identical on host (numpy) and device (dl_fill_synth).

    u(seed, stream, i) = ((splitmix64(seed*0xD1B54A32D192ED03 + (stream<<40) + i) >> 40) - 2^23) * 2^-23
    value              = base + u*scale  (+ add[i])       -- fp32, each op correctly rounded

Inputs of an outer step (values "stand in for H inner steps"):
    θ_0[t]          = base_t + u(42, t, ·)·scale_t          (reference-like init, trees.init_spec)
    inner[s, r][t]  = θ_{s-1}[t] + u(1000·s + r, t, ·)·1e-3   (step s >= 1, DP rank r)
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

MASK = (1 << 64) - 1
OUTER_SEED = 42
NOISE_SCALE = 1e-3
_BLOCK = 1 << 22


def noise_seed(step: int, rank: int) -> int:
    return 1000 * step + rank


def uniform(seed: int, stream: int, n: int, start: int = 0) -> np.ndarray:
    """u in [-1, 1) as float32, elements [start, start+n) of stream `stream`."""
    key0 = np.uint64((seed * 0xD1B54A32D192ED03 + (stream << 40) + start) & MASK)
    out = np.empty(n, dtype=np.float32)
    with np.errstate(over="ignore"):
        for b0 in range(0, n, _BLOCK):
            b1 = min(n, b0 + _BLOCK)
            z = np.arange(b0, b1, dtype=np.uint64) + key0
            z += np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            hi = (z >> np.uint64(40)).astype(np.int64) - 8388608
            out[b0:b1] = hi.astype(np.float32) * np.float32(2.0 ** -23)
    return out


def values(seed: int, stream: int, n: int, base: float, scale: float, add=None) -> np.ndarray:
    u = uniform(seed, stream, n)
    x = np.float32(base) + u * np.float32(scale)
    if add is not None:
        x = x + np.asarray(add, dtype=np.float32).reshape(-1)
    return x.astype(np.float32, copy=False)


def outer_tree(numels: Sequence[int], init_spec) -> List[np.ndarray]:
    return [values(OUTER_SEED, t, n, b, s) for t, (n, (b, s)) in enumerate(zip(numels, init_spec))]


def inner_tree(theta: Sequence[np.ndarray], step: int, rank: int) -> List[np.ndarray]:
    seed = noise_seed(step, rank)
    return [values(seed, t, x.size, 0.0, NOISE_SCALE, add=x) for t, x in enumerate(theta)]


# ---- device side ---------------------------------------------------------------------------
def fill_device(dst, seed: int, stream: int, base: float, scale: float, add=None) -> None:
    """dst (contiguous fp32 cuda tensor) <- values(...) via the HIP kernel dl_fill_synth."""
    import torch

    from . import _lib

    assert dst.is_cuda and dst.dtype == torch.float32 and dst.is_contiguous()
    if add is not None:
        assert add.is_cuda and add.dtype == torch.float32 and add.is_contiguous()
        assert add.numel() == dst.numel()
    s = torch.cuda.current_stream(dst.device).cuda_stream
    _lib.call(
        "dl_fill_synth", dst.data_ptr(), dst.numel(), seed, stream, base, scale,
        add.data_ptr() if add is not None else None, s,
    )


def outer_tree_device(spec, device):
    import torch

    out = []
    for t, (n, (b, s)) in enumerate(zip(spec.numels(), spec.init_spec())):
        x = torch.empty(n, dtype=torch.float32, device=device)
        fill_device(x, OUTER_SEED, t, b, s)
        out.append(x)
    return out


def inner_tree_device(theta, step: int, rank: int, out=None):
    """inner[t] = theta[t] + noise; writes into `out` tensors when given."""
    import torch

    seed = noise_seed(step, rank)
    res = []
    for t, x in enumerate(theta):
        y = out[t] if out is not None else torch.empty_like(x)
        fill_device(y.view(-1), seed, t, 0.0, NOISE_SCALE, add=x.reshape(-1))
        res.append(y)
    return res
