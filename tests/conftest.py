"""Shared test setup: package paths, the `gpu` marker, golden-fixture loaders."""
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "diloco-swarm_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        # the eight-process tests first, while this process holds no GPU queues yet: their
        # eight ranks (GPU_MAX_HW_QUEUES = 1, 3 compute queues each) then fill the firmware
        # scheduler's 24 queue slots exactly, so it never time-slices or remaps them -- the
        # condition under which a rank's kernel lost an XCD's share of its work
        items.sort(key=lambda it: 0 if ("_eight_peers_" in it.name
                                        and it.get_closest_marker("gpu")) else 1)
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def load_npz(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def split(flat, numels):
    out, o = [], 0
    for n in numels:
        out.append(flat[o:o + n])
        o += n
    return out


def normwise_ok(got, ref, tol=1e-6):
    """|got - ref| <= tol * max|ref| per tensor (per-element relative error is
    ill-posed under cancellation once the all-reduce order differs)."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    scale = max(np.abs(ref).max(initial=0.0), np.finfo(np.float32).tiny)
    return float(np.abs(got - ref).max(initial=0.0)) <= tol * scale


def inner_tree_device_verified(theta, step, rank, out):
    """synth.inner_tree_device into `out`, then every tensor generated once more into a
    scratch buffer and compared on the device. The parity checks must judge the outer step on
    the inputs they were meant to get, so a mismatch fails the test at once -- an
    AssertionError naming the tensor, the number of wrong elements and the phases (index mod
    8, i.e. the XCD of the fill's workgroup) of the wrong 256-element blocks. Nothing is
    regenerated or retried."""
    import torch

    from diloco_amd import synth

    synth.inner_tree_device(theta, step, rank, out=out)
    seed = synth.noise_seed(step, rank)
    for t, (x, y) in enumerate(zip(theta, out)):
        ref = torch.empty_like(y)
        synth.fill_device(ref.view(-1), seed, t, 0.0, synth.NOISE_SCALE, add=x.reshape(-1))
        bad = ref.view(-1) != y.view(-1)
        if bool(bad.any()):
            nb = bad.numel() // 256
            blocks = torch.nonzero(bad[:nb * 256].view(nb, 256).any(1)).flatten()
            phases = torch.bincount(blocks % 8, minlength=8).tolist()
            raise AssertionError(f"input tensor {t} (step {step}, rank {rank}): "
                                 f"{int(bad.sum())} elements differ between two generations; "
                                 f"wrong 256-element blocks by phase {phases}")
        del ref, bad


def spin(ms, device=None):
    """A slow producer: the library's dl_spin occupies the current stream for `ms` ms."""
    import torch

    from diloco_amd import _lib

    _lib.call("dl_spin", int(ms * 1e6), torch.cuda.current_stream(device).cuda_stream)
