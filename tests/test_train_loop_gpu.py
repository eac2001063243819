"""End-to-end DiLoCo training loop on the GPU, in the style of the reference's integration test
(tests/test_memorize.py:10-84: run the training loop under several topologies, require a clean
exit and that the model memorised its data).

Each DP rank trains a small MLP to memorise a fixed random mapping with AdamW inner steps on
the GPU and runs the outer step every H inner steps exactly as src/train.py:244-269 does:

    compute_pseudo_gradient(inner, outer)   src/train.py:263
    comm.sync_gradients(outer)              src/train.py:265
    outer_optimizer.step()                  src/train.py:267
    sync_inner_model(outer, inner)          src/train.py:269

twice from the same initial state: once with the reference's per-tensor CPU outer step
(oracle/torch_restatement.py: host outer model, per-tensor gloo all_reduce, torch SGD-Nesterov)
and once with diloco_amd's drop-in functions (HIP kernels). The inner steps are identical GPU
work, so the two runs must end bit-identical at one and two peers, and the loss
must fall. Two peers run as two processes on the one GPU with a gloo DP group
(DILOCO_DP_BACKEND=gloo; RCCL refuses two ranks on one device).
"""
import os
import socket
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu

H, OUTER_STEPS = 4, 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Cfg:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def _model(dev):
    torch.manual_seed(42)  # every rank starts from the same weights (src/config.py:48)
    return torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.GELU(),
                               torch.nn.Linear(64, 64), torch.nn.GELU(),
                               torch.nn.Linear(64, 8)).to(dev)


def _data(rank, dev):
    g = torch.Generator().manual_seed(7)  # one mapping to memorise, rank-specific batches
    x = torch.randn(64, 32, generator=g)
    y = torch.randn(64, 8, generator=g)
    idx = torch.arange(64).view(4, 16)[rank % 4]
    return x[idx].to(dev), y[idx].to(dev)


def _train(rank, world, impl):
    """One training run; returns (final inner params flat, first loss, last loss)."""
    from diloco_amd.comm import TrainingComm
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)
    from diloco_amd.world import World
    from oracle.torch_restatement import TorchOuterStep

    dev = torch.device("cuda", 0)
    inner = _model(dev)
    xb, yb = _data(rank, dev)
    opt = torch.optim.AdamW(inner.parameters(), lr=1e-2, weight_decay=0.0, foreach=False)
    if impl == "reference":
        cpu_group = dist.new_group(list(range(world))) if world > 1 else None
        ref = TorchOuterStep([p.data.cpu() for p in inner.parameters()], group=cpu_group)
    else:
        outer = get_outer_model(inner)  # src/train.py:382
        outer_opt = get_optimizer(outer, _Cfg(type="SGD", lr=0.7, momentum=0.9, nesterov=True))
        comm = TrainingComm(World.from_default_group(1), (1, 1, 8), None)
    with torch.no_grad():
        first = float(torch.nn.functional.mse_loss(inner(xb), yb))
    for step in range(1, H * OUTER_STEPS + 1):
        opt.zero_grad()
        torch.nn.functional.mse_loss(inner(xb), yb).backward()
        opt.step()
        if step % H == 0:  # src/train.py:248 do_sync
            torch.cuda.synchronize()
            if impl == "reference":
                # the reference keeps the outer model on the CPU: inner params cross to the
                # host, the per-tensor CPU step runs, the result crosses back
                host_inner = [p.data.cpu() for p in inner.parameters()]
                ref.inner = host_inner
                ref.step()
                with torch.no_grad():
                    for p, h in zip(inner.parameters(), host_inner):
                        p.copy_(h.to(dev))
            else:
                compute_pseudo_gradient(inner, outer)
                comm.sync_gradients(outer)
                outer_opt.step()
                sync_inner_model(outer, inner)
    torch.cuda.synchronize()
    with torch.no_grad():
        last = float(torch.nn.functional.mse_loss(inner(xb), yb))
    flat = np.concatenate([p.detach().cpu().numpy().reshape(-1) for p in inner.parameters()])
    return flat, first, last


def _worker(rank, world, port, out):
    for p in (PKG, REPO, os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["DILOCO_DP_BACKEND"] = "gloo"
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    rec = {}
    for impl in ("reference", "dropin"):
        flat, first, last = _train(rank, world, impl)
        rec[f"{impl}_params"] = flat
        rec[f"{impl}_loss"] = np.array([first, last])
    np.savez(os.path.join(out, f"r{rank}.npz"), **rec)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
def test_diloco_training_loop_matches_reference_outer_step(world):
    out = tempfile.mkdtemp(prefix="dl_loop_")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    recs = [dict(np.load(os.path.join(out, f"r{r}.npz"))) for r in range(world)]
    for r, rec in enumerate(recs):
        assert rec["dropin_params"].tobytes() == rec["reference_params"].tobytes(), r
        first, last = rec["dropin_loss"]
        assert last < 0.8 * first, (first, last)  # the loop trains through the outer steps
        # replicas agree after the last outer step (every rank applied the same average)
        assert rec["dropin_params"].tobytes() == recs[0]["dropin_params"].tobytes()
