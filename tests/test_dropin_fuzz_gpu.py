"""Seeded random trees through the reference's four calls (src/train.py:263-269) with the HIP
kernels and three processes on the one GPU (gloo DP group: RCCL refuses two ranks per
device), against the C oracle (ragged inputs, empty tensors, many small buckets;
§8a rows a1-a5 behind §8b1's surface).

Each case draws a tree (1-30 tensors: empty, tiny, chunk-boundary and up to 200k-element
tensors, some 2-D), a bucket cap (one chunk to larger than the tree), the outer model's
placement (the default lazy host, or HBM), the exchange behind sync_gradients (the default
sharded reduce_scatter -> shard SGD -> all_gather, the replicated all_reduce, the rank-order
all_to_all) or the int8 wire, the SGD configuration, and whether anything reads .grad between
the calls; three outer steps. Checked every step: θ, the momentum (opt.state, gathered),
.grad (the average) and the inner params (= θ), against the oracle -- byte-equal for the
rank-order exchange and the int8 wire, normwise 1e-6 per tensor for the RCCL-style sums
(gloo's order at 3 peers) -- and θ identical on every rank."""
import hashlib
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

WORLD = 3
CASES = 12


class _Cfg:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def _tree(rng):
    k = int(rng.integers(1, 31))
    numels = []
    for kind in rng.integers(0, 5, size=k):
        if kind == 0:
            numels.append(int(rng.integers(0, 11)))          # empty / tiny
        elif kind == 1:
            numels.append(int(rng.integers(11, 4096)))
        elif kind == 2:                                       # around a chunk boundary
            numels.append(4096 * int(rng.integers(1, 4)) + int(rng.integers(-3, 4)))
        elif kind == 3:
            numels.append(int(rng.integers(4096, 40000)))
        else:
            numels.append(int(rng.integers(40000, 200000)))
    if not any(numels):
        numels[0] = 1
    return numels


def _shape(n, rng):
    for d in (64, 32, 8, 3):
        if n and n % d == 0 and rng.integers(0, 2):
            return (n // d, d)
    return (n,)


def _case(case):
    rng = np.random.default_rng(7000 + case)
    numels = _tree(rng)
    c = dict(numels=numels, shapes=[_shape(n, rng) for n in numels],
             cap=int(rng.choice([4096, 8192, 50000, 1 << 20])),
             placement=[None, "device"][case % 2],
             exchange=["sharded", "replicated", "a2a", "int8"][(case // 2) % 4],
             sgd=[(0.9, True), (0.9, False), (0.0, False)][int(rng.integers(0, 3))],
             lr=float(rng.choice([0.7, 0.3])), quiet=bool(rng.integers(0, 2)))
    c["theta0"] = [(rng.standard_normal(n) * 0.02).astype(np.float32) for n in numels]
    return c


def _inner(theta, step, rank):
    """Every rank's inner tree, generated on each rank alike (a stand-in for H inner steps)."""
    g = np.random.default_rng(100000 + 1000 * step + rank)
    return [(t + g.standard_normal(t.size).astype(np.float32) * 1e-3).astype(np.float32)
            for t in theta]


def _close(got, want, exact):
    if exact:
        return got.tobytes() == want.tobytes()
    den = float(np.linalg.norm(want.astype(np.float64)))
    num = float(np.linalg.norm(got.astype(np.float64) - want.astype(np.float64)))
    return num <= 1e-6 * max(den, 1e-30)


def _run_case(case, rank, world, dev):
    from diloco_amd.comm import TrainingComm
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  outer_mirror, sync_inner_model)
    from diloco_amd.world import World
    from oracle import oracle

    c = _case(case)
    numels, shapes = c["numels"], c["shapes"]
    momentum, nesterov = c["sgd"]
    os.environ["DILOCO_OUTER_BUCKET_ELEMS"] = str(c["cap"])
    inner = torch.nn.Module()
    inner.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.from_numpy(t.copy()).view(s))
                                       for t, s in zip(c["theta0"], shapes)])
    wire = "int8" if c["exchange"] == "int8" else None
    # every exchange by name: the placements' defaults differ (host replicated, device sharded)
    exchange = None if c["exchange"] == "int8" else c["exchange"]
    outer = get_outer_model(inner, c["placement"], wire=wire, exchange=exchange)
    inner = inner.to(dev)
    opt = get_optimizer(outer, _Cfg(type="SGD", lr=c["lr"], momentum=momentum,
                                    nesterov=nesterov))
    comm = TrainingComm(World.from_default_group(1), (1, 1, 8), None)
    m = outer_mirror(outer, dev)  # the device outer model takes the inner model's device
    if c["placement"] == "device":  # its parameters now live in the HBM arena
        assert all(p.device == torch.device(dev) for p in outer.parameters()), (
            case, [str(p.device) for p in outer.parameters()])
    tree = getattr(m, "dev", m).tree
    st = oracle.OuterState(c["theta0"], lr=c["lr"], momentum=momentum, nesterov=nesterov)
    exact = c["exchange"] in ("a2a", "int8")
    where = {k: c[k] for k in ("exchange", "placement", "cap", "sgd", "lr", "quiet")}
    bad = []

    def flat(ts):
        return [t.detach().cpu().numpy().reshape(-1) for t in ts]

    def check(name, got, want, s):
        for t, (a, b) in enumerate(zip(got, want)):
            if not _close(a, b, exact):
                bad.append(f"case {case} {where} step {s} {name} tensor {t} numel {numels[t]}")
                return

    for s in (1, 2, 3):
        inners = [_inner(st.theta, s, r) for r in range(world)]
        with torch.no_grad():
            for p, v in zip(inner.parameters(), inners[rank]):
                p.copy_(torch.from_numpy(v).view(p.shape))
        if c["exchange"] == "int8":
            first = st.steps == 0
            deltas = [[oracle.delta(st.theta[t], ir[t]) for t in range(len(numels))]
                      for ir in inners]
            avg = oracle.q8_average(deltas, numels,
                                    [c1 - c0 for c0, c1 in tree.bucket_chunks])
            for t in range(len(numels)):
                if momentum and st.buf[t] is None:
                    st.buf[t] = np.empty_like(st.theta[t])
                oracle.sgd(st.theta[t], st.buf[t], avg[t], st.lr, momentum, nesterov, first)
            st.steps += 1
        else:
            _, avg = st.step(inners)
        compute_pseudo_gradient(inner, outer)
        comm.sync_gradients(outer)
        if not c["quiet"]:
            check("avg (read between the calls)", flat(p.grad for p in outer.parameters()),
                  avg, s)
        opt.step()
        sync_inner_model(outer, inner)
        theta = flat(outer.parameters())
        check("theta", theta, st.theta, s)
        check("avg", flat(p.grad for p in outer.parameters()), avg, s)
        if momentum:
            check("momentum", flat(opt.state[p]["momentum_buffer"] for p in outer.parameters()),
                  st.buf, s)
        if dev != "cpu":
            torch.cuda.synchronize()
        if any(a.tobytes() != b.tobytes() for a, b in zip(flat(inner.parameters()), theta)):
            bad.append(f"case {case} {where} step {s}: inner != theta")
        h = hashlib.sha256(b"".join(t.tobytes() for t in theta)).hexdigest()
        hs = [None] * world
        dist.all_gather_object(hs, h)
        if len(set(hs)) != 1:
            bad.append(f"case {case} {where} step {s}: replicas differ")
    return bad


def _worker(rank, world, port, out, dev, cases):
    for p in (PKG, REPO, os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["DILOCO_DP_BACKEND"] = "gloo"
    if dev == "cpu":  # the orchestration on CPU, the oracle checker as the kernel backend
        from diloco_amd import kernels
        from oracle_kernels import OracleKernels

        torch.set_num_threads(1)
        kernels.set_default_kernels(OracleKernels())
    else:
        torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    bad = []
    for case in cases:
        bad += _run_case(case, rank, world, dev)
    with open(os.path.join(out, f"r{rank}.txt"), "w") as f:
        f.write("\n".join(bad))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(dev, cases):
    out = tempfile.mkdtemp(prefix="dl_fuzz_")
    # CPU: forked workers (no HIP state in this process to inherit); the GPU: fresh ones
    mp.start_processes(_worker, args=(WORLD, _free_port(), out, dev, list(cases)), nprocs=WORLD,
                       join=True, start_method="fork" if dev == "cpu" else "spawn")
    bad = []
    for r in range(WORLD):
        with open(os.path.join(out, f"r{r}.txt")) as f:
            bad += [ln for ln in f.read().splitlines() if ln]
    assert not bad, "\n".join(bad[:20])


@pytest.mark.gpu
def test_random_trees_through_the_reference_calls_three_peers():
    """Every case with the HIP kernels on the GPU."""
    _spawn("cuda:0", range(CASES))


def test_random_trees_through_the_reference_calls_three_peers_cpu():
    """The first eight cases (every placement x exchange) on CPU: the orchestration above the
    kernels with the oracle checker as the backend."""
    _spawn("cpu", range(8))


def test_case_table_covers_every_form():
    """The seeded draw covers both placements x every exchange, empty tensors and caps below
    the largest tensor (host only: no GPU work)."""
    cs = [_case(i) for i in range(CASES)]
    assert {(c["placement"], c["exchange"]) for c in cs} == {
        (p, e) for p in (None, "device") for e in ("sharded", "replicated", "a2a", "int8")}
    assert any(0 in c["numels"] for c in cs)
    assert any(c["cap"] < max(c["numels"]) for c in cs)
    assert {c["quiet"] for c in cs} == {True, False}
