"""Seeded random trees through every one-replica engine variant and the emulated n-replica
exchange, against the C oracle, bit-exact (ragged inputs, empty tensors, unaligned
storage, many small buckets; §8a rows a2-a5).

Each case draws a tree (1-40 tensors: empty, tiny, chunk-boundary and up to 300k-element
tensors), places every tensor at a random 0-3 element offset inside one allocation (16-B and
4-B aligned storage: the vector and the scalar paths), a bucket cap (from one chunk to larger
than the tree), an SGD mode and a learning rate, then runs three outer steps (the first-step
and the steady-state momentum modes) and checks θ_outer, the momentum, the inner parameters
(= θ after the step), the kept pseudo-gradient where the variant keeps one, and that the
alignment padding of the packed θ stays zero."""
import numpy as np
import pytest
import torch

from diloco_amd.outer import OuterSync
from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
VARIANTS = ["fused_keep_wire", "fused", "two_kernel_f32", "two_kernel_bf16", "tiled_f32",
            "tiled_bf16", "int8", "replicas_2", "replicas_3", "replicas_4"]
CASES = 30


def _tree(rng):
    k = int(rng.integers(1, 41))
    kinds = rng.integers(0, 5, size=k)
    numels = []
    for kind in kinds:
        if kind == 0:
            numels.append(int(rng.integers(0, 11)))          # empty / tiny
        elif kind == 1:
            numels.append(int(rng.integers(11, 4096)))
        elif kind == 2:                                       # around a chunk boundary
            numels.append(4096 * int(rng.integers(1, 4)) + int(rng.integers(-3, 4)))
        elif kind == 3:
            numels.append(int(rng.integers(4096, 40000)))
        else:
            numels.append(int(rng.integers(40000, 300000)))
    if not any(numels):
        numels[0] = 1
    return numels


def _place(rng, host):
    """Device copies of the host tensors at random 0-3 element offsets in one allocation."""
    offs = [int(rng.integers(0, 4)) for _ in host]
    base = torch.zeros(sum(h.size + o for h, o in zip(host, offs)) + 4, device=DEV)
    params, at = [], 0
    for h, o in zip(host, offs):
        at += o
        p = base[at:at + h.size]
        p.copy_(torch.from_numpy(h))
        params.append(p)
        at += h.size
    return base, params


def _h(t):
    return t.detach().reshape(-1).cpu().numpy()


def _oracle_q8_step(st, inner, numels, bucket_chunks):
    deltas = [oracle.delta(st.theta[t], inner[t]) for t in range(len(numels))]
    g = oracle.q8_average([deltas], numels, bucket_chunks)
    first = st.steps == 0
    for t in range(len(numels)):
        if st.momentum != 0 and st.buf[t] is None:
            st.buf[t] = np.empty_like(st.theta[t])
        oracle.sgd(st.theta[t], st.buf[t], g[t], st.lr, st.momentum, st.nesterov, first)
    st.steps += 1
    return deltas


@pytest.mark.parametrize("case", range(CASES))
def test_random_tree_matches_oracle(case):
    rng = np.random.default_rng(1000 + case)
    variant = VARIANTS[case % len(VARIANTS)]
    numels = _tree(rng)
    cap = int(rng.choice([4096, 8192, 50000, 1 << 20, 64 << 20]))
    momentum, nesterov = [(0.9, True), (0.9, False), (0.0, False)][int(rng.integers(0, 3))]
    lr = float(rng.choice([0.7, 0.3]))
    n = int(variant.split("_")[1]) if variant.startswith("replicas") else 1
    wire = ("bf16" if variant.endswith("bf16") else "int8" if variant == "int8" else "f32")
    dtype = {"f32": torch.float32, "bf16": torch.bfloat16, "int8": torch.int8}[wire]
    theta0 = [(rng.standard_normal(m) * 0.02).astype(np.float32) for m in numels]
    bases, replicas = [], []
    for _ in range(n):
        base, params = _place(rng, theta0)
        bases.append(base)
        replicas.append(params)
    kw = dict(lr=lr, momentum=momentum, nesterov=nesterov, world_size=n,
              bucket_cap_elems=cap, wire_dtype=dtype)
    if variant == "fused_keep_wire":
        kw.update(fuse_single=True, keep_wire=True)
    elif variant == "fused":
        kw.update(fuse_single=True)
    elif variant.startswith("two_kernel"):
        kw.update(fuse_single=False, tile_chunks=0)
    elif variant.startswith("tiled"):
        kw.update(fuse_single=False, tile_chunks=int(rng.choice([1, 2, 3, 7])))
    elif n > 1:
        kw.update(shard=False)
    engines = [OuterSync(p, **kw) for p in replicas]
    e0 = engines[0]
    st = oracle.OuterState(theta0, lr=lr, momentum=momentum, nesterov=nesterov)
    where = f"case {case} {variant} cap {cap} m {momentum} nesterov {nesterov} tree {numels}"
    for step in range(3):
        inners = []
        for r, params in enumerate(replicas):
            inner = [(t + rng.standard_normal(t.size).astype(np.float32) * 1e-3).astype(np.float32)
                     for t in st.theta]
            for p, x in zip(params, inner):
                p.copy_(torch.from_numpy(x))
            inners.append(inner)
        if wire == "int8":
            deltas = [_oracle_q8_step(st, inners[0], numels,
                                      [c1 - c0 for c0, c1 in e0.tree.bucket_chunks])]
        else:
            deltas, _ = st.step(inners, wire=wire)
        if n == 1:
            e0.step()
        else:  # the replicated exchange, the all-reduce emulated on the device in rank order
            for e in engines:
                e.pseudo_gradient()
            total = engines[0].wire.clone()
            for e in engines[1:]:
                total += e.wire
            for e in engines:
                e.wire.copy_(total)
                e.apply()
                e.steps_done += 1
        torch.cuda.synchronize()
        for r, (e, params) in enumerate(zip(engines, replicas)):
            th = e.unpacked(e.theta)
            for t in range(len(numels)):
                got = _h(th[t])
                assert got.tobytes() == st.theta[t].tobytes(), (where, step, r, t, "theta")
                assert _h(params[t]).tobytes() == got.tobytes(), (where, step, r, t, "inner")
                if momentum:
                    assert _h(e.unpacked(e.mom)[t]).tobytes() == st.buf[t].tobytes(), \
                        (where, step, r, t, "momentum")
                if variant in ("fused_keep_wire", "two_kernel_f32", "tiled_f32"):
                    assert _h(e.unpacked(e.wire)[t]).tobytes() == deltas[0][t].tobytes(), \
                        (where, step, t, "wire")
            mask = torch.ones(e.tree.total, dtype=torch.bool, device=DEV)
            for t, m in enumerate(numels):
                lo = int(e.tree.seg_off[t])
                mask[lo:lo + m] = False
            assert not e.theta[mask].any(), (where, step, "padding")
    for e in engines:
        e.close()
