"""BASELINE config #3 at its full T125 size, and configs #4 and #5 at their full 1.3B workload (T1.3B: 292 tensors, 1,313,722,368
params, 25 buckets of <= 256 MiB), several replicas on the one GPU of the box.

The collectives are emulated bucket by bucket with torch on the device, in rank order (what
the replicas' RCCL exchange computes up to summation order; RCCL itself carries these paths in
tests/test_rccl_gpu.py at one rank and in bench.py at N > 1):
    config #4  fp32 wire, bucketed: delta_pack(b) -> Σ_r wire_r(b) -> unpack_sgd(b), n = 2;
               the sharded default at DP = 8: delta_pack(b) -> reduce-scatter (Σ, slice r)
               -> dl_shard_sgd -> all-gather -> dl_scatter, n = 8
    config #5  bf16 wire (in-kernel cast) + SGD fused into the unpack, n = 2 and n = 8; and
               with the ordered exchange (exchange="a2a": all_to_all, the n bf16 slices summed
               in fp32 in rank order, never re-rounded), n = 8
Expected values come from the C oracle (oracle/diloco_oracle.c) on sampled tensors -- wte
(103 M elements; a 4 Mi-element window at n = 8), the first block's tensors and the last
tensor -- restated per slice from the counter-based inputs (every step is elementwise), 2
outer steps. fp32: bit-exact (the emulation sums in rank order like the oracle; the
reference's gloo order agrees bit-exactly at n = 2). bf16 wire: bit-exact
against the oracle's restatement of the codec (each delta rounded to bf16 RNE, each partial
sum rounded to bf16, / n in fp32), and every element's update within the a-priori rounding
bound of the codec (codec_bound below) of the fp32 oracle's.
"""
import gc

import numpy as np
import pytest
import torch

from diloco_amd import synth
from diloco_amd.outer import OuterSync, bf16_codec_bound
from diloco_amd.trees import get_tree
from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
F32 = np.float32
SPEC = get_tree("t1.3b")
STEPS = 2


@pytest.fixture(autouse=True)
def _free_hbm():
    yield
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _picks(full_wte, spec=SPEC):
    """(tensor, first element, count): wte, the first block's tensors, the last tensor."""
    numels = spec.numels()
    wte = (0, 0, numels[0]) if full_wte else (0, 37_000_011, 4 << 20)
    return [wte] + [(t, 0, numels[t]) for t in range(1, 10)] + [(len(numels) - 1, 0, numels[-1])]


def _slice_inputs(t, lo, m, step, ranks, theta):
    """Every rank's inner values on elements [lo, lo+m) of tensor t at `step`, given θ there
    (synth.inner_tree restated on a window: u(1000*step + r, t, lo + i))."""
    out = []
    for r in range(ranks):
        u = synth.uniform(synth.noise_seed(step, r), t, m, start=lo)
        x = F32(0.0) + u * F32(synth.NOISE_SCALE)
        out.append((x + theta).astype(F32))
    return out


U_F32 = 2.0 ** -24


def codec_bound(sabs, n, wire):
    """Per-element bound on the averaged g of a bf16 wire against fp32
    (diloco_amd.outer.bf16_codec_bound: the replicated RCCL bf16 all-reduce, or the ordered
    exchange's fp32 rank-order sum of bf16 slices)."""
    return bf16_codec_bound(sabs, n, "a2a" if wire == "bf16_a2a" else "rccl").astype(F32)


def _expected(n, wire, full_wte, spec=SPEC):
    """Oracle θ and momentum on the sampled slices after each of STEPS outer steps; bf16
    wires also carry the per-element codec bound of each step's g (codec_bound)."""
    init = spec.init_spec()
    exp = {}
    for t, lo, m in _picks(full_wte, spec):
        b, sc = init[t]
        th = (F32(b) + synth.uniform(synth.OUTER_SEED, t, m, start=lo) * F32(sc)).astype(F32)
        th32 = th.copy()
        buf, buf32 = np.empty_like(th), np.empty_like(th)
        bound = np.zeros_like(th)
        for s in range(1, STEPS + 1):
            if wire.startswith("bf16"):
                raw = [oracle.delta(th, x) for x in _slice_inputs(t, lo, m, s, n, th)]
                bound = codec_bound(np.sum(np.abs(raw), axis=0, dtype=np.float64), n, wire)
            if wire == "bf16_a2a":
                # exchange="a2a": deltas cast RNE, summed in fp32 in rank order, / n
                g = oracle.sum_avg([oracle.bf16_round(oracle.delta(th, x))
                                    for x in _slice_inputs(t, lo, m, s, n, th)])
                g32 = oracle.sum_avg([oracle.delta(th32, x)
                                      for x in _slice_inputs(t, lo, m, s, n, th32)])
                oracle.sgd(th32, buf32, g32, 0.7, 0.9, True, s == 1)
            elif wire == "bf16":
                # the bf16 wire: deltas cast RNE, partial sums rounded to bf16 (RCCL's bf16
                # reduction, rank order), then g = sum / n in fp32 inside dl_unpack_sgd
                d = [oracle.bf16_round(oracle.delta(th, x))
                     for x in _slice_inputs(t, lo, m, s, n, th)]
                acc = d[0]
                for dr in d[1:]:
                    acc = oracle.bf16_round((acc + dr).astype(F32))
                g = acc if n == 1 else (acc / F32(n)).astype(F32)
                # the fp32 path on the same inner values, for the codec's error bound
                g32 = oracle.sum_avg([oracle.delta(th32, x)
                                      for x in _slice_inputs(t, lo, m, s, n, th32)])
                oracle.sgd(th32, buf32, g32, 0.7, 0.9, True, s == 1)
            else:
                g = oracle.sum_avg([oracle.delta(th, x)
                                    for x in _slice_inputs(t, lo, m, s, n, th)])
            oracle.sgd(th, buf, g, 0.7, 0.9, True, s == 1)
            exp[(t, lo, s)] = (th.copy(), buf.copy(), th32.copy(), bound.copy())
    return exp


def _replicas(n, wire=torch.float32, shard=False, exchange="rccl", spec=SPEC, buckets=25):
    shapes = [s for _, s in spec.params()]
    engines, inners = [], []
    for r in range(n):
        inner = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, DEV), shapes)]
        engines.append(OuterSync(inner, world_size=n, wire_dtype=wire, shard=shard, rank=r,
                                 exchange=exchange))
        inners.append(inner)
    if buckets is not None:
        assert engines[0].tree.n_buckets == buckets
    return engines, inners


def _set_inner(engines, inners, step):
    for r, (e, inner) in enumerate(zip(engines, inners)):
        th = [x.reshape(-1) for x in e.unpacked(e.theta)]
        synth.inner_tree_device(th, step, r, out=[p.view(-1) for p in inner])


def _replicated_step(engines, inners, step):
    """delta_pack(b) on every replica -> Σ in rank order (the all-reduce) -> unpack_sgd(b)."""
    _set_inner(engines, inners, step)
    for b in range(engines[0].tree.n_buckets):
        for e in engines:
            e.pseudo_gradient(b)
        total = engines[0].bucket_view(b).clone()
        for e in engines[1:]:
            total += e.bucket_view(b)  # bf16 wire: each partial sum rounded to bf16
        for e in engines:
            e.bucket_view(b).copy_(total)
            e.apply(b)
        del total
    for e in engines:
        e.steps_done += 1
    torch.cuda.synchronize()


def _sharded_step(engines, inners, step):
    _set_inner(engines, inners, step)
    e0 = engines[0]
    for b in range(e0.tree.n_buckets):
        for e in engines:
            e.pseudo_gradient(b)
        total = engines[0].bucket_view(b).clone()
        for e in engines[1:]:
            total += e.bucket_view(b)
        sl = e0._shard_len(b)
        for r, e in enumerate(engines):
            e._shard(e.g_shard, b).copy_(total[r * sl:(r + 1) * sl])
            e.shard_apply(b)
        del total
        gathered = torch.cat([e.th_shard_view(b) for e in engines])
        lo, hi = e0.tree.bucket_ranges[b]
        for e in engines:
            e.theta[lo:hi].copy_(gathered)
            e.write_inner(b)
        del gathered
    for e in engines:
        e.steps_done += 1
    torch.cuda.synchronize()


def _a2a_step(engines, inners, step):
    """exchange="a2a": delta_pack(b) -> all_to_all (peer r gets slice r of every rank's wire,
    in rank order) -> dl_shard_reduce_sgd -> all-gather -> dl_scatter."""
    _set_inner(engines, inners, step)
    e0 = engines[0]
    for b in range(e0.tree.n_buckets):
        for e in engines:
            e.pseudo_gradient(b)
        sl = e0._shard_len(b)
        for r, e in enumerate(engines):
            recv = e._a2a_slices(b)
            for q, src in enumerate(engines):
                recv[q * sl:(q + 1) * sl].copy_(src.bucket_view(b)[r * sl:(r + 1) * sl])
            e.shard_apply(b)
        gathered = torch.cat([e.th_shard_view(b) for e in engines])
        lo, hi = e0.tree.bucket_ranges[b]
        for e in engines:
            e.theta[lo:hi].copy_(gathered)
            e.write_inner(b)
        del gathered
    for e in engines:
        e.steps_done += 1
    torch.cuda.synchronize()


def _check(engines, inners, exp, step, n, full_wte, wire, sharded=False, spec=SPEC):
    e0 = engines[0]
    mom_full = e0.momentum_full() if not sharded else None
    if sharded:  # assemble the momentum shards of every replica (the all-gather of the state)
        mom_full = torch.zeros_like(e0.theta)
        for b, (lo, hi) in enumerate(e0.tree.bucket_ranges):
            mom_full[lo:hi] = torch.cat([e._shard(e.mom_shard, b) for e in engines])
    worst, worst_ratio = 0.0, 0.0
    for t, lo, m in _picks(full_wte, spec):
        th_exp, buf_exp, th32, bnd = exp[(t, lo, step)]
        o = int(e0.tree.seg_off[t]) + lo
        for e, inner in zip(engines, inners):
            got = e.theta[o:o + m].cpu().numpy()
            assert got.tobytes() == th_exp.tobytes(), (t, lo, step)
            assert inner[t].reshape(-1)[lo:lo + m].cpu().numpy().tobytes() == th_exp.tobytes()
        assert mom_full[o:o + m].cpu().numpy().tobytes() == buf_exp.tobytes(), (t, step)
        if wire.startswith("bf16"):  # the codec's error on the applied update, vs fp32
            th0 = exp[(t, lo, step - 1)][0] if step > 1 else None
            if th0 is not None:
                u_bf, u_32 = th0 - th_exp, exp[(t, lo, step - 1)][2] - th32
            else:
                init = spec.init_spec()[t]
                base = (F32(init[0]) + synth.uniform(synth.OUTER_SEED, t, m, start=lo)
                        * F32(init[1])).astype(F32)
                u_bf, u_32 = base - th_exp, base - th32
            scale = max(float(np.abs(u_32).max()), 1e-30)
            err = np.abs(u_bf - u_32)
            worst = max(worst, float(err.max()) / scale)
            # the update u = θ_{s-1} - θ_s = lr·((1+m)·g_s + m²·buf_{s-1}) (Nesterov): the codec
            # error of g_s and of step s-1's g (buf_1 = g_1), plus a few fp32 ulps of θ for the
            # roundings of the two SGD evaluations and of the θ difference
            prev = exp[(t, lo, step - 1)][3] if step > 1 else np.zeros_like(bnd)
            th_prev = th0 if th0 is not None else base
            e_max = (F32(0.7) * (F32(1.9) * bnd + F32(0.81) * prev)
                     + F32(4 * U_F32) * (np.abs(th_prev) + np.abs(th_exp) + 2 * np.abs(u_32)))
            assert np.all(err <= e_max), (t, step, float((err / e_max).max()))
            worst_ratio = max(worst_ratio, float((err / e_max).max()))
    if wire.startswith("bf16"):
        print(f"bf16 wire {wire} n={n} step {step}: max|du|/max|u| = {worst:.3e}, "
              f"max err/bound = {worst_ratio:.3f}")
    # every replica holds the same full state (a size-independent property over all 1.3 B)
    for e in engines[1:]:
        assert torch.equal(e.theta, e0.theta)


@pytest.mark.parametrize("wire", ["f32", "bf16"])
def test_t13b_two_replicas_bucketed_exchange(wire):
    """Configs #4 (fp32) / #5 (bf16 wire + SGD fused into the unpack) at 1.3B, n = 2, the
    25-bucket replicated path, 2 outer steps, wte compared whole."""
    wdt = torch.float32 if wire == "f32" else torch.bfloat16
    exp = _expected(2, wire, full_wte=True)
    engines, inners = _replicas(2, wdt)
    for s in range(1, STEPS + 1):
        _replicated_step(engines, inners, s)
        _check(engines, inners, exp, s, 2, True, wire)
    for e in engines:
        e.close()


def test_t13b_eight_replicas_sharded_fp32():
    """Config #4 at DP = 8 (the n > 1 default: reduce-scatter -> shard SGD -> all-gather ->
    scatter), 1.3B, 8 replicas on one GPU (~18 GB each), 2 outer steps."""
    exp = _expected(8, "f32", full_wte=False)
    engines, inners = _replicas(8, shard=True)
    assert engines[0].sharded and engines[0].tree.total % (64 * 8) == 0
    for s in range(1, STEPS + 1):
        _sharded_step(engines, inners, s)
        _check(engines, inners, exp, s, 8, False, "f32", sharded=True)
    for e in engines:
        e.close()


def test_t13b_eight_replicas_bf16_wire():
    """Config #5 at DP = 8: bf16 wire (replicated all-reduce, the bf16 default) + SGD fused
    into the unpack, 1.3B, 8 replicas, 2 outer steps."""
    exp = _expected(8, "bf16", full_wte=False)
    engines, inners = _replicas(8, torch.bfloat16)
    assert not engines[0].sharded
    for s in range(1, STEPS + 1):
        _replicated_step(engines, inners, s)
        _check(engines, inners, exp, s, 8, False, "bf16")
    for e in engines:
        e.close()


def test_t13b_eight_replicas_bf16_wire_ordered_exchange():
    """Config #5 at DP = 8 with exchange="a2a": the bf16 slices of every replica summed in fp32
    in rank order by dl_shard_reduce_sgd (SGD on the shard), all-gather, scatter; bit-exact
    against the oracle's restatement, within 2^-8 of the fp32 oracle at any n."""
    exp = _expected(8, "bf16_a2a", full_wte=False)
    engines, inners = _replicas(8, torch.bfloat16, shard=None, exchange="a2a")
    assert engines[0].sharded and engines[0].a2a
    for s in range(1, STEPS + 1):
        _a2a_step(engines, inners, s)
        _check(engines, inners, exp, s, 8, False, "bf16_a2a", sharded=True)
    for e in engines:
        e.close()


T125 = get_tree("t125")


@pytest.mark.parametrize("path", ["replicated", "sharded"])
def test_t125_two_replicas_config3_vs_oracle(path):
    """BASELINE config #3 (T125: 148 tensors, 124,475,904 params, DP = 2, fp32) at full size
    against the C oracle (src/comm.py:122-123, src/utils.py:221): 2 emulated replicas, 2 outer
    steps, through the replicated path (delta_pack -> Σ -> unpack_sgd with the inner write)
    and the sharded one (reduce-scatter -> dl_shard_sgd -> all-gather -> dl_scatter). θ, the
    momentum and the inner params bit-exact on wte (38.6 M elements, whole), the first block
    and the last tensor; every replica's whole θ identical."""
    exp = _expected(2, "f32", full_wte=True, spec=T125)
    engines, inners = _replicas(2, shard=path == "sharded", spec=T125, buckets=None)
    assert engines[0].tree.n_buckets >= 2  # 256 MiB buckets: the bucketed exchange
    assert engines[0].sharded == (path == "sharded")
    step = _sharded_step if path == "sharded" else _replicated_step
    for s in range(1, STEPS + 1):
        step(engines, inners, s)
        _check(engines, inners, exp, s, 2, True, "f32", sharded=path == "sharded", spec=T125)
    for e in engines:
        e.close()
