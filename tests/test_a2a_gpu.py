"""exchange="a2a": the sharded outer step with an all_to_all of the wire slices and a
rank-order reduce (dl_shard_reduce_sgd) in place of the SUM reduce-scatter.

The reduce sums the n copies of a shard in rank order in fp32 (a bf16 wire is summed in fp32
and never re-rounded), which is oracle/or_sum_avg's order: the result is bit-exact against the
oracle's restatement at every n, whatever RCCL's algorithm. Here: the kernel against the oracle
(n = 1 ... 8 compiled, 11 through the run-time-n path), and n replicas on one GPU with the
all_to_all / all_gather emulated, against the oracle (fp32 and bf16 wires) and the reference
fixtures (fp32, n <= 2 bit-exact; n = 4, 8 normwise). The RCCL transport itself is exercised
over a one-rank communicator in tests/test_rccl_gpu.py and over gloo ranks on CPU in
tests/test_dist_gloo.py.
"""
import numpy as np
import pytest
import torch

from conftest import load_npz, normwise_ok, split
from diloco_amd import synth
from diloco_amd.outer import OuterSync
from diloco_amd.trees import get_tree
from expect import expected_rank_order
from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _host(ts):
    return [t.detach().reshape(-1).float().cpu().numpy() for t in ts]


@pytest.mark.parametrize("wire", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 11])
@pytest.mark.parametrize("momentum,nesterov", [(0.9, True), (0.9, False), (0.0, False)])
def test_shard_reduce_sgd_matches_oracle(wire, n, momentum, nesterov):
    """dl_shard_reduce_sgd == oracle.sum_avg over the slices (rank order) + oracle.sgd, bit-exact,
    first and steady-state steps, lengths from one float4 to several rounds of workgroups."""
    from diloco_amd.kernels import default_kernels

    k = default_kernels()
    for length in (4, 64, 2048 + 4, 3 * 2048 * 256 + 64 * 7 + 12):
        sl = [synth.values(50 + q, length, length, 0.0, 1e-3) for q in range(n)]
        if wire == torch.bfloat16:
            sl = [oracle.bf16_round(x) for x in sl]
        dev_sl = torch.from_numpy(np.concatenate(sl)).to(DEV).to(wire)
        th = synth.values(6, n, length, 0.0, 0.02)
        buf = synth.values(7, n, length, 0.0, 1e-3)
        dth = torch.from_numpy(th.copy()).to(DEV)
        dm = torch.from_numpy(buf.copy()).to(DEV) if momentum else None
        rth, rbuf = th.copy(), buf.copy()
        g = oracle.sum_avg(sl)
        for first in (True, False):
            k.shard_reduce_sgd(dev_sl, n, dth, dm, 0.7, momentum, nesterov, first)
            oracle.sgd(rth, rbuf if momentum else None, g, 0.7, momentum, nesterov, first)
        torch.cuda.synchronize()
        assert dth.cpu().numpy().tobytes() == rth.tobytes(), length
        if momentum:
            assert dm.cpu().numpy().tobytes() == rbuf.tobytes(), length


@pytest.mark.parametrize("wire", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 11])
def test_shard_reduce_avg_matches_oracle(wire, n):
    """dl_shard_reduce_avg (GradSync(exchange="a2a")'s reduce) == oracle.sum_avg, bit-exact,
    IEEE specials included (signed zeros survive: no SGD arithmetic touches the average)."""
    from diloco_amd.kernels import default_kernels

    k = default_kernels()
    for length in (4, 2048 + 4, 3 * 2048 * 256 + 64 * 7 + 12):
        sl = [synth.values(70 + q, length, length, 0.0, 1.0) for q in range(n)]
        sl[0][:4] = [-0.0, 0.0, np.inf, -1e-40]
        if wire == torch.bfloat16:
            sl = [oracle.bf16_round(x) for x in sl]
        out = torch.full((length,), 7.0, device=DEV)
        k.shard_reduce_avg(torch.from_numpy(np.concatenate(sl)).to(DEV).to(wire), n, out)
        torch.cuda.synchronize()
        assert out.cpu().numpy().tobytes() == oracle.sum_avg(sl).tobytes(), length


def _emulated_a2a_steps(n, wire, steps=2):
    """n replicas of the micro tree on this GPU, exchange="a2a", collectives emulated:
    all_to_all = peer r receives slice r of every rank's wire bucket, in rank order;
    all_gather = concatenation of the θ shards. Yields (step, engines, inners)."""
    spec = get_tree("micro")
    theta0 = synth.outer_tree_device(spec, DEV)
    shapes = [s for _, s in spec.params()]
    engines, inners = [], []
    for r in range(n):
        inner = [t.clone().view(s) for t, s in zip(theta0, shapes)]
        engines.append(OuterSync(inner, world_size=n, bucket_cap_elems=4096, exchange="a2a",
                                 wire_dtype=wire, rank=r))
        inners.append(inner)
    e0 = engines[0]
    assert e0.sharded and e0.a2a and e0.tree.n_buckets > 2
    for s in range(1, steps + 1):
        for r, (e, inner) in enumerate(zip(engines, inners)):
            th = [t.reshape(-1) for t in e.unpacked(e.theta)]
            synth.inner_tree_device(th, s, r, out=[p.view(-1) for p in inner])
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
        for e in engines:
            e.steps_done += 1
        torch.cuda.synchronize()
        yield s, engines, inners


def _mom_full(engines):
    e0 = engines[0]
    out = torch.zeros_like(e0.theta)
    for b in range(e0.tree.n_buckets):
        lo, hi = e0.tree.bucket_ranges[b]
        out[lo:hi] = torch.cat([e._shard(e.mom_shard, b) for e in engines])
    return out


@pytest.mark.parametrize("wire", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_a2a_step_emulated_is_bit_exact_against_rank_order_oracle(wire, n):
    exp = expected_rank_order(n, wire="bf16" if wire == torch.bfloat16 else "f32")
    g = load_npz(f"micro_n{n}.npz")
    numels = get_tree("micro").numels()
    for s, engines, inners in _emulated_a2a_steps(n, wire):
        e0 = engines[0]
        th = np.concatenate(_host(e0.unpacked(e0.theta)))
        buf = np.concatenate(_host(e0.unpacked(_mom_full(engines))))
        assert th.tobytes() == exp[f"theta_s{s}"].tobytes(), s
        assert buf.tobytes() == exp[f"buf_s{s}"].tobytes(), s
        for e, inner in zip(engines, inners):  # every replica holds the same θ and inner
            assert np.concatenate(_host(e.unpacked(e.theta))).tobytes() == th.tobytes()
            assert np.concatenate(_host(inner)).tobytes() == th.tobytes()
        if wire == torch.float32:  # and the reference's own gloo run
            if n <= 2:
                assert th.tobytes() == g[f"theta_s{s}"].tobytes(), s
                assert buf.tobytes() == g[f"buf_s{s}"].tobytes(), s
            else:
                for a, b in zip(split(th, numels), split(g[f"theta_s{s}"], numels)):
                    assert normwise_ok(a, b, 1e-6), s
        else:  # the bf16 wire stays within the codec's bound of the fp32 reference
            ref = g[f"theta_s{s}"] - g["theta0"] if s == 1 else None
            if ref is not None:
                got = th - g["theta0"]
                assert np.linalg.norm(got - ref) <= 2.0 ** -8 * np.linalg.norm(ref), s
