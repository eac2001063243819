"""Pin the CPU oracle to the reference's own outputs (golden fixtures) -- CPU only.

The fixtures were produced by running the reference's compute_pseudo_gradient /
TrainingComm.sync_gradients (gloo) / get_optimizer SGD-Nesterov / sync_inner_model under
torchrun (tests/golden/make_golden.py). Bit-exact at n <= 2; normwise 1e-6 at n = 4, where the
reference's gloo summation order is not rank order.
"""
import hashlib

import numpy as np
import pytest
import torch

from conftest import load_json, load_npz, normwise_ok, split
from diloco_amd import synth
from diloco_amd.trees import TREES, get_tree
from oracle import oracle


def test_tree_specs_match_reference_parameters():
    ref = load_json("trees.json")
    for name, spec in TREES.items():
        got = [(n, list(s)) for n, s in spec.params()]
        assert got == [(x[0], x[1]) for x in ref[name]["params"]], name
        assert spec.total() == ref[name]["total"]
    # SURVEY.md §8d sizes
    assert (len(TREES["t125"].params()), TREES["t125"].total()) == (148, 124_475_904)
    assert (len(TREES["t1.3b"].params()), TREES["t1.3b"].total()) == (292, 1_313_722_368)
    assert (len(TREES["tiny"].params()), TREES["tiny"].total()) == (53, 13_802_240)


@pytest.mark.parametrize("n,seed,stream,base,scale", [
    (1, 42, 0, 0.0, 0.02), (1000, 42, 7, 1.0, 0.5), (4099, 2001, 291, 0.0, 1e-3),
])
def test_synth_numpy_equals_c_generator(n, seed, stream, base, scale):
    add = np.linspace(-1, 1, n, dtype=np.float32)
    a = synth.values(seed, stream, n, base, scale, add=add)
    b = oracle.fill_synth(n, seed, stream, base, scale, add=add)
    assert a.tobytes() == b.tobytes()
    u = synth.uniform(seed, stream, n)
    assert u.min() >= -1.0 and u.max() < 1.0


def test_micro_inputs_regenerate_bit_exact():
    spec = get_tree("micro")
    g = load_npz("micro_n1.npz")
    theta0 = synth.outer_tree(spec.numels(), spec.init_spec())
    assert np.concatenate(theta0).tobytes() == g["theta0"].tobytes()
    inner = synth.inner_tree(theta0, 1, 0)
    assert np.concatenate(inner).tobytes() == g["inner_s1_r0"].tobytes()


def _run_oracle(spec, n, steps=2):
    numels = spec.numels()
    st = oracle.OuterState(synth.outer_tree(numels, spec.init_spec()))
    out = {}
    for s in range(1, steps + 1):
        inners = [synth.inner_tree(st.theta, s, r) for r in range(n)]
        deltas, avg = st.step(inners)
        out[f"delta_s{s}_r0"] = np.concatenate(deltas[0])
        out[f"delta_s{s}_rlast"] = np.concatenate(deltas[-1])
        out[f"avg_s{s}"] = np.concatenate(avg)
        out[f"theta_s{s}"] = np.concatenate(st.theta)
        out[f"buf_s{s}"] = np.concatenate(st.buf)
    return out


@pytest.mark.parametrize("n", [1, 2])
def test_oracle_matches_reference_micro_bit_exact(n):
    g = load_npz(f"micro_n{n}.npz")
    got = _run_oracle(get_tree("micro"), n)
    for k, v in got.items():
        assert v.tobytes() == g[k].tobytes(), k


@pytest.mark.parametrize("n", [4, 8])  # 8: the north star's DP = 8
def test_oracle_matches_reference_micro_normwise(n):
    spec = get_tree("micro")
    g = load_npz(f"micro_n{n}.npz")
    got = _run_oracle(spec, n)
    for k in ("delta_s1_r0", "delta_s1_rlast"):
        assert got[k].tobytes() == g[k].tobytes(), k  # step-1 per-rank deltas are exact
    # from step 2 on, θ carries the step-1 summation-order difference
    for k in ("delta_s2_r0", "avg_s1", "avg_s2", "theta_s1", "theta_s2", "buf_s1", "buf_s2"):
        for a, b in zip(split(got[k], spec.numels()), split(g[k], spec.numels())):
            assert normwise_ok(a, b, 1e-6), k


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()


@pytest.mark.parametrize("n", [1, 2, 4])
def test_oracle_matches_reference_tiny_digests(n):
    spec = get_tree("tiny")
    ref = load_json("tiny_digests.json")[str(n)]
    got = _run_oracle(spec, n)
    numels = spec.numels()
    for s in (1, 2):
        for key in (f"delta_s{s}", f"avg_s{s}", f"theta_s{s}", f"buf_s{s}"):
            flat = got[f"{key}_r0"] if key.startswith("delta") else got[key]
            for t, (a, d) in enumerate(zip(split(flat, numels), ref["rank0"][key])):
                if n <= 2 or key == "delta_s1":
                    assert _sha(a) == d["sha256"], (key, t)
                else:
                    l2 = float(np.sqrt((a.astype(np.float64) ** 2).sum()))
                    assert abs(l2 - d["l2"]) <= 1e-6 * max(d["l2"], 1e-30), (key, t)


# ---- the arithmetic the oracle restates, against torch itself ---------------------------------
@pytest.mark.parametrize("n", [1, 3, 17, 1000, 4099])
@pytest.mark.parametrize("momentum,nesterov", [(0.9, True), (0.9, False), (0.0, False), (0.5, True)])
def test_oracle_sgd_equals_torch_sgd(n, momentum, nesterov):
    g0 = torch.Generator().manual_seed(n)
    p = torch.randn(n, generator=g0)
    theta = p.numpy().copy()
    buf = np.zeros(n, dtype=np.float32)
    opt = torch.optim.SGD([p], lr=0.7, momentum=momentum, nesterov=nesterov)
    for step in range(3):
        g = torch.randn(n, generator=g0) * 1e-3
        p.grad = g.clone()
        opt.step()
        oracle.sgd(theta, buf, g.numpy().copy(), 0.7, momentum, nesterov, step == 0)
        assert theta.tobytes() == p.detach().numpy().tobytes()
        if momentum:
            assert buf.tobytes() == opt.state[p]["momentum_buffer"].numpy().tobytes()


@pytest.mark.parametrize("nranks", [1, 2, 3, 5, 8])
def test_oracle_average_is_true_division(nranks):
    g0 = torch.Generator().manual_seed(nranks)
    xs = [torch.randn(4099, generator=g0) for _ in range(nranks)]
    s = xs[0].clone()
    for x in xs[1:]:
        s += x
    if nranks > 1:
        s /= nranks  # src/comm.py:123 (int divisor)
    got = oracle.sum_avg([x.numpy() for x in xs])
    assert got.tobytes() == s.numpy().tobytes()


def test_oracle_bf16_round_equals_torch():
    x = torch.randn(10007) * 3
    x[:4] = torch.tensor([float("inf"), -float("inf"), float("nan"), 0.0])
    ref = x.to(torch.bfloat16).float().numpy()
    got = oracle.bf16_round(x.numpy())
    assert np.array_equal(np.isnan(ref), np.isnan(got))
    m = ~np.isnan(ref)
    assert got[m].tobytes() == ref[m].tobytes()


def test_oracle_plan_rule_matches_fixture():
    ref = load_json("plan_tables.json")
    for name in ("micro", "tiny", "t125", "t1.3b"):
        numels = ref[name]["numels"]
        assert numels == get_tree(name).numels()
        for p in ref[name]["plans"]:
            seg, bnd = oracle.plan_tables(numels, p["cap"], p["align"])
            assert seg.tolist() == p["seg_off"] and bnd.tolist() == p["bkt_bounds"]
    for e in ref["edge"]:
        seg, bnd = oracle.plan_tables(e["numels"], e["cap"], e["align"])
        assert seg.tolist() == e["seg_off"] and bnd.tolist() == e["bkt_bounds"], e
