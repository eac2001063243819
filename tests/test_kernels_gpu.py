"""Parity of the HIP path (through the C-ABI) against the reference's outputs and the oracle.

Bit-exact wherever the reference is deterministic: n = 1 and n = 2 (an all-reduce of two
values is order-free), every per-rank delta, the copy-back and the integer tables. The n = 2
all-reduce is emulated on one GPU by summing the two replicas' wire buffers (the RCCL step
itself is exercised by bench.py at N > 1 and by tests/test_dist_gloo.py on CPU).
"""
import hashlib

import numpy as np
import pytest
import torch

from conftest import load_json, load_npz, split
from diloco_amd import _lib, synth
from diloco_amd.outer import OuterSync
from diloco_amd.plan import SLOT_GRAD, SLOT_INNER, PackedTree
from diloco_amd.trees import get_tree
from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()


def _host(ts):
    return [t.detach().reshape(-1).cpu().numpy() for t in ts]


def _engines(spec, n, wire=torch.float32, cap=None, **kw):
    """n replicas of one tree on this GPU, θ_0 from synth, as get_outer_model sees it."""
    theta0 = synth.outer_tree_device(spec, DEV)
    shapes = [s for _, s in spec.params()]
    engines, inners = [], []
    for _ in range(n):
        inner = [t.clone().view(s) for t, s in zip(theta0, shapes)]
        extra = {} if cap is None else {"bucket_cap_elems": cap}
        kw.setdefault("shard", False)  # the emulated all-reduce drives the replicated variant
        engines.append(OuterSync(inner, world_size=n, wire_dtype=wire, **extra, **kw))
        inners.append(inner)
    return engines, inners


def _emulated_step(engines, inners, step, per_bucket=False):
    """One outer step of n replicas on one GPU; returns each replica's delta (host)."""
    n = len(engines)
    for r, (e, inner) in enumerate(zip(engines, inners)):
        theta = e.unpacked(e.theta)
        synth.inner_tree_device([t.reshape(-1) for t in theta], step, r,
                                out=[p.view(-1) for p in inner])
    buckets = range(engines[0].tree.n_buckets) if per_bucket else [_lib.ALL_BUCKETS]
    deltas = [None] * n
    for b in buckets:
        for e in engines:
            e.pseudo_gradient(b)
    for r, e in enumerate(engines):
        deltas[r] = _host(e.unpacked(e.wire.float()))
    if n > 1:
        total = engines[0].wire.clone()
        for e in engines[1:]:
            total += e.wire
        for e in engines:
            e.wire.copy_(total)
    for b in buckets:
        for e in engines:
            e.apply(b)
    for e in engines:
        e.steps_done += 1
    torch.cuda.synchronize()
    return deltas


def test_fill_synth_matches_numpy():
    for n, seed, stream in [(1, 42, 0), (4097, 7, 3), (1 << 20, 2001, 291)]:
        x = torch.empty(n, device=DEV)
        add = torch.linspace(-1, 1, n, device=DEV)
        synth.fill_device(x, seed, stream, 0.5, 0.25, add=add)
        ref = synth.values(seed, stream, n, 0.5, 0.25, add=add.cpu().numpy())
        assert x.cpu().numpy().tobytes() == ref.tobytes()


@pytest.mark.parametrize("n", [1, 2])
@pytest.mark.parametrize("per_bucket", [False, True])
def test_micro_matches_reference_bit_exact(n, per_bucket):
    spec = get_tree("micro")
    g = load_npz(f"micro_n{n}.npz")
    engines, inners = _engines(spec, n, cap=4096 if per_bucket else None)
    if per_bucket:
        assert engines[0].tree.n_buckets > 2
    assert np.concatenate(_host(engines[0].unpacked(engines[0].theta))).tobytes() == g["theta0"].tobytes()
    for s in (1, 2):
        deltas = _emulated_step(engines, inners, s, per_bucket)
        assert np.concatenate(deltas[0]).tobytes() == g[f"delta_s{s}_r0"].tobytes()
        assert np.concatenate(deltas[-1]).tobytes() == g[f"delta_s{s}_rlast"].tobytes()
        for e, inner in zip(engines, inners):
            th = np.concatenate(_host(e.unpacked(e.theta)))
            assert th.tobytes() == g[f"theta_s{s}"].tobytes()
            assert np.concatenate(_host(e.unpacked(e.mom))).tobytes() == g[f"buf_s{s}"].tobytes()
            assert np.concatenate(_host(inner)).tobytes() == th.tobytes()  # sync_inner_model


@pytest.mark.parametrize("n", [1, 2])
def test_tiny_matches_reference_digests(n):
    spec = get_tree("tiny")
    ref = load_json("tiny_digests.json")[str(n)]["rank0"]
    engines, inners = _engines(spec, n)
    numels = spec.numels()
    for s in (1, 2):
        deltas = _emulated_step(engines, inners, s)
        e = engines[0]
        got = {f"delta_s{s}": deltas[0], f"theta_s{s}": _host(e.unpacked(e.theta)),
               f"buf_s{s}": _host(e.unpacked(e.mom))}
        for key, tensors in got.items():
            for t, (a, d) in enumerate(zip(tensors, ref[key])):
                assert _sha(a) == d["sha256"], (key, t)


def test_t125_full_size_bit_exact_vs_oracle():
    """BASELINE config #1 tree at full size, two outer steps, against the C oracle."""
    spec = get_tree("t125")
    engines, inners = _engines(spec, 1)
    e = engines[0]
    st = oracle.OuterState(_host(e.unpacked(e.theta)))
    for s in (1, 2):
        _emulated_step(engines, inners, s)
        inner_host = [synth.values(synth.noise_seed(s, 0), t, x.size, 0.0, synth.NOISE_SCALE, add=x)
                      for t, x in enumerate(st.theta)]
        st.step([inner_host])
        got = _host(e.unpacked(e.theta))
        for t in range(len(got)):
            assert got[t].tobytes() == st.theta[t].tobytes(), t
        mom = _host(e.unpacked(e.mom))
        for t in range(len(mom)):
            assert mom[t].tobytes() == st.buf[t].tobytes(), t


RAGGED = [1, 3, 5, 4097, 0, 64, 65, 12345, 8191, 4096 * 3 + 7, 2]


@pytest.mark.parametrize("momentum,nesterov", [(0.9, True), (0.9, False), (0.0, False)])
@pytest.mark.parametrize("misaligned", [False, True])
def test_ragged_tree_and_misaligned_params(momentum, nesterov, misaligned):
    """Tails, empty tensors, 4-B-aligned (not 16-B) parameter storage -> scalar path."""
    g0 = torch.Generator().manual_seed(3)
    host = [torch.randn(n, generator=g0) for n in RAGGED]
    if misaligned:
        base = torch.empty(sum(RAGGED) + len(RAGGED), device=DEV)
        params, o = [], 1
        for h in host:
            params.append(base[o:o + h.numel()])
            o += h.numel() + 1
        for p, h in zip(params, host):
            p.copy_(h)
    else:
        params = [h.to(DEV) for h in host]
    e = OuterSync(params, lr=0.7, momentum=momentum, nesterov=nesterov, world_size=1,
                  bucket_cap_elems=5000)
    st = oracle.OuterState([h.numpy() for h in host], lr=0.7, momentum=momentum, nesterov=nesterov)
    for s in (1, 2, 3):
        noise = [torch.randn(n, generator=g0) * 1e-3 for n in RAGGED]
        inner_host = [(np.asarray(t) + z.numpy()).astype(np.float32) for t, z in zip(st.theta, noise)]
        for p, x in zip(params, inner_host):
            p.copy_(torch.from_numpy(x))
        deltas, _ = st.step([inner_host])
        for b in range(e.tree.n_buckets):
            e.pseudo_gradient(b)
        wire = _host(e.unpacked(e.wire))
        for b in range(e.tree.n_buckets):
            e.apply(b)
        e.steps_done += 1
        torch.cuda.synchronize()
        for t in range(len(RAGGED)):
            assert wire[t].tobytes() == deltas[0][t].tobytes(), (s, t)
            assert _host([params[t]])[0].tobytes() == st.theta[t].tobytes(), (s, t)
        # padding of every packed buffer stays zero
        mask = torch.ones(e.tree.total, dtype=torch.bool, device=DEV)
        for t, n in enumerate(RAGGED):
            lo = int(e.tree.seg_off[t])
            mask[lo:lo + n] = False
        assert not e.theta[mask].any() and not e.wire[mask].any()


def test_bf16_wire_rounds_like_torch():
    spec = get_tree("micro")
    engines, inners = _engines(spec, 1, wire=torch.bfloat16)
    f32, f32_inners = _engines(spec, 1)
    for s in (1, 2):
        e = engines[0]
        d_bf = _emulated_step(engines, inners, s)[0]
        d_32 = _emulated_step(f32, f32_inners, s)[0]
        for a, b in zip(d_bf, d_32):
            ref = torch.from_numpy(b).to(torch.bfloat16).float().numpy() if s == 1 else None
            if ref is not None:
                assert a.tobytes() == ref.tobytes()
    # bf16 wire error vs the fp32 path is bounded by bf16 resolution of the deltas
    th_bf = np.concatenate(_host(engines[0].unpacked(engines[0].theta)))
    th_32 = np.concatenate(_host(f32[0].unpacked(f32[0].theta)))
    assert np.abs(th_bf - th_32).max() <= 0.7 * 2 * 1e-3 * 2 ** -7 * 3


def test_unpack_avg_gather_scatter_roundtrip():
    numels = RAGGED
    g0 = torch.Generator().manual_seed(11)
    grads = [torch.randn(n, generator=g0).to(DEV) for n in numels]
    dst = [torch.empty(n, device=DEV) for n in numels]
    tree = PackedTree(numels, 6000)
    s = torch.cuda.current_stream().cuda_stream
    tree.bind(SLOT_GRAD, grads, s)
    tree.bind(SLOT_INNER, dst, s)
    packed = torch.zeros(tree.total, device=DEV)
    for b in range(tree.n_buckets):
        _lib.call("dl_gather", tree.handle, b, SLOT_GRAD, packed.data_ptr(), _lib.DL_F32, s)
    for div in (1, 3, 8):
        for b in range(tree.n_buckets):
            _lib.call("dl_unpack_avg", tree.handle, b, packed.data_ptr(), _lib.DL_F32, div,
                      SLOT_INNER, None, s)
        torch.cuda.synchronize()
        for g, d in zip(grads, dst):
            ref = g.cpu() if div == 1 else g.cpu() / div
            assert d.cpu().numpy().tobytes() == ref.numpy().tobytes()
    # packed -> packed average in place, then scatter back
    _lib.call("dl_unpack_avg", tree.handle, _lib.ALL_BUCKETS, packed.data_ptr(), _lib.DL_F32, 2,
              -1, packed.data_ptr(), s)
    _lib.call("dl_scatter", tree.handle, _lib.ALL_BUCKETS, packed.data_ptr(), SLOT_INNER, s)
    torch.cuda.synchronize()
    for g, d in zip(grads, dst):
        assert d.cpu().numpy().tobytes() == (g.cpu() / 2).numpy().tobytes()
    tree.close()


def test_kernel_argument_errors_are_raised():
    tree = PackedTree([10, 20])
    s = torch.cuda.current_stream().cuda_stream
    buf = torch.zeros(tree.total, device=DEV)
    with pytest.raises(_lib.DilocoHipError, match="not bound"):
        _lib.call("dl_delta_pack", tree.handle, -1, SLOT_INNER, buf.data_ptr(), buf.data_ptr(),
                  _lib.DL_F32, s)
    with pytest.raises(_lib.DilocoHipError, match="bucket"):
        _lib.call("dl_scatter", tree.handle, 5, buf.data_ptr(), SLOT_INNER, s)
    params = [torch.zeros(10, device=DEV), torch.zeros(20, device=DEV)]
    tree.bind(SLOT_INNER, params, s)
    with pytest.raises(_lib.DilocoHipError, match="aligned"):
        _lib.call("dl_gather", tree.handle, -1, SLOT_INNER, buf.data_ptr() + 4, _lib.DL_F32, s)
    with pytest.raises(_lib.DilocoHipError, match="divisor"):
        _lib.call("dl_unpack_avg", tree.handle, -1, buf.data_ptr(), _lib.DL_F32, 0, SLOT_INNER,
                  None, s)
    tree.close()


@pytest.mark.parametrize("tree", ["micro", "tiny"])
def test_fused_single_peer_step_matches_reference(tree):
    """dl_delta_sgd (one replica: delta + SGD + copy-back in one pass) vs the reference."""
    spec = get_tree(tree)
    theta0 = synth.outer_tree_device(spec, DEV)
    shapes = [s for _, s in spec.params()]
    params = [t.clone().view(s) for t, s in zip(theta0, shapes)]
    e = OuterSync(params, world_size=1, fuse_single=True)
    for s in (1, 2):
        th = [t.reshape(-1) for t in e.unpacked(e.theta)]
        synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in params])
        e.step()
        torch.cuda.synchronize()
        got_t = _host(e.unpacked(e.theta))
        got_m = _host(e.unpacked(e.mom))
        assert np.concatenate(_host(params)).tobytes() == np.concatenate(got_t).tobytes()
        if tree == "micro":
            g = load_npz("micro_n1.npz")
            assert np.concatenate(got_t).tobytes() == g[f"theta_s{s}"].tobytes()
            assert np.concatenate(got_m).tobytes() == g[f"buf_s{s}"].tobytes()
        else:
            ref = load_json("tiny_digests.json")["1"]["rank0"]
            for t, (a, d) in enumerate(zip(got_t, ref[f"theta_s{s}"])):
                assert _sha(a) == d["sha256"], t


@pytest.mark.parametrize("momentum,nesterov", [(0.9, True), (0.9, False), (0.0, False)])
def test_fused_single_peer_ragged_vs_two_kernel_path(momentum, nesterov):
    g0 = torch.Generator().manual_seed(5)
    host = [torch.randn(n, generator=g0) for n in RAGGED]
    pa = [h.to(DEV) for h in host]
    pb = [h.to(DEV) for h in host]
    ea = OuterSync(pa, momentum=momentum, nesterov=nesterov, world_size=1, fuse_single=True)
    eb = OuterSync(pb, momentum=momentum, nesterov=nesterov, world_size=1, fuse_single=False)
    for _ in range(3):
        noise = [torch.randn(n, generator=g0).to(DEV) * 1e-3 for n in RAGGED]
        for p, q, z in zip(pa, pb, noise):
            p.add_(z)
            q.add_(z)
        ea.step()
        eb.step()
        torch.cuda.synchronize()
        for p, q in zip(pa, pb):
            assert p.cpu().numpy().tobytes() == q.cpu().numpy().tobytes()
        assert ea.theta.cpu().numpy().tobytes() == eb.theta.cpu().numpy().tobytes()


@pytest.mark.parametrize("wire", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("momentum,nesterov", [(0.9, True), (0.9, False), (0.0, False)])
@pytest.mark.parametrize("misaligned", [False, True])
def test_delta_pack_sgd_equals_two_kernel_pair(wire, momentum, nesterov, misaligned):
    """dl_delta_pack_sgd (one pass, the pseudo-gradient kept in the wire) is bit-identical to
    dl_delta_pack -> dl_unpack_sgd: θ, momentum, inner AND the wire, ragged tensors (tails,
    empty), 4-B-aligned storage (scalar path), fp32 and bf16 wires, every SGD mode."""
    g0 = torch.Generator().manual_seed(23)
    host = [torch.randn(n, generator=g0) for n in RAGGED]

    def place():
        if not misaligned:
            return [h.to(DEV) for h in host]
        base = torch.empty(sum(RAGGED) + len(RAGGED), device=DEV)
        out, o = [], 1
        for h in host:
            out.append(base[o:o + h.numel()])
            out[-1].copy_(h)
            o += h.numel() + 1
        return out

    pa, pb = place(), place()
    ea = OuterSync(pa, momentum=momentum, nesterov=nesterov, world_size=1, wire_dtype=wire,
                   fuse_single=True, keep_wire=True)
    eb = OuterSync(pb, momentum=momentum, nesterov=nesterov, world_size=1, wire_dtype=wire,
                   fuse_single=False, tile_chunks=0)
    iview = torch.int16 if wire == torch.bfloat16 else torch.int32
    for _ in range(3):
        noise = [torch.randn(n, generator=g0).to(DEV) * 1e-3 for n in RAGGED]
        for p, q, z in zip(pa, pb, noise):
            p.add_(z)
            q.add_(z)
        ea.step()
        eb.step()
        torch.cuda.synchronize()
        assert torch.equal(ea.theta.view(torch.int32), eb.theta.view(torch.int32))
        assert torch.equal(ea.wire.view(iview), eb.wire.view(iview))
        if momentum:
            assert torch.equal(ea.mom.view(torch.int32), eb.mom.view(torch.int32))
        for p, q in zip(pa, pb):
            assert p.cpu().numpy().tobytes() == q.cpu().numpy().tobytes()


@pytest.mark.parametrize("kernel", ["delta_pack_sgd", "delta_pack_sgd_bf16", "delta_sgd",
                                    "two_kernel", "two_kernel_bf16"])
@pytest.mark.parametrize("misaligned", [False, True])
def test_store_policies_are_bit_identical(kernel, misaligned):
    """dl_tree_tune's store policies in the product library (plain and non-temporal stores
    after non-temporal loads) change only the timing: θ, momentum, the wire (fp32 and bf16)
    and the inner params equal the AUTO policy's bit for bit, ragged tails and the 4-B-aligned
    scalar path included. The tuning-only policies (plain loads, write-through for every
    kernel: make TUNING=1) are refused by the product library."""
    sizes = RAGGED + [300 * 4096 + 77]
    g0 = torch.Generator().manual_seed(37)
    host = [torch.randn(n, generator=g0) for n in sizes]

    def place():
        if not misaligned:
            return [h.to(DEV) for h in host]
        base = torch.empty(sum(sizes) + len(sizes), device=DEV)
        out, o = [], 1
        for h in host:
            out.append(base[o:o + h.numel()])
            out[-1].copy_(h)
            o += h.numel() + 1
        return out

    wire = torch.bfloat16 if kernel.endswith("bf16") else torch.float32
    kw = {"delta_pack_sgd": dict(fuse_single=True, keep_wire=True, wire_dtype=wire),
          "delta_sgd": dict(fuse_single=True),
          "two_kernel": dict(fuse_single=False, tile_chunks=0, wire_dtype=wire)}[
              kernel.replace("_bf16", "")]
    NTL, NTS, WT = _lib.TUNE_NT_LOADS, _lib.TUNE_NT_STORES, _lib.TUNE_WT_STORES
    PR = _lib.TUNE_PAIRS  # dl_delta_pack's two chunks per workgroup (odd counts, ragged)
    policies = [NTL, NTL | NTS]
    if _lib.load().dl_tuning_build():
        policies += [NTL | WT, NTL | NTS | WT, WT, 0, NTS, NTL | PR, NTL | NTS | PR]
    ref_p = place()
    ref = OuterSync(ref_p, world_size=1, **kw)
    if not _lib.load().dl_tuning_build():
        for f in (NTL | WT, WT, 0, NTS, NTL | PR):
            with pytest.raises(_lib.DilocoHipError, match="TUNING"):
                ref.tree.tune(0, f)
    runs = []
    for f in policies:
        p = place()
        e = OuterSync(p, world_size=1, **kw)
        e.tree.tune(0, f)
        runs.append((e, p))
    for _ in range(2):
        noise = [torch.randn(n, generator=g0).to(DEV) * 1e-3 for n in sizes]
        for ps in [ref_p] + [p for _, p in runs]:
            for t, z in zip(ps, noise):
                t.add_(z)
        ref.step()
        for e, _ in runs:
            e.step()
        torch.cuda.synchronize()
        for e, p in runs:
            assert torch.equal(e.theta.view(torch.int32), ref.theta.view(torch.int32))
            assert torch.equal(e.mom.view(torch.int32), ref.mom.view(torch.int32))
            if ref.wire is not None and kernel != "delta_sgd":
                assert torch.equal(e.wire.view(torch.uint8), ref.wire.view(torch.uint8))
            for a, b in zip(p, ref_p):
                assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    for e, _ in runs:
        e.close()
    ref.close()


def test_delta_pack_sgd_micro_matches_reference():
    """The one-pass step with the wire kept reproduces the reference's outer steps AND its
    outer.grad (the wire holds delta_s{s}_r0 after step s), micro tree, n = 1."""
    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    params = [t.clone().view(s) for t, s in zip(synth.outer_tree_device(spec, DEV), shapes)]
    e = OuterSync(params, world_size=1, fuse_single=True, keep_wire=True)
    g = load_npz("micro_n1.npz")
    for s in (1, 2):
        th = [t.reshape(-1) for t in e.unpacked(e.theta)]
        synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in params])
        e.step()
        torch.cuda.synchronize()
        assert np.concatenate(_host(e.unpacked(e.wire))).tobytes() == g[f"delta_s{s}_r0"].tobytes()
        assert np.concatenate(_host(e.unpacked(e.theta))).tobytes() == g[f"theta_s{s}"].tobytes()
        assert np.concatenate(_host(e.unpacked(e.mom))).tobytes() == g[f"buf_s{s}"].tobytes()
        assert np.concatenate(_host(params)).tobytes() == g[f"theta_s{s}"].tobytes()
    e.close()


@pytest.mark.parametrize("wire", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("momentum,nesterov", [(0.9, True), (0.9, False), (0.0, False)])
def test_tiled_pack_sgd_equals_whole_range_launches(wire, momentum, nesterov):
    """dl_pack_sgd_tiled (Infinity-Cache-blocked delta_pack -> unpack_sgd) is bit-identical to
    the two whole-range launches for tiles of 1, 3 and 7 chunks (tiles cut tensors and end
    inside ragged tails) and leaves the same wire."""
    g0 = torch.Generator().manual_seed(11)
    host = [torch.randn(n, generator=g0) for n in RAGGED]
    ps = {t: [h.to(DEV) for h in host] for t in (0, 1, 3, 7)}
    es = {t: OuterSync(p, momentum=momentum, nesterov=nesterov, world_size=1, wire_dtype=wire,
                       fuse_single=False, tile_chunks=t) for t, p in ps.items()}
    for _ in range(3):
        noise = [torch.randn(n, generator=g0).to(DEV) * 1e-3 for n in RAGGED]
        for t in es:
            for p, z in zip(ps[t], noise):
                p.add_(z)
            es[t].step()
        torch.cuda.synchronize()
        ref = es[0]
        for t in (1, 3, 7):
            assert es[t].theta.cpu().numpy().tobytes() == ref.theta.cpu().numpy().tobytes(), t
            assert es[t].wire.cpu().view(torch.int16 if wire == torch.bfloat16 else
                                         torch.int32).numpy().tobytes() == \
                ref.wire.cpu().view(torch.int16 if wire == torch.bfloat16 else
                                    torch.int32).numpy().tobytes(), t
            if momentum:
                assert es[t].mom.cpu().numpy().tobytes() == ref.mom.cpu().numpy().tobytes()
            for p, q in zip(ps[t], ps[0]):
                assert p.cpu().numpy().tobytes() == q.cpu().numpy().tobytes(), t


def test_tiled_pack_sgd_micro_matches_reference():
    """The tiled one-replica pipeline reproduces the reference's micro-tree outer steps."""
    spec = get_tree("micro")
    theta0 = synth.outer_tree_device(spec, DEV)
    shapes = [s for _, s in spec.params()]
    params = [t.clone().view(s) for t, s in zip(theta0, shapes)]
    e = OuterSync(params, world_size=1, fuse_single=False, tile_chunks=2)
    g = load_npz("micro_n1.npz")
    for s in (1, 2):
        th = [t.reshape(-1) for t in e.unpacked(e.theta)]
        synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in params])
        e.step()
        torch.cuda.synchronize()
        assert np.concatenate(_host(e.unpacked(e.theta))).tobytes() == g[f"theta_s{s}"].tobytes()
        assert np.concatenate(_host(e.unpacked(e.mom))).tobytes() == g[f"buf_s{s}"].tobytes()
        assert np.concatenate(_host(params)).tobytes() == g[f"theta_s{s}"].tobytes()


def test_direct_exchange_from_inner_arena_single_replica():
    """exchange='xgmi_inner' at one replica: the inner parameters move into the engine's packed
    arena (values unchanged), the outer steps equal the reference's (micro tree, n = 1), and a
    parameter whose storage is replaced afterwards is refused."""
    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    params = [t.clone().view(s) for t, s in zip(synth.outer_tree_device(spec, DEV), shapes)]
    before = [p.clone() for p in params]
    e = OuterSync(params, world_size=1, exchange="xgmi_inner")
    base = e.inner_arena.data_ptr()
    assert all(base <= p.data_ptr() < base + 4 * e.tree.total for p in params)
    assert all(torch.equal(p, b) for p, b in zip(params, before))
    g = load_npz("micro_n1.npz")
    for s in (1, 2):
        th = [t.reshape(-1) for t in e.unpacked(e.theta)]
        synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in params])
        e.step()
        torch.cuda.synchronize()
        assert np.concatenate(_host(e.unpacked(e.theta))).tobytes() == g[f"theta_s{s}"].tobytes()
        assert np.concatenate(_host(e.unpacked(e.momentum_full()))).tobytes() == \
            g[f"buf_s{s}"].tobytes()
        assert np.concatenate(_host(params)).tobytes() == g[f"theta_s{s}"].tobytes()
    params[3].data = params[3].data.clone()
    with pytest.raises(RuntimeError, match="storage was replaced"):
        e.step()
    e.close()


def test_t13b_full_size_sampled_tensors_vs_oracle_and_fused():
    """BASELINE configs #4/#5 tree at full size (1.31 B params): the two-kernel path equals the
    one-pass kernel everywhere (size-independent property), and the largest (wte, 103 M),
    first-block and last tensors equal the C oracle bit for bit."""
    spec = get_tree("t1.3b")
    shapes = [s for _, s in spec.params()]
    pa = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, DEV), shapes)]
    pb = [t.clone() for t in pa]
    pc = [t.clone() for t in pa]
    ea = OuterSync(pa, world_size=1, fuse_single=False)
    eb = OuterSync(pb, world_size=1, fuse_single=True)
    ec = OuterSync(pc, world_size=1, fuse_single=True, keep_wire=True)
    for e, ps in ((ea, pa), (eb, pb), (ec, pc)):
        th = [t.reshape(-1) for t in e.unpacked(e.theta)]
        synth.inner_tree_device(th, 1, 0, out=[p.view(-1) for p in ps])
        e.step()
    torch.cuda.synchronize()
    assert torch.equal(ea.theta, eb.theta) and torch.equal(ea.mom, eb.mom)
    assert torch.equal(ea.theta, ec.theta) and torch.equal(ea.mom, ec.mom)
    assert torch.equal(ea.wire, ec.wire)  # the kept pseudo-gradient == dl_delta_pack's
    assert all(torch.equal(x, y) for x, y in zip(pa, pb))
    assert all(torch.equal(x, y) for x, y in zip(pa, pc))
    ec.close()
    del ec, pc
    numels, init = spec.numels(), spec.init_spec()
    for t in (0, 2, 4, len(numels) - 1):
        th0 = synth.values(synth.OUTER_SEED, t, numels[t], *init[t])
        inner = synth.values(synth.noise_seed(1, 0), t, numels[t], 0.0, synth.NOISE_SCALE, add=th0)
        st = oracle.OuterState([th0])
        st.step([[inner]])
        got = ea.unpacked(ea.theta)[t].reshape(-1).cpu().numpy()
        assert got.tobytes() == st.theta[0].tobytes(), t
    ea.close()
    eb.close()


# ---- int8 wire codec -----------------------------------------------------
def _q8_emulated_step(engines, inners, step):
    """n int8-wire replicas on one GPU: all_to_all / all_gather emulated with copies, the
    reduce is the product kernel (dl_q8_reduce)."""
    from diloco_amd.kernels import Q8_SLOT

    n = len(engines)
    for r, (e, inner) in enumerate(zip(engines, inners)):
        th = [t.reshape(-1) for t in e.unpacked(e.theta)]
        synth.inner_tree_device(th, step, r, out=[p.view(-1) for p in inner])
    for b in range(engines[0].tree.n_buckets):
        for e in engines:
            e.pseudo_gradient(b)
        _nch, m, _ = engines[0].q8_plan[b]
        regions = [e.q8_region(b) for e in engines]
        outs = []
        for p, e in enumerate(engines):  # peer p reduces slots [p*m, (p+1)*m) of every replica
            recv = torch.cat([reg[p * m * Q8_SLOT:(p + 1) * m * Q8_SLOT] for reg in regions])
            out = torch.zeros(m * Q8_SLOT, dtype=torch.uint8, device=DEV)
            e.k.q8_reduce(recv, n, m, n, out)
            outs.append(out)
        gathered = torch.cat(outs)
        for reg in regions:
            reg.copy_(gathered)
        for e in engines:
            e.apply(b)
    for e in engines:
        e.steps_done += 1
    torch.cuda.synchronize()


@pytest.mark.parametrize("n", [1, 2, 4])
def test_int8_wire_matches_oracle_restatement(n):
    from expect import MICRO_Q8_CAP, expected_q8

    exp = expected_q8(n)
    spec = get_tree("micro")
    theta0 = synth.outer_tree_device(spec, DEV)
    shapes = [s for _, s in spec.params()]
    engines, inners = [], []
    for _ in range(n):
        inner = [t.clone().view(s) for t, s in zip(theta0, shapes)]
        engines.append(OuterSync(inner, world_size=n, wire_dtype=torch.int8,
                                 bucket_cap_elems=MICRO_Q8_CAP))
        inners.append(inner)
    for s in (1, 2):
        if n == 1:  # the engine's own single-replica path
            e = engines[0]
            th = [t.reshape(-1) for t in e.unpacked(e.theta)]
            synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in inners[0]])
            e.step()
            torch.cuda.synchronize()
        else:
            _q8_emulated_step(engines, inners, s)
        for e, inner in zip(engines, inners):
            th = np.concatenate(_host(e.unpacked(e.theta)))
            assert th.tobytes() == exp[f"theta_s{s}"].tobytes(), (n, s)
            assert np.concatenate(_host(inner)).tobytes() == th.tobytes()


def test_int8_wire_t125_error_and_ragged_tails():
    """Full T125 tree (tails, 148 tensors): one step through the int8 wire vs the exact fp32
    step -- deltas quantised twice, each |err| <= s/2 with s = amax/127 per 4096-chunk."""
    spec = get_tree("t125")
    shapes = [s for _, s in spec.params()]
    pa = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, DEV), shapes)]
    pb = [t.clone() for t in pa]
    ea = OuterSync(pa, world_size=1, wire_dtype=torch.int8)
    eb = OuterSync(pb, world_size=1)
    for e, ps in ((ea, pa), (eb, pb)):
        th = [t.reshape(-1) for t in e.unpacked(e.theta)]
        synth.inner_tree_device(th, 1, 0, out=[p.view(-1) for p in ps])
        e.step()
    torch.cuda.synchronize()
    # θ_1 = θ_0 - lr*(1+m)*g: compare the applied updates
    th0 = synth.outer_tree_device(spec, DEV)
    worst = 0.0
    for a, b, t0 in zip(ea.unpacked(ea.theta), eb.unpacked(eb.theta), th0):
        ua, ub = (t0.view(-1) - a.reshape(-1)), (t0.view(-1) - b.reshape(-1))
        worst = max(worst, float((ua - ub).abs().max() / ub.abs().max().clamp_min(1e-30)))
    assert worst < 1.6e-2, worst
    ea.close()
    eb.close()


@pytest.mark.parametrize("wire", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("divisor", [1, 2, 3, 8])
@pytest.mark.parametrize("momentum,nesterov", [(0.9, True), (0.9, False), (0.0, False)])
def test_shard_sgd_matches_oracle(wire, divisor, momentum, nesterov):
    """dl_shard_sgd (the sharded step's a3 /n + a4 on a flat shard) == the oracle's division and
    SGD, bit-exact, first and steady-state steps, lengths with partial chunks and < 4 tails."""
    from diloco_amd.kernels import default_kernels

    k = default_kernels()
    for n in (1, 3, 64, 4096 + 5, 3 * 4096 + 64 * 7 + 2):
        g = torch.from_numpy(synth.values(5, n, n, 0.0, 1e-3))
        if wire == torch.bfloat16:
            g = g.to(torch.bfloat16).float()
        th = synth.values(6, n, n, 0.0, 0.02)
        buf = synth.values(7, n, n, 0.0, 1e-3)
        dg, dth = g.to(DEV).to(wire), torch.from_numpy(th.copy()).to(DEV)
        dm = torch.from_numpy(buf.copy()).to(DEV) if momentum else None
        rth, rbuf = th.copy(), buf.copy()
        for first in (True, False):
            k.shard_sgd(dg, divisor, dth, dm, 0.7, momentum, nesterov, first)
            gg = g.numpy().copy()
            if divisor != 1:
                gg = (gg / np.float32(divisor)).astype(np.float32)
            oracle.sgd(rth, rbuf if momentum else None, gg, 0.7, momentum, nesterov, first)
        torch.cuda.synchronize()
        assert dth.cpu().numpy().tobytes() == rth.tobytes(), n
        if momentum:
            assert dm.cpu().numpy().tobytes() == rbuf.tobytes(), n


def test_sharded_engine_single_rank_layout():
    """The sharded engine's tree: buckets start at multiples of 64·n elements and split into n
    equal shards; θ_outer starts as the inner params (a1)."""
    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, DEV), shapes)]
    e = OuterSync(params, world_size=4, bucket_cap_elems=4096, shard=True)
    for lo, hi in e.tree.bucket_ranges:
        assert lo % 256 == 0 and (hi - lo) % 256 == 0
    assert e.shard_total * 4 == e.tree.total
    assert np.concatenate(_host(e.unpacked(e.theta))).tobytes() == \
        np.concatenate(_host(params)).tobytes()
    e.close()


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_sharded_step_emulated_matches_reference(n):
    """The sharded variant of n replicas on one GPU, collectives emulated (reduce-scatter = sum
    of the replicas' wire buckets, peer r keeps slice r; all-gather = concatenation of the θ
    shards): θ, momentum and inner bit-exact vs the reference at n <= 2, normwise at n = 4, 8."""
    from conftest import normwise_ok

    spec = get_tree("micro")
    g = load_npz(f"micro_n{n}.npz")
    theta0 = synth.outer_tree_device(spec, DEV)
    shapes = [s for _, s in spec.params()]
    engines, inners = [], []
    for r in range(n):
        inner = [t.clone().view(s) for t, s in zip(theta0, shapes)]
        engines.append(OuterSync(inner, world_size=n, bucket_cap_elems=4096, shard=True, rank=r))
        inners.append(inner)
    e0 = engines[0]
    assert e0.tree.n_buckets > 2
    for s in (1, 2):
        for r, (e, inner) in enumerate(zip(engines, inners)):
            th = [t.reshape(-1) for t in e.unpacked(e.theta)]
            synth.inner_tree_device(th, s, r, out=[p.view(-1) for p in inner])
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
            gathered = torch.cat([e.th_shard_view(b) for e in engines])
            lo, hi = e0.tree.bucket_ranges[b]
            for e in engines:
                e.theta[lo:hi].copy_(gathered)
                e.write_inner(b)
        for e in engines:
            e.steps_done += 1
        torch.cuda.synchronize()
        mom = [torch.cat([e.mom_shard[e.shard_off[b]:e.shard_off[b] + e0._shard_len(b)]
                          for e in engines]) for b in range(e0.tree.n_buckets)]
        mom_full = torch.zeros_like(e0.theta)
        for b, m in enumerate(mom):
            lo, hi = e0.tree.bucket_ranges[b]
            mom_full[lo:hi] = m
        th = np.concatenate(_host(e0.unpacked(e0.theta)))
        buf = np.concatenate(_host(e0.unpacked(mom_full)))
        for e, inner in zip(engines, inners):
            assert np.concatenate(_host(e.unpacked(e.theta))).tobytes() == th.tobytes()
            assert np.concatenate(_host(inner)).tobytes() == th.tobytes()
        if n <= 2:
            assert th.tobytes() == g[f"theta_s{s}"].tobytes(), s
            assert buf.tobytes() == g[f"buf_s{s}"].tobytes(), s
        else:
            numels = spec.numels()
            for a, b in zip(split(th, numels), split(g[f"theta_s{s}"], numels)):
                assert normwise_ok(a, b, 1e-6)
            for a, b in zip(split(buf, numels), split(g[f"buf_s{s}"], numels)):
                assert normwise_ok(a, b, 1e-6)


def test_sharded_single_replica_without_process_group():
    """shard=True, one replica, no process group: the collectives are local copies and the step
    equals the reference's single-peer step bit-exact (momentum via momentum_full())."""
    spec = get_tree("micro")
    g = load_npz("micro_n1.npz")
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, DEV), shapes)]
    e = OuterSync(params, world_size=1, bucket_cap_elems=4096, shard=True)
    for s in (1, 2):
        th = [t.reshape(-1) for t in e.unpacked(e.theta)]
        synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in params])
        e.step()
        torch.cuda.synchronize()
        assert np.concatenate(_host(e.unpacked(e.theta))).tobytes() == g[f"theta_s{s}"].tobytes()
        assert np.concatenate(_host(e.unpacked(e.momentum_full()))).tobytes() == \
            g[f"buf_s{s}"].tobytes()
        assert np.concatenate(_host(params)).tobytes() == g[f"theta_s{s}"].tobytes()
    e.close()


def test_sharded_bf16_wire_equals_replicated_bf16_wire():
    """bf16 wire, n = 2 emulated on one GPU: reduce-scatter (sum of two bf16 values, rounded to
    bf16 as RCCL does) -> dl_shard_sgd equals all-reduce -> dl_unpack_sgd bit-exact."""
    spec = get_tree("micro")
    n = 2
    rep, rep_in = _engines(spec, n, wire=torch.bfloat16, cap=4096)
    theta0 = synth.outer_tree_device(spec, DEV)
    shapes = [s for _, s in spec.params()]
    sh, sh_in = [], []
    for r in range(n):
        inner = [t.clone().view(s) for t, s in zip(theta0, shapes)]
        sh.append(OuterSync(inner, world_size=n, wire_dtype=torch.bfloat16, bucket_cap_elems=4096,
                            shard=True, rank=r))
        sh_in.append(inner)
    for s in (1, 2):
        _emulated_step(rep, rep_in, s, per_bucket=True)
        for r, (e, inner) in enumerate(zip(sh, sh_in)):
            th = [t.reshape(-1) for t in e.unpacked(e.theta)]
            synth.inner_tree_device(th, s, r, out=[p.view(-1) for p in inner])
        e0 = sh[0]
        for b in range(e0.tree.n_buckets):
            for e in sh:
                e.pseudo_gradient(b)
            total = sh[0].bucket_view(b) + sh[1].bucket_view(b)  # bf16 + bf16 -> bf16
            sl = e0._shard_len(b)
            for r, e in enumerate(sh):
                e._shard(e.g_shard, b).copy_(total[r * sl:(r + 1) * sl])
                e.shard_apply(b)
            gathered = torch.cat([e.th_shard_view(b) for e in sh])
            lo, hi = e0.tree.bucket_ranges[b]
            for e in sh:
                e.theta[lo:hi].copy_(gathered)
                e.write_inner(b)
        for e in sh:
            e.steps_done += 1
        torch.cuda.synchronize()
        want = np.concatenate(_host(rep[0].unpacked(rep[0].theta)))
        for e, inner in zip(sh, sh_in):
            assert np.concatenate(_host(e.unpacked(e.theta))).tobytes() == want.tobytes(), s
            assert np.concatenate(_host(inner)).tobytes() == want.tobytes(), s


def test_sharded_t125_full_size_equals_replicated():
    """Full T125 tree (148 tensors, 2 buckets), n = 2 emulated on one GPU, 2 outer steps: the
    sharded step (bucket-aligned layout, shard SGD, all-gather, scatter) equals the replicated
    step bit-exact for θ, momentum and the inner parameters."""
    spec = get_tree("t125")
    n = 2
    rep, rep_in = _engines(spec, n, cap=64 << 20)
    theta0 = synth.outer_tree_device(spec, DEV)
    shapes = [s for _, s in spec.params()]
    sh, sh_in = [], []
    for r in range(n):
        inner = [t.clone().view(s) for t, s in zip(theta0, shapes)]
        sh.append(OuterSync(inner, world_size=n, shard=True, rank=r))
        sh_in.append(inner)
    del theta0
    e0 = sh[0]
    for s in (1, 2):
        _emulated_step(rep, rep_in, s, per_bucket=True)
        for r, (e, inner) in enumerate(zip(sh, sh_in)):
            th = [t.reshape(-1) for t in e.unpacked(e.theta)]
            synth.inner_tree_device(th, s, r, out=[p.view(-1) for p in inner])
        for b in range(e0.tree.n_buckets):
            for e in sh:
                e.pseudo_gradient(b)
            total = sh[0].bucket_view(b) + sh[1].bucket_view(b)
            sl = e0._shard_len(b)
            for r, e in enumerate(sh):
                e._shard(e.g_shard, b).copy_(total[r * sl:(r + 1) * sl])
                e.shard_apply(b)
            gathered = torch.cat([e.th_shard_view(b) for e in sh])
            lo, hi = e0.tree.bucket_ranges[b]
            for e in sh:
                e.theta[lo:hi].copy_(gathered)
                e.write_inner(b)
            del total, gathered
        for e in sh:
            e.steps_done += 1
        torch.cuda.synchronize()
        for a, b in zip(rep[0].unpacked(rep[0].theta), e0.unpacked(e0.theta)):
            assert torch.equal(a, b), s
        mom = torch.zeros_like(e0.theta)
        for b in range(e0.tree.n_buckets):
            lo, hi = e0.tree.bucket_ranges[b]
            mom[lo:hi] = torch.cat([e._shard(e.mom_shard, b) for e in sh])
        for a, b in zip(rep[0].unpacked(rep[0].mom), e0.unpacked(mom)):
            assert torch.equal(a, b), s
        for x, y in zip(rep_in[1], sh_in[1]):
            assert torch.equal(x, y), s
    for e in rep + sh:
        e.close()


def test_tensor_larger_than_int32_elements():
    """A tensor of 2^31 + 5 elements (8.6 GB; 64-bit offsets in the planner, chunk table and
    kernels) between two small ones: one outer step through the two-kernel path and the fused
    path agree bit-exact, and elements around the 2^31 boundary and at the end equal the
    oracle's step computed on the host."""
    big = (1 << 31) + 5
    numels = [3, big, 7]
    n_total = sum(numels)
    free, _ = torch.cuda.mem_get_info()
    if free < 12 * 4 * n_total:
        pytest.skip("needs ~100 GB of free HBM")
    params = [torch.empty(n, device=DEV) for n in numels]
    for i, p in enumerate(params):
        synth.fill_device(p, 42, i, 0.0, 0.02)
    pb = [p.clone() for p in params]
    ea = OuterSync(params, world_size=1, fuse_single=False)
    eb = OuterSync(pb, world_size=1, fuse_single=True)
    assert ea.tree.seg_off[-1] > (1 << 31)
    for e, ps in ((ea, params), (eb, pb)):
        for i, p in enumerate(ps):  # inner = θ_0 + noise
            synth.fill_device(p, 7, i, 0.0, 1e-3, add=e.unpacked(e.theta)[i])
        e.step()
    torch.cuda.synchronize()
    for x, y in zip(params, pb):
        assert torch.equal(x, y)
    del pb, eb
    # host check of slices of the big tensor (SGD first step: θ1 = θ0 - lr*(1+m)*(θ0 - inner))
    for lo, n in ((0, 16), ((1 << 31) - 8, 13), (big - 9, 9)):  # 13: up to the last element
        th0 = np.float32(0.0) + synth.uniform(42, 1, n, start=lo) * np.float32(0.02)
        inner = (np.float32(0.0) + synth.uniform(7, 1, n, start=lo) * np.float32(1e-3)) + th0
        st = oracle.OuterState([th0])
        st.step([[inner]])
        got = params[1][lo:lo + n].cpu().numpy()
        assert got.size == n and got.tobytes() == st.theta[0].tobytes(), lo
    ea.close()


def test_peer_gather_copies_every_source():
    """dl_peer_gather (the xGMI link probe's kernel) with local sources: dst holds each source's
    bytes in order, ragged lengths included."""
    import ctypes

    for nsrc, each in ((1, 16), (3, 4096 * 4 + 48), (8, 1 << 20)):
        srcs = [torch.arange(each // 4, dtype=torch.float32, device=DEV) + 1000 * i
                for i in range(nsrc)]
        dst = torch.full((nsrc * each // 4,), -1.0, device=DEV)
        arr = np.asarray([t.data_ptr() for t in srcs], dtype=np.uint64)
        _lib.call("dl_peer_gather", arr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), nsrc,
                  each, dst.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(dst, torch.cat(srcs)), (nsrc, each)


def test_slot_rebound_on_another_stream_waits_for_the_first_streams_work():
    """A slot bound and used on stream A, then rebound to other tensors and used on stream B
    with no ordering by the caller: B's bind waits for A's kernel (the per-slot event), so
    A's kernel reads the first binding and B's the second (dl_tree_bind)."""
    from diloco_amd.kernels import HipKernels

    k = HipKernels()
    sizes = [4096 * 2048 + 5, 777, 4096 * 1024]  # ~12.6 M elements: A's kernel runs a while
    tree = k.tree(sizes, torch.device(DEV))
    g = torch.Generator().manual_seed(7)
    theta = torch.randn(tree.total, generator=g).to(DEV)
    xs = [torch.randn(n, generator=g).to(DEV) for n in sizes]
    ys = [torch.randn(n, generator=g).to(DEV) for n in sizes]
    wa = torch.empty(tree.total, device=DEV)
    wb = torch.empty(tree.total, device=DEV)
    sa, sb = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    torch.cuda.synchronize()
    for _ in range(3):
        with torch.cuda.stream(sa):
            tree.bind(SLOT_INNER, xs, sa.cuda_stream)
            for _ in range(4):  # keep stream A busy reading the first binding
                k.delta_pack(tree, _lib.ALL_BUCKETS, SLOT_INNER, theta, wa)
        tree._bound[SLOT_INNER] = None  # force the rebind through the C-ABI
        with torch.cuda.stream(sb):
            tree.bind(SLOT_INNER, ys, sb.cuda_stream)
            k.delta_pack(tree, _lib.ALL_BUCKETS, SLOT_INNER, theta, wb)
        torch.cuda.synchronize()
        tree._bound[SLOT_INNER] = None
        for t, (o, n) in enumerate(zip(tree.seg_off[:-1], sizes)):
            th = theta[int(o):int(o) + n]
            assert torch.equal(wa[int(o):int(o) + n], th - xs[t]), t
            assert torch.equal(wb[int(o):int(o) + n], th - ys[t]), t
    tree.close()
