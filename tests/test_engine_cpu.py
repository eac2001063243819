"""OuterSync's single-process behaviour on CPU, through the oracle kernel backend
(tests/oracle_kernels.py): the sharded step's local path (one replica, no process group),
momentum export, and the engine's argument errors. The HIP kernels themselves are covered by
the -m gpu tests; here the orchestration is checked against the reference fixtures."""
import numpy as np
import pytest
import torch

from conftest import load_npz
from diloco_amd import kernels, synth
from diloco_amd.outer import OuterSync
from diloco_amd.trees import get_tree
from oracle_kernels import OracleKernels


@pytest.fixture(autouse=True)
def _oracle_backend():
    prev = kernels._DEFAULT
    kernels.set_default_kernels(OracleKernels())
    yield
    kernels._DEFAULT = prev


def _micro_params():
    spec = get_tree("micro")
    theta0 = synth.outer_tree(spec.numels(), spec.init_spec())
    return spec, [torch.from_numpy(v.copy()) for v in theta0]


def _flat(ts):
    return np.concatenate([t.reshape(-1).numpy() for t in ts])


@pytest.mark.parametrize("shard,exchange", [(False, "rccl"), (True, "rccl"), (None, "a2a")])
def test_single_replica_engine_matches_reference(shard, exchange):
    spec, params = _micro_params()
    g = load_npz("micro_n1.npz")
    e = OuterSync(params, world_size=1, bucket_cap_elems=4096, shard=shard, fuse_single=False,
                  exchange=exchange)
    assert e.sharded == (shard is not False) and e.tree.n_buckets > 2
    for s in (1, 2):
        vals = synth.inner_tree([t.numpy().reshape(-1) for t in e.unpacked(e.theta)], s, 0)
        for p, v in zip(params, vals):
            p.copy_(torch.from_numpy(v).view(p.shape))
        e.step()
        assert _flat(e.unpacked(e.theta)).tobytes() == g[f"theta_s{s}"].tobytes()
        assert _flat(e.unpacked(e.momentum_full())).tobytes() == g[f"buf_s{s}"].tobytes()
        assert _flat(params).tobytes() == g[f"theta_s{s}"].tobytes()


def test_engine_argument_errors():
    _, params = _micro_params()
    with pytest.raises(ValueError, match="int8 wire has its own exchange"):
        OuterSync(params, world_size=2, wire_dtype=torch.int8, shard=True)
    with pytest.raises(ValueError, match="wire dtype"):
        OuterSync(params, world_size=1, wire_dtype=torch.float16)
    with pytest.raises(ValueError, match="Nesterov momentum requires a momentum"):
        OuterSync(params, world_size=1, momentum=0.0, nesterov=True)
    with pytest.raises(ValueError, match="exchanges the f32 or bf16 wire"):
        OuterSync(params, world_size=2, wire_dtype=torch.int8, exchange="a2a")
    with pytest.raises(ValueError, match="shard=False contradicts"):
        OuterSync(params, world_size=2, shard=False, exchange="a2a")
    assert OuterSync(params, world_size=4, wire_dtype=torch.bfloat16, exchange="a2a").sharded
    with pytest.raises(ValueError, match="at least one parameter"):
        OuterSync([], world_size=1)
    e = OuterSync(params, world_size=1, shard=True)
    with pytest.raises(RuntimeError, match="sharded step"):
        e.apply()
    with pytest.raises(RuntimeError, match="sharded step"):
        e.all_reduce(0)


def test_automatic_variant_choice():
    _, params = _micro_params()
    assert OuterSync(params, world_size=4).sharded            # fp32 wire, n > 1
    assert not OuterSync(params, world_size=4, wire_dtype=torch.bfloat16).sharded
    assert not OuterSync(params, world_size=4, wire_dtype=torch.int8).sharded
    assert not OuterSync(params, world_size=1).sharded
    e = OuterSync(params, world_size=4, bucket_cap_elems=4096)
    for lo, hi in e.tree.bucket_ranges:  # buckets split into 4 equal 64-aligned shards
        assert lo % 256 == 0 and (hi - lo) % 256 == 0


@pytest.mark.parametrize("src_shard,dst_shard", [(False, True), (True, False), (True, True),
                                               (False, "a2a"), ("a2a", False)])
def test_checkpoint_resume_across_variants(src_shard, dst_shard):
    """state_dict after step 1 of one engine, loaded into a fresh engine of another variant /
    bucket layout: step 2 from the restored state equals the reference's step 2."""
    def kw(v):
        return {"shard": None, "exchange": "a2a"} if v == "a2a" else {"shard": v}

    spec, params = _micro_params()
    g = load_npz("micro_n1.npz")
    a = OuterSync(params, world_size=1, bucket_cap_elems=4096, fuse_single=False, **kw(src_shard))
    vals = synth.inner_tree([t.numpy().reshape(-1) for t in a.unpacked(a.theta)], 1, 0)
    for p, v in zip(params, vals):
        p.copy_(torch.from_numpy(v).view(p.shape))
    a.step()
    st = a.state_dict()
    assert st["steps"] == 1 and len(st["momentum"]) == len(params)
    _, params2 = _micro_params()
    b = OuterSync(params2, world_size=1, bucket_cap_elems=8192, fuse_single=False,
                  **kw(dst_shard))
    b.load_state_dict(st)
    assert _flat(params2).tobytes() == g["theta_s1"].tobytes()  # inner = θ_1
    vals = synth.inner_tree([t.numpy().reshape(-1) for t in b.unpacked(b.theta)], 2, 0)
    for p, v in zip(params2, vals):
        p.copy_(torch.from_numpy(v).view(p.shape))
    b.step()
    assert _flat(b.unpacked(b.theta)).tobytes() == g["theta_s2"].tobytes()
    assert _flat(b.unpacked(b.momentum_full())).tobytes() == g["buf_s2"].tobytes()


def test_load_state_dict_rejects_other_trees():
    _, params = _micro_params()
    e = OuterSync(params, world_size=1)
    st = e.state_dict()
    st["theta"] = st["theta"][:-1]
    with pytest.raises(ValueError, match="does not match"):
        e.load_state_dict(st)


def test_direct_exchange_arguments():
    _, params = _micro_params()
    with pytest.raises(ValueError, match="exchange"):
        OuterSync(params, world_size=1, exchange="tcp")
    with pytest.raises(ValueError, match="fp32 wire"):
        OuterSync(params, world_size=1, exchange="xgmi", wire_dtype=torch.bfloat16)
    e = OuterSync(params, world_size=1, exchange="xgmi")  # one rank: no peers to map
    assert e.xgmi and not e.sharded and e.peers.ok
    # xgmi_inner: the inner parameters move into the engine's packed arena, values unchanged
    before = [p.detach().clone() for p in params]
    ei = OuterSync(params, world_size=1, exchange="xgmi_inner")
    assert ei.xgmi and ei.xgmi_inner and ei.wire is None
    base, nbytes = ei.inner_arena.data_ptr(), 4 * ei.tree.total
    assert all(base <= p.data_ptr() < base + nbytes for p in params)
    assert all(torch.equal(p, b) for p, b in zip(params, before))
    with pytest.raises(RuntimeError, match="no wire"):
        ei.pseudo_gradient()
    with pytest.raises(RuntimeError, match="exchange='xgmi'"):
        e.apply()


class _CountingKernels(OracleKernels):
    """The oracle backend, counting pointer-table binds per slot."""

    def __init__(self):
        super().__init__()
        self.binds = 0

    def bind(self, tree, slot, tensors, device):
        self.binds += 1
        return super().bind(tree, slot, tensors, device)


@pytest.mark.parametrize("kind", ["sharded", "tiled", "two_kernel", "int8", "fused"])
def test_one_bind_per_outer_step(kind):
    """step() binds the inner slot once, however many buckets the step walks (the per-bucket
    building blocks only bind when called on their own)."""
    _, params = _micro_params()
    k = _CountingKernels()
    kw = {"sharded": dict(shard=True, fuse_single=False),
          "tiled": dict(fuse_single=False, tile_chunks=1),
          "two_kernel": dict(fuse_single=False, tile_chunks=0),
          "int8": dict(wire_dtype=torch.int8),
          "fused": dict(fuse_single=True, keep_wire=True)}[kind]
    e = OuterSync(params, world_size=1, bucket_cap_elems=4096, kernels=k, **kw)
    assert e.tree.n_buckets > 2
    for _ in range(3):
        before = k.binds
        e.step()
        assert k.binds - before == 1, kind
    before = k.binds
    e.pseudo_gradient(0)  # on its own: binds
    assert k.binds - before == 1


def test_int8_single_replica_whole_tree_equals_per_bucket():
    """The one-replica int8 step in three whole-tree launches equals the per-bucket sequence
    (dl_delta_q8 -> dl_q8_reduce -> dl_unpack_sgd_q8 per bucket): at n = 1 no bucket is padded,
    so the slots of consecutive buckets are the tree's chunks in order."""
    spec, params_a = _micro_params()
    _, params_b = _micro_params()
    a = OuterSync(params_a, world_size=1, bucket_cap_elems=4096, wire_dtype=torch.int8)
    b = OuterSync(params_b, world_size=1, bucket_cap_elems=4096, wire_dtype=torch.int8)
    assert a.tree.n_buckets > 2
    for s in (1, 2):
        vals = synth.inner_tree([t.numpy().reshape(-1) for t in a.unpacked(a.theta)], s, 0)
        for pa, pb, v in zip(params_a, params_b, vals):
            pa.copy_(torch.from_numpy(v).view(pa.shape))
            pb.copy_(torch.from_numpy(v).view(pb.shape))
        a.step()
        for k in range(b.tree.n_buckets):  # the pre-round-2 per-bucket sequence
            b.pseudo_gradient(k)
            _nch, m, _ = b.q8_plan[k]
            region = b.q8_region(k)
            b.k.q8_reduce(region, 1, m, 1, region)
            b.apply(k)
        b.steps_done += 1
        assert a.theta.numpy().tobytes() == b.theta.numpy().tobytes()
        assert a.mom.numpy().tobytes() == b.mom.numpy().tobytes()
        assert a.q_slots.numpy().tobytes() == b.q_slots.numpy().tobytes()
        assert _flat(params_a).tobytes() == _flat(params_b).tobytes()


def test_gradsync_single_replica_without_group_is_identity():
    """GradSync at one replica with no process group: gather -> identity -> /1 back, every
    gradient unchanged (the path runs; nothing is exchanged)."""
    from diloco_amd.gradsync import GradSync

    params = [torch.nn.Parameter(torch.zeros(n)) for n in (1, 3, 5000, 64, 4097)]
    for i, p in enumerate(params):
        p.grad = torch.full_like(p, float(i) + 0.25)
    gs = GradSync(params, None, 1, bucket_cap_elems=4096)
    assert gs.tree.n_buckets > 1
    gs.sync()
    for i, p in enumerate(params):
        assert torch.equal(p.grad, torch.full_like(p, float(i) + 0.25))
        o = int(gs.tree.seg_off[i])
        assert torch.equal(gs.wire[o:o + p.numel()], p.grad)
