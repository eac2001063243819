"""The RCCL transport on the one-GPU box: a single-rank `nccl` process group.

RCCL refuses two ranks on one device, so multi-peer sums are covered elsewhere (gloo on CPU,
gloo on one GPU, bench.py's parity self-check at N > 1). Here every collective code path --
async all_reduce on wire buckets, work.wait() ordering against the HIP kernels on the compute
stream, bf16 wires, device-gradient packing, the host mirror's device all-reduce -- runs over
a real RCCL communicator (an identity reduction) and must reproduce the reference bit-exact.
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

from conftest import PKG, REPO, load_npz, spin

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _flat(ts):
    return np.concatenate([t.detach().float().cpu().numpy().reshape(-1) for t in ts])


def _worker(rank, port, out):
    for p in (PKG, REPO, os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from datetime import timedelta

    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0),
                            timeout=timedelta(seconds=120))
    from diloco_amd import synth
    from diloco_amd.gradsync import GradSync
    from diloco_amd.outer import OuterSync
    from diloco_amd.trees import get_tree

    rec = {}
    # 1. engine, bucketed pipeline through RCCL, micro tree, many buckets
    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, "cuda:0"), shapes)]
    eng = OuterSync(params, world_size=1, bucket_cap_elems=4096)
    assert eng.tree.n_buckets > 2
    for s in (1, 2):
        th = [t.reshape(-1) for t in eng.unpacked(eng.theta)]
        synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in params])
        eng.step(pipeline=True)
        torch.cuda.synchronize()
        rec[f"theta_s{s}"] = _flat(eng.unpacked(eng.theta))
        rec[f"buf_s{s}"] = _flat(eng.unpacked(eng.mom))
        rec[f"inner_s{s}"] = _flat(params)
    # 2. T125 through RCCL (16 buckets) == the fused one-pass kernel, 2 steps
    spec = get_tree("t125")
    shapes = [s for _, s in spec.params()]
    pa = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, "cuda:0"), shapes)]
    pb = [t.clone() for t in pa]
    ea = OuterSync(pa, world_size=1, bucket_cap_elems=8 << 20)
    eb = OuterSync(pb, world_size=1, fuse_single=True)
    rec["t125_buckets"] = np.array([ea.tree.n_buckets])
    for s in (1, 2):
        for e, ps in ((ea, pa), (eb, pb)):
            th = [t.reshape(-1) for t in e.unpacked(e.theta)]
            synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in ps])
        ea.step(pipeline=True)
        eb.step()
    torch.cuda.synchronize()
    rec["t125_equal"] = np.array([bool(torch.equal(ea.theta, eb.theta)) and
                                  bool(torch.equal(ea.mom, eb.mom)) and
                                  all(torch.equal(x, y) for x, y in zip(pa, pb))])
    ea.close()
    eb.close()
    del ea, eb, pa, pb
    # 3. bf16 wire through RCCL == bf16 wire without the collective
    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    qa = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, "cuda:0"), shapes)]
    qb = [t.clone() for t in qa]
    fa = OuterSync(qa, world_size=1, wire_dtype=torch.bfloat16, bucket_cap_elems=4096)
    fb = OuterSync(qb, world_size=1, wire_dtype=torch.bfloat16, fuse_single=False)
    for e, ps in ((fa, qa), (fb, qb)):
        th = [t.reshape(-1) for t in e.unpacked(e.theta)]
        synth.inner_tree_device(th, 1, 0, out=[p.view(-1) for p in ps])
    fa.step(pipeline=True)
    fb.step()
    torch.cuda.synchronize()
    rec["bf16_equal"] = np.array([bool(torch.equal(fa.theta, fb.theta))])
    # 4. device-gradient DP sync (GradSync) through RCCL: identity average
    g = torch.Generator().manual_seed(9)
    gp = [torch.nn.Parameter(torch.zeros(n, device="cuda:0")) for n in (1, 3, 5000, 64, 4097)]
    for p in gp:
        p.grad = torch.randn(p.numel(), generator=g).cuda()
    before = [p.grad.clone() for p in gp]
    GradSync(gp, None, 1, bucket_cap_elems=4096).sync()
    torch.cuda.synchronize()
    rec["gradsync_equal"] = np.array([all(torch.equal(a, p.grad) for a, p in zip(before, gp))])
    # 5. the sharded variant (reduce_scatter -> dl_shard_sgd -> all_gather -> dl_scatter)
    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    sp = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, "cuda:0"), shapes)]
    es = OuterSync(sp, world_size=1, bucket_cap_elems=4096, shard=True)
    assert es.sharded and es.tree.n_buckets > 2
    for s in (1, 2):
        th = [t.reshape(-1) for t in es.unpacked(es.theta)]
        synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in sp])
        es.step()
        torch.cuda.synchronize()
        rec[f"sh_theta_s{s}"] = _flat(es.unpacked(es.theta))
        rec[f"sh_buf_s{s}"] = _flat(es.unpacked(es.momentum_full()))
        rec[f"sh_inner_s{s}"] = _flat(sp)
    # 6. the ordered sharded variant (all_to_all -> dl_shard_reduce_sgd -> all_gather), fp32
    #    on the micro tree vs the reference, bf16 vs the oracle's rank-order restatement
    for wire, tag in ((torch.float32, "a2a"), (torch.bfloat16, "a2a_bf16")):
        ap = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, "cuda:0"), shapes)]
        ea = OuterSync(ap, world_size=1, bucket_cap_elems=4096, exchange="a2a", wire_dtype=wire)
        assert ea.sharded and ea.a2a and not ea._local() and ea.tree.n_buckets > 2
        for s in (1, 2):
            th = [t.reshape(-1) for t in ea.unpacked(ea.theta)]
            synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in ap])
            ea.step()
            torch.cuda.synchronize()
            rec[f"{tag}_theta_s{s}"] = _flat(ea.unpacked(ea.theta))
            rec[f"{tag}_buf_s{s}"] = _flat(ea.unpacked(ea.momentum_full()))
            rec[f"{tag}_inner_s{s}"] = _flat(ap)
        ea.close()
    # 7. the ordered DP grad sync (GradSync(exchange="a2a")): identity average through RCCL
    for p in gp:
        p.grad = torch.randn(p.numel(), generator=g).cuda()
    before = [p.grad.clone() for p in gp]
    GradSync(gp, None, 1, bucket_cap_elems=4096, exchange="a2a").sync()
    torch.cuda.synchronize()
    rec["gradsync_a2a_equal"] = np.array([all(torch.equal(a, p.grad) for a, p in zip(before, gp))])
    np.savez(os.path.join(out, "rccl.npz"), **rec)
    dist.destroy_process_group()


def test_rccl_single_rank_transport_bit_exact():
    out = tempfile.mkdtemp(prefix="dl_rccl_")
    mp.spawn(_worker, args=(_free_port(), out), nprocs=1, join=True)
    rec = dict(np.load(os.path.join(out, "rccl.npz")))
    g = load_npz("micro_n1.npz")
    for s in (1, 2):
        assert rec[f"theta_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()
        assert rec[f"buf_s{s}"].tobytes() == g[f"buf_s{s}"].tobytes()
        assert rec[f"inner_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()
    assert rec["t125_buckets"][0] >= 8
    assert rec["t125_equal"][0]
    assert rec["bf16_equal"][0]
    assert rec["gradsync_equal"][0]
    assert rec["gradsync_a2a_equal"][0]
    for s in (1, 2):
        assert rec[f"sh_theta_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()
        assert rec[f"sh_buf_s{s}"].tobytes() == g[f"buf_s{s}"].tobytes()
        assert rec[f"sh_inner_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()
    from expect import expected_rank_order

    exp = expected_rank_order(1, wire="bf16")
    for s in (1, 2):
        for k in ("theta", "buf"):
            assert rec[f"a2a_{k}_s{s}"].tobytes() == g[f"{k}_s{s}"].tobytes(), (k, s)
            assert rec[f"a2a_bf16_{k}_s{s}"].tobytes() == exp[f"{k}_s{s}"].tobytes(), (k, s)
        assert rec[f"a2a_inner_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()
        assert rec[f"a2a_bf16_inner_s{s}"].tobytes() == exp[f"theta_s{s}"].tobytes()


def _worker_q8(rank, port, out):
    for p in (PKG, REPO, os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from datetime import timedelta

    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0),
                            timeout=timedelta(seconds=120))
    from diloco_amd import synth
    from diloco_amd.outer import OuterSync
    from diloco_amd.trees import get_tree
    from expect import MICRO_Q8_CAP

    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, "cuda:0"), shapes)]
    eng = OuterSync(params, world_size=1, wire_dtype=torch.int8, bucket_cap_elems=MICRO_Q8_CAP)
    rec = {}
    for s in (1, 2):
        th = [t.reshape(-1) for t in eng.unpacked(eng.theta)]
        synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in params])
        eng.step(pipeline=True)  # all_to_all + all_gather through RCCL
        torch.cuda.synchronize()
        rec[f"theta_s{s}"] = _flat(eng.unpacked(eng.theta))
    np.savez(os.path.join(out, "q8.npz"), **rec)
    dist.destroy_process_group()


def test_rccl_single_rank_int8_exchange():
    from expect import expected_q8

    out = tempfile.mkdtemp(prefix="dl_rccl_q8_")
    mp.spawn(_worker_q8, args=(_free_port(), out), nprocs=1, join=True)
    rec = dict(np.load(os.path.join(out, "q8.npz")))
    exp = expected_q8(1)
    for s in (1, 2):
        assert rec[f"theta_s{s}"].tobytes() == exp[f"theta_s{s}"].tobytes()


def _worker_cabi(rank, port, out):
    for p in (PKG, REPO, os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from datetime import timedelta

    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0),
                            timeout=timedelta(seconds=120))
    from diloco_amd import _lib, rccl, synth
    from diloco_amd.kernels import default_kernels
    from diloco_amd.plan import SLOT_INNER
    from diloco_amd.trees import get_tree

    rec = {}
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(100_003, generator=g).to(dev)
    for name, comm in (("torch", rccl.Comm.from_process_group(None, dev)),
                       ("own", rccl.Comm.create(1, 0, rccl.Comm.unique_id()))):
        a, b = x.clone(), x.to(torch.bfloat16)
        comm.all_reduce(a)
        comm.all_reduce(b)
        rs, ag = torch.empty_like(x), torch.empty_like(x)
        comm.reduce_scatter(rs, x)
        comm.all_gather(ag, rs)
        torch.cuda.synchronize()
        rec[f"{name}_identity"] = np.array([
            torch.equal(a, x) and torch.equal(b, x.to(torch.bfloat16)) and torch.equal(rs, x)
            and torch.equal(ag, x)])
        comm.close()
    # the outer step through the C-ABI alone: dl_delta_pack -> dl_allreduce per bucket ->
    # dl_unpack_sgd (divisor 1: one peer), on torch's communicator
    comm = rccl.Comm.from_process_group(None, dev)
    k = default_kernels()
    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, dev), shapes)]
    tree = k.tree(spec.numels(), dev, 4096)
    k.bind(tree, SLOT_INNER, params, dev)
    theta = torch.zeros(tree.total, device=dev)
    mom = torch.zeros_like(theta)
    wire = torch.zeros_like(theta)
    k.gather(tree, _lib.ALL_BUCKETS, SLOT_INNER, theta)
    for s in (1, 2):
        th = [theta[int(o):int(o) + n] for o, n in zip(tree.seg_off[:-1], spec.numels())]
        synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in params])
        for b in range(tree.n_buckets):
            lo, hi = tree.bucket_ranges[b]
            k.delta_pack(tree, b, SLOT_INNER, theta, wire)
            comm.all_reduce(wire[lo:hi])
            k.unpack_sgd(tree, b, wire, 1, theta, mom, 0.7, 0.9, True, s == 1, SLOT_INNER)
        torch.cuda.synchronize()
        rec[f"cabi_theta_s{s}"] = _flat(params)
    rec["buckets"] = np.array([tree.n_buckets])
    tree.close()
    np.savez(os.path.join(out, "cabi.npz"), **rec)
    dist.destroy_process_group()


def test_rccl_through_the_c_abi():
    """dl_allreduce / dl_reduce_scatter / dl_all_gather on torch's communicator and on one the
    library creates (identity at one rank), and a whole outer step driven through the C-ABI
    only, bit-exact vs the reference."""
    out = tempfile.mkdtemp(prefix="dl_cabi_")
    mp.spawn(_worker_cabi, args=(_free_port(), out), nprocs=1, join=True)
    rec = dict(np.load(os.path.join(out, "cabi.npz")))
    assert rec["torch_identity"][0] and rec["own_identity"][0]
    assert rec["buckets"][0] > 2
    g = load_npz("micro_n1.npz")
    for s in (1, 2):
        assert rec[f"cabi_theta_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()


def _worker_t13b(rank, port, out):
    """BASELINE configs #4/#5 at the full 1.3B tree through the bucketed collective paths over
    a one-rank RCCL communicator (25 buckets of <= 256 MiB): the pipelined all-reduce path
    (fp32 and bf16 wire) and the sharded reduce-scatter / all-gather path, each against the
    same step without the collectives, 2 outer steps, on the device (torch.equal)."""
    for p in (PKG, REPO, os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from datetime import timedelta

    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0),
                            timeout=timedelta(seconds=120))
    from diloco_amd import synth
    from diloco_amd.outer import OuterSync
    from diloco_amd.trees import get_tree

    spec = get_tree("t1.3b")
    shapes = [s for _, s in spec.params()]
    rec = {}
    cases = (("f32_pipelined", dict(wire_dtype=torch.float32, shard=False), dict(fuse_single=True)),
             ("bf16_pipelined", dict(wire_dtype=torch.bfloat16, shard=False),
              dict(wire_dtype=torch.bfloat16, fuse_single=False, tile_chunks=0)),
             ("f32_sharded", dict(wire_dtype=torch.float32, shard=True), dict(fuse_single=True)))
    for name, ka, kb in cases:
        pa = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, "cuda:0"), shapes)]
        pb = [t.clone() for t in pa]
        ea = OuterSync(pa, world_size=1, **ka)
        eb = OuterSync(pb, world_size=1, **kb)
        rec[f"{name}_buckets"] = np.array([ea.tree.n_buckets])
        for s in (1, 2):
            for e, ps in ((ea, pa), (eb, pb)):
                th = [t.reshape(-1) for t in e.unpacked(e.theta)]
                synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in ps])
            ea.step(pipeline=True)  # every bucket through RCCL (identity at one rank)
            eb.step()
        torch.cuda.synchronize()
        ma, mb = ea.momentum_full(), eb.momentum_full()
        rec[f"{name}_equal"] = np.array([
            bool(torch.equal(ea.theta, eb.theta)) and bool(torch.equal(ma, mb))
            and all(torch.equal(x, y) for x, y in zip(pa, pb))])
        rec[f"{name}_sharded"] = np.array([ea.sharded])
        ea.close()
        eb.close()
        del ea, eb, pa, pb, ma, mb
        torch.cuda.empty_cache()
    np.savez(os.path.join(out, "t13b.npz"), **rec)
    dist.destroy_process_group()


def test_rccl_t13b_bucketed_paths_match_single_pass():
    out = tempfile.mkdtemp(prefix="dl_rccl_t13b_")
    mp.spawn(_worker_t13b, args=(_free_port(), out), nprocs=1, join=True)
    rec = dict(np.load(os.path.join(out, "t13b.npz")))
    for name in ("f32_pipelined", "bf16_pipelined", "f32_sharded"):
        assert rec[f"{name}_buckets"][0] == 25, name
        assert rec[f"{name}_equal"][0], name
    assert rec["f32_sharded_sharded"][0] and not rec["f32_pipelined_sharded"][0]


def _worker_p2p(rank, port, out):
    """The RCCL payload leg of the device pipeline transport (src/comm.py:33-38,64-69): framed
    (8, 1024, 768) activations (dl_serialize on the GPU, fp32 and bf16 payloads) sent with
    dl_send and received with dl_recv (one RCCL group: a send to self on a one-rank
    communicator), on torch's communicator and on one the library creates."""
    for p in (PKG, REPO, os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from datetime import timedelta

    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0),
                            timeout=timedelta(seconds=120))
    from diloco_amd import rccl
    from diloco_amd.serializer import Serializer

    dev = torch.device("cuda", 0)
    shape = (8, 1024, 768)
    g = torch.Generator().manual_seed(17)
    acts = [torch.randn(shape, generator=g), torch.randn(shape, generator=g).to(torch.bfloat16)]
    rec = {}
    for name, comm in (("torch", rccl.Comm.from_process_group(None, dev)),
                       ("own", rccl.Comm.create(1, 0, rccl.Comm.unique_id()))):
        for i, a in enumerate(acts):
            frame = Serializer(shape).serialize(a.to(dev), (3, 40 + i))
            got = torch.full_like(frame, float("nan"))
            with rccl.group():
                comm.send(frame, 0)
                comm.recv(got, 0)
            torch.cuda.synchronize()
            payload, meta = Serializer(shape).deserialize(got)
            rec[f"{name}_{i}_meta"] = np.array(meta)
            rec[f"{name}_{i}_bytes_equal"] = np.array([bool(torch.equal(
                got.view(torch.int32)[1], frame.view(torch.int32)[1])) and bool(torch.equal(
                    got[0].flatten()[:2], frame[0].flatten()[:2]))])
            rec[f"{name}_{i}_payload"] = np.array([bool(torch.equal(payload.cpu(), a.float()))])
        comm.close()
    np.savez(os.path.join(out, "p2p.npz"), **rec)
    dist.destroy_process_group()


def test_rccl_p2p_payload_leg_carries_serialized_frames():
    out = tempfile.mkdtemp(prefix="dl_rccl_p2p_")
    mp.spawn(_worker_p2p, args=(_free_port(), out), nprocs=1, join=True)
    rec = dict(np.load(os.path.join(out, "p2p.npz")))
    for name in ("torch", "own"):
        for i in range(2):
            assert rec[f"{name}_{i}_meta"].tolist() == [3, 40 + i]
            assert rec[f"{name}_{i}_bytes_equal"][0] and rec[f"{name}_{i}_payload"][0], (name, i)


def _worker_mirror(rank, port, out):
    """The fused device outer model's exchanges over a real one-rank RCCL communicator
    (ADVICE r03): DeviceOuterMirror.all_reduce(rccl_group, 1) called directly with buckets of
    4096 elements (several per tree), so every bucket's collective is still in flight when the
    call returns and OuterSGD.step waits on the held Work handles bucket by bucket -- the
    replicated all_reduce, the sharded reduce_scatter -> shard SGD -> all_gather(θ) -> scatter,
    and the ordered all_to_all form -- then sync_inner_model; θ, the momentum buffers (gathered
    on read), the inner params and .grad recorded after each of 2 outer steps."""
    for p in (PKG, REPO, os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from datetime import timedelta
    from types import SimpleNamespace

    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      DILOCO_OUTER_BUCKET_ELEMS="4096")
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev, timeout=timedelta(seconds=120))
    from diloco_amd import synth
    from diloco_amd.trees import get_tree
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  outer_mirror, sync_inner_model)

    group = dist.new_group([0], backend="nccl")
    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    rec = {}
    for ex in ("replicated", "sharded", "a2a"):
        inner = torch.nn.Module()
        inner.ps = torch.nn.ParameterList([torch.nn.Parameter(t.view(s)) for t, s in zip(
            synth.outer_tree_device(spec, dev), shapes)])
        outer = get_outer_model(inner, "device", fused=True, exchange=ex)
        opt = get_optimizer(outer, SimpleNamespace(type="SGD", lr=0.7, momentum=0.9,
                                                   nesterov=True))
        m = outer_mirror(outer)
        rec[f"{ex}_buckets"] = np.array([m.tree.n_buckets])
        for s in (1, 2):
            synth.inner_tree_device([p.data.view(-1) for p in outer.parameters()], s, 0,
                                    out=[p.data.view(-1) for p in inner.parameters()])
            compute_pseudo_gradient(inner, outer)
            m.all_reduce(group, 1)  # TrainingComm.sync_gradients at n > 1 calls exactly this
            rec[f"{ex}_inflight_s{s}"] = np.array([m._works is not None])
            opt.step()
            sync_inner_model(outer, inner)
            rec[f"{ex}_sharded_s{s}"] = np.array([m._mom_stale])
            rec[f"{ex}_theta_s{s}"] = _flat(outer.parameters())
            rec[f"{ex}_buf_s{s}"] = _flat(opt.state[p]["momentum_buffer"]
                                          for p in outer.parameters())
            rec[f"{ex}_inner_s{s}"] = _flat(inner.parameters())
            rec[f"{ex}_avg_s{s}"] = _flat(p.grad for p in outer.parameters())
        m.close()
    np.savez(os.path.join(out, "mirror.npz"), **rec)
    dist.destroy_process_group()


def test_rccl_single_rank_device_mirror_exchanges():
    out = tempfile.mkdtemp(prefix="dl_rccl_mirror_")
    mp.spawn(_worker_mirror, args=(_free_port(), out), nprocs=1, join=True)
    rec = dict(np.load(os.path.join(out, "mirror.npz")))
    g = load_npz("micro_n1.npz")
    for ex in ("replicated", "sharded", "a2a"):
        assert rec[f"{ex}_buckets"][0] > 2, ex
        for s in (1, 2):
            assert rec[f"{ex}_inflight_s{s}"][0], ex
            assert rec[f"{ex}_sharded_s{s}"][0] == (ex != "replicated"), ex
            for k in ("theta", "buf"):
                assert rec[f"{ex}_{k}_s{s}"].tobytes() == g[f"{k}_s{s}"].tobytes(), (ex, k, s)
            assert rec[f"{ex}_inner_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes(), (ex, s)
            assert rec[f"{ex}_avg_s{s}"].tobytes() == g[f"delta_s{s}_r0"].tobytes(), (ex, s)


def _ports():
    """A port p with p + 1 free too (World puts its TCPStore on MASTER_PORT + 1)."""
    for _ in range(50):
        p = _free_port()
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", p + 1))
            except OSError:
                continue
        return p
    raise RuntimeError("no free port pair")


def _worker_train_wiring(rank, port, out):
    """The process groups src/train.py runs with, on one rank: World(swarm)
    makes the TCPStore and the gloo default group (src/world.py:32-33); TrainingComm over it;
    the DP group from DPSync.dp_group(cuda) -- the RCCL subgroup created with
    use_local_synchronization=True (diloco_amd/comm.py). No torch.cuda.set_device: the reference
    never calls it (src/train.py:368 only names cuda:local_rank). The outer model is built
    while the inner one is on the CPU (src/train.py:382), both placements; the exchange the
    mirror makes at n > 1 is called explicitly over the RCCL subgroup (sync_gradients returns
    early at one peer), its buckets in flight until OuterSGD.step waits on them; a deliberately
    slow producer (a spin kernel ahead of the packs) on the caller's stream each step."""
    for p in (PKG, REPO, os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from types import SimpleNamespace

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0", DILOCO_OUTER_BUCKET_ELEMS="4096")
    from diloco_amd import synth
    from diloco_amd.comm import TrainingComm
    from diloco_amd.trees import get_tree
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)
    from diloco_amd.world import World

    world = World(SimpleNamespace(num_stages=1))
    rec = {"default_backend": np.array([dist.get_backend()])}
    comm = TrainingComm(world, (1, 1, 32), None)
    device = torch.device("cuda", world.local_rank)  # src/utils.py:36-40
    group = comm.dp.dp_group(device)
    rec["dp_backend"] = np.array([dist.get_backend(group)])
    rec["dp_is_default"] = np.array([group is dist.group.WORLD])
    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    theta0 = synth.outer_tree(spec.numels(), spec.init_spec())
    for placement in ("host", "device"):
        inner = torch.nn.Module()
        inner.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.from_numpy(v.copy()).view(s))
                                           for v, s in zip(theta0, shapes)])
        outer = get_outer_model(inner, placement)  # src/train.py:382, inner still on the CPU
        opt = get_optimizer(outer, SimpleNamespace(type="SGD", lr=0.7, momentum=0.9,
                                                   nesterov=True))
        inner = inner.to(device)  # src/train.py:163
        for s in (1, 2):
            prev = [p.detach().cpu().numpy().reshape(-1).copy() for p in outer.parameters()]
            with torch.no_grad():
                for p, v in zip(inner.parameters(), synth.inner_tree(prev, s, 0)):
                    p.copy_(torch.from_numpy(v).view(p.shape))
            compute_pseudo_gradient(inner, outer)
            comm.sync_gradients(outer)  # one peer: returns at once (src/comm.py:118-119)
            spin(200)  # a slow producer ahead of the packs: dl_spin, 200 ms
            m = outer._diloco_mirror
            m.all_reduce(group, 1)  # what sync_gradients makes at n > 1, over the RCCL subgroup
            dm = getattr(m, "dev", m)
            rec[f"{placement}_inflight_s{s}"] = np.array([dm._works is not None])
            opt.step()
            sync_inner_model(outer, inner)
            rec[f"{placement}_theta_s{s}"] = _flat(outer.parameters())
            rec[f"{placement}_buf_s{s}"] = _flat(opt.state[p]["momentum_buffer"]
                                                 for p in outer.parameters())
            rec[f"{placement}_inner_s{s}"] = _flat(inner.parameters())
            rec[f"{placement}_avg_s{s}"] = _flat(p.grad for p in outer.parameters())
        rec[f"{placement}_device"] = np.array([str(dm.device)])
        m.close()
    np.savez(os.path.join(out, "wiring.npz"), **rec)
    dist.destroy_process_group()


def test_train_py_process_groups_rccl_dp_subgroup_over_gloo_default():
    out = tempfile.mkdtemp(prefix="dl_rccl_wiring_")
    mp.spawn(_worker_train_wiring, args=(_ports(), out), nprocs=1, join=True)
    rec = dict(np.load(os.path.join(out, "wiring.npz")))
    g = load_npz("micro_n1.npz")
    assert rec["default_backend"][0] == "gloo"
    assert rec["dp_backend"][0] == "nccl" and not rec["dp_is_default"][0]
    for placement in ("host", "device"):
        assert rec[f"{placement}_device"][0] == "cuda:0", placement
        for s in (1, 2):
            assert rec[f"{placement}_inflight_s{s}"][0], (placement, s)
            for k in ("theta", "buf"):
                assert rec[f"{placement}_{k}_s{s}"].tobytes() == g[f"{k}_s{s}"].tobytes(), \
                    (placement, k, s)
            assert rec[f"{placement}_inner_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()
            assert rec[f"{placement}_avg_s{s}"].tobytes() == g[f"delta_s{s}_r0"].tobytes()
