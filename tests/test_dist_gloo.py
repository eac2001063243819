"""Multi-process (gloo, CPU) tests of the N > 1 path: the drop-in surface and the engines.

Each case spawns world_size processes on 127.0.0.1. The kernel backend is the oracle checker
(tests/oracle_kernels.py); everything above it -- TrainingComm.sync_gradients, the host outer
mirror and its coherence, OuterSGD, OuterSync's bucket pipeline over a real process group,
World's stage/DP-group topology -- is the product code. Results are compared with the
reference's own outputs (tests/golden/micro_n{2,4}.npz): bit-exact at 2 peers, normwise at 4.
"""
import os
import socket
import sys
import tempfile
from collections import namedtuple

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO, load_npz, normwise_ok, split
from expect import MICRO_Q8_CAP, expected_bf16_allreduce, expected_q8, expected_rank_order

MICRO_STEPS = 2
# stand-in for src/metrics.py Outputs (a pydantic model there); module level so it pickles
Outputs = namedtuple("Outputs", "step tokens num_micro_batches time loss lr norm micro_step_time")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Cfg:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def _micro_module(values, shapes):
    m = torch.nn.Module()
    m.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.from_numpy(v.copy()).view(s))
                                   for v, s in zip(values, shapes)])
    return m


def _worker(rank, world, port, mode, num_stages, out):
    for p in (PKG, REPO, os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    torch.set_num_threads(1)
    os.environ["DILOCO_P2P_BACKEND"] = "gloo"  # the device transport's data groups, on CPU
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    from diloco_amd import kernels, synth
    from diloco_amd.comm import TrainingComm
    from diloco_amd.outer import OuterSync
    from diloco_amd.trees import get_tree
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)
    from diloco_amd.world import World
    from oracle_kernels import OracleKernels

    if mode != "dropin_host":
        kernels.set_default_kernels(OracleKernels())
    world_ = World.from_default_group(num_stages)
    dp_rank = world_.dp_ranks.index(rank)
    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    theta0 = synth.outer_tree(spec.numels(), spec.init_spec())
    rec = {}
    if mode in ("dropin", "dropin_device", "dropin_deferred", "dropin_host",
                "dropin_device_quiet", "dropin_device_eager", "dropin_device_bf16",
                "dropin_device_bf16_eager", "dropin_device_quiet_buckets",
                "dropin_device_quiet_replicated", "dropin_device_quiet_a2a",
                "dropin_device_a2a_dp", "dropin_a2a_dp", "dropin_device_momentum_first",
                "dropin_device_eager_a2a_dp", "dropin_sync", "dropin_sync_a2a_dp",
                "dropin_quiet", "dropin_quiet_sharded", "dropin_device_int8",
                "dropin_device_int8_eager", "dropin_int8"):
        if mode in ("dropin_device_quiet_buckets", "dropin_device_quiet_a2a",
                    "dropin_device_momentum_first", "dropin_device_int8",
                    "dropin_device_int8_eager", "dropin_int8"):  # several buckets: the
            os.environ["DILOCO_OUTER_BUCKET_ELEMS"] = "4096"  # SGD waits bucket by bucket
        if mode.endswith("_a2a_dp"):  # DILOCO_DP_EXCHANGE=a2a behind sync_gradients
            import diloco_amd.comm as comm_mod

            comm_mod.DP_EXCHANGE = "a2a"
        exchange = ("replicated" if mode.endswith("_replicated")
                    else "sharded" if mode.endswith("_sharded")
                    else "a2a" if mode == "dropin_device_quiet_a2a" else None)
        from diloco_amd.utils import flush_outer_model, has_mirror

        deferred = mode == "dropin_deferred"
        # dropin / dropin_quiet / dropin_a2a_dp: the default host placement (write_back "lazy",
        # the outer step on an HBM twin); dropin_sync*: the host tensors authoritative
        sync = mode.startswith("dropin_sync")
        # quiet: nothing reads the outer model between the four calls (src/train.py:261-269),
        # so the fused device model defers the delta and the /n into its one SGD pass
        quiet = mode in ("dropin_device_quiet", "dropin_device_bf16", "dropin_device_quiet_buckets",
                         "dropin_device_quiet_replicated", "dropin_device_quiet_a2a",
                         "dropin_device_a2a_dp", "dropin_device_momentum_first", "dropin_quiet",
                         "dropin_quiet_sharded", "dropin_device_int8")
        device = mode.startswith("dropin_device")
        inner = _micro_module(theta0, shapes)
        outer = get_outer_model(inner, placement="device" if device else None,
                                write_back="deferred" if deferred else "sync" if sync else None,
                                fused="_eager" not in mode,
                                wire="bf16" if "bf16" in mode else "int8" if "int8" in mode
                                else None, exchange=exchange)
        opt = get_optimizer(outer, _Cfg(type="SGD", lr=0.7, momentum=0.9, nesterov=True))
        assert type(opt).__name__ == "OuterSGD"
        from diloco_amd.utils import outer_mirror
        if mode == "dropin_host":  # the product's own host path: no kernel backend, no mirror
            assert not has_mirror(outer)
        else:
            assert type(outer_mirror(outer)).__name__ == (
                "DeviceOuterMirror" if device else
                "HostOuterMirror" if (sync or deferred) else "LazyHostOuterMirror")
            if device:
                assert outer_mirror(outer).fused == ("_eager" not in mode)
                if "DILOCO_OUTER_BUCKET_ELEMS" in os.environ:
                    assert outer_mirror(outer).tree.n_buckets > 2
        comm = TrainingComm(world_, (1, 1, 32), None)
        for s in range(1, MICRO_STEPS + 1):
            prev = [p.detach().numpy().reshape(-1).copy() for p in outer.parameters()]
            vals = synth.inner_tree(prev, s, dp_rank)
            with torch.no_grad():
                for p, v in zip(inner.parameters(), vals):
                    p.copy_(torch.from_numpy(v).view(p.shape))
            def host(ts):
                return np.concatenate([t.detach().numpy().reshape(-1) for t in ts])

            # deferred write-back: outer step 1 flushes after every call (the mid-sequence
            # flush path), outer step 2 reads the host tensors only after sync_inner_model
            mid = not quiet and (not deferred or s == 1)
            compute_pseudo_gradient(inner, outer)
            if deferred and s == 1:
                flush_outer_model(outer)
            if mid:
                rec[f"delta_s{s}"] = host(p.grad for p in outer.parameters())
            comm.sync_gradients(outer)
            if deferred and s == 1:
                flush_outer_model(outer)
            if mid:
                rec[f"avg_s{s}"] = host(p.grad for p in outer.parameters())
            elif deferred and len(world_.dp_ranks) > 1:  # the host still has step 1's averages
                assert host(p.grad for p in outer.parameters()).tobytes() == rec["avg_s1"].tobytes()
            opt.step()
            if quiet and len(world_.dp_ranks) > 1:  # which exchange the step ran
                m = outer_mirror(outer)
                m = getattr(m, "dev", m)  # the lazy host placement's HBM twin
                rec["sharded_step"] = np.array([m._mom_stale, m._xmode is not None])
            if deferred and s == 1:
                flush_outer_model(outer)
            if mid:
                rec[f"theta_s{s}"] = host(outer.parameters())
                rec[f"buf_s{s}"] = host(opt.state[p]["momentum_buffer"] for p in outer.parameters())
            sync_inner_model(outer, inner)
            if not mid:
                if deferred:  # quiet: reading .grad itself completes the pending /n
                    flush_outer_model(outer)
                if mode == "dropin_device_momentum_first":
                    # the sharded momentum gathered first (through a deepcopy of the state and
                    # a torch.save round trip), .grad after it
                    import copy
                    import io

                    st = copy.deepcopy(dict(opt.state))  # MomentumBuffer.__deepcopy__
                    assert all(type(v["momentum_buffer"]) is torch.Tensor for v in st.values())
                    rec[f"buf_s{s}"] = host(v["momentum_buffer"] for v in st.values())
                    bio = io.BytesIO()
                    torch.save(opt.state_dict(), bio)
                    bio.seek(0)
                    ld = torch.load(bio, weights_only=True)
                    assert host(ld["state"][i]["momentum_buffer"] for i in range(
                        len(ld["state"]))).tobytes() == rec[f"buf_s{s}"].tobytes()
                rec[f"avg_s{s}"] = host(p.grad for p in outer.parameters())
                rec[f"theta_s{s}"] = host(outer.parameters())
                bufs = host(opt.state[p]["momentum_buffer"] for p in outer.parameters())
                if mode == "dropin_device_momentum_first":
                    assert bufs.tobytes() == rec[f"buf_s{s}"].tobytes()
                rec[f"buf_s{s}"] = bufs
            rec[f"inner_s{s}"] = np.concatenate([p.detach().numpy().reshape(-1) for p in inner.parameters()])
        if mode == "dropin_host":
            assert not has_mirror(outer)  # every call took the reference's host semantics
    elif mode in ("engine", "engine_ar", "engine_a2a"):
        # engine: the default at n > 1, reduce-scatter -> shard SGD -> all-gather;
        # engine_ar: the replicated variant, all-reduce -> full SGD on every peer;
        # engine_a2a: the sharded step with all_to_all + rank-order reduce (exchange="a2a")
        params = [torch.from_numpy(v.copy()) for v in theta0]
        eng = OuterSync(params, lr=0.7, momentum=0.9, nesterov=True,
                        group=world_.curr_stage_group, world_size=len(world_.dp_ranks),
                        bucket_cap_elems=4096, shard=None if mode != "engine_ar" else False,
                        exchange="a2a" if mode == "engine_a2a" else "rccl")
        assert eng.sharded == (mode != "engine_ar") and eng.a2a == (mode == "engine_a2a")
        assert eng.tree.n_buckets > 2
        for s in range(1, MICRO_STEPS + 1):
            th = eng.unpacked(eng.theta)
            vals = synth.inner_tree([t.numpy().reshape(-1) for t in th], s, dp_rank)
            for p, v in zip(params, vals):
                p.copy_(torch.from_numpy(v))
            eng.step()
            rec[f"theta_s{s}"] = np.concatenate([t.numpy().reshape(-1) for t in eng.unpacked(eng.theta)])
            mom = eng.momentum_full()
            rec[f"buf_s{s}"] = np.concatenate([t.numpy().reshape(-1) for t in eng.unpacked(mom)])
            rec[f"inner_s{s}"] = np.concatenate([p.numpy().reshape(-1) for p in params])
    elif mode == "engine_resume":
        # sharded engine: step 1, state_dict (momentum all-gathered), a fresh sharded engine
        # with another bucket layout loads it (each rank takes its own shards), step 2
        params = [torch.from_numpy(v.copy()) for v in theta0]
        grp, n = world_.curr_stage_group, len(world_.dp_ranks)
        a = OuterSync(params, group=grp, world_size=n, bucket_cap_elems=4096)
        vals = synth.inner_tree([t.numpy().reshape(-1) for t in a.unpacked(a.theta)], 1, dp_rank)
        for p, v in zip(params, vals):
            p.copy_(torch.from_numpy(v))
        a.step()
        st = a.state_dict()
        params2 = [torch.from_numpy(v.copy()) for v in theta0]
        b = OuterSync(params2, group=grp, world_size=n, bucket_cap_elems=12288)
        assert b.sharded and b.tree.n_buckets != a.tree.n_buckets
        b.load_state_dict(st)
        vals = synth.inner_tree([t.numpy().reshape(-1) for t in b.unpacked(b.theta)], 2, dp_rank)
        for p, v in zip(params2, vals):
            p.copy_(torch.from_numpy(v))
        b.step()
        rec["theta_s2"] = np.concatenate([t.numpy().reshape(-1) for t in b.unpacked(b.theta)])
        rec["buf_s2"] = np.concatenate([t.numpy().reshape(-1)
                                        for t in b.unpacked(b.momentum_full())])
    elif mode == "engine_q8":
        params = [torch.from_numpy(v.copy()) for v in theta0]
        eng = OuterSync(params, lr=0.7, momentum=0.9, nesterov=True, wire_dtype=torch.int8,
                        group=world_.curr_stage_group, world_size=len(world_.dp_ranks),
                        bucket_cap_elems=MICRO_Q8_CAP)
        assert eng.tree.n_buckets > 2
        for s in range(1, MICRO_STEPS + 1):
            th = eng.unpacked(eng.theta)
            vals = synth.inner_tree([t.numpy().reshape(-1) for t in th], s, dp_rank)
            for p, v in zip(params, vals):
                p.copy_(torch.from_numpy(v))
            eng.step()
            rec[f"theta_s{s}"] = np.concatenate([t.numpy().reshape(-1) for t in eng.unpacked(eng.theta)])
            rec[f"inner_s{s}"] = np.concatenate([p.numpy().reshape(-1) for p in params])
    elif mode == "dpsync_a2a":
        # TrainingComm.sync_gradients on a plain-DP model (device grads under the oracle
        # backend) with DILOCO_DP_EXCHANGE=a2a: the ordered GradSync behind the reference call
        import diloco_amd.comm as comm_mod

        comm_mod.DP_EXCHANGE = "a2a"
        g = torch.Generator().manual_seed(100 + rank)
        m = torch.nn.Module()
        m.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.zeros(n))
                                       for n in (1, 3, 5000, 64, 4097)])
        for p in m.parameters():
            p.grad = torch.randn(p.numel(), generator=g)
        TrainingComm(world_, (1, 1, 4), None).sync_gradients(m)
        rec["got"] = np.concatenate([p.grad.numpy() for p in m.parameters()])
    elif mode in ("gradsync", "gradsync_a2a"):
        from diloco_amd.gradsync import GradSync

        g = torch.Generator().manual_seed(100 + rank)
        params = [torch.nn.Parameter(torch.zeros(n)) for n in (1, 3, 5000, 64, 4097)]
        for p in params:
            p.grad = torch.randn(p.numel(), generator=g)
        ref = [p.grad.clone() for p in params]
        for r in ref:  # the reference's loop, src/comm.py:120-123
            dist.all_reduce(r, op=dist.ReduceOp.SUM, group=world_.curr_stage_group)
            r /= len(world_.dp_ranks)
        gs = GradSync(params, world_.curr_stage_group, len(world_.dp_ranks), bucket_cap_elems=4096,
                      exchange="a2a" if mode == "gradsync_a2a" else "rccl")
        gs.sync()
        rec["got"] = np.concatenate([p.grad.numpy() for p in params])
        rec["ref"] = np.concatenate([r.numpy() for r in ref])
    elif mode == "p2p_device":
        # header over the stage gloo group + payload over a data group
        # (gloo here: CPU); stage 0 sends forward to random stage-1 ranks (src/comm.py:91),
        # stage 1 answers backward to the sender
        import random

        from diloco_amd.serializer import Serializer

        class CpuSerializer(Serializer):  # the reference's framing, on CPU tensors
            def serialize(self, t, m):
                meta = torch.zeros(t.numel())
                meta[0], meta[1] = float(m[0]), float(m[1])
                return torch.cat([meta.view(t.shape)[None], t[None].float()])

        shape = (1, 4, 8)
        comm = TrainingComm(world_, shape, None, transport="device",
                            device=torch.device("cpu"), serializer_factory=CpuSerializer)
        K = 5
        random.seed(100 + rank)
        stage1 = world_.stage2ranks[1]
        if world_.stage == 0:
            for i in range(K):
                t = torch.arange(32, dtype=torch.float32).view(shape) + 1000 * rank + i
                comm.send_forward(t, (rank, i))
            got = []
            for _ in range(K):
                src, t, meta = comm.recv_backward()
                got.append((src, meta[0], meta[1], float(t.sum())))
            rec["got"] = np.array(sorted(got), dtype=np.float64)
        else:
            # each sender draws K choices in sequence: replay them exactly
            n_in = 0
            for r in world_.stage2ranks[0]:
                g = random.Random(100 + r)
                n_in += sum(g.choice(stage1) == rank for _ in range(K))
            seen = []
            for _ in range(n_in):
                src, t, meta = comm.recv_forward()
                assert t.requires_grad and t.shape == shape
                seen.append((src, meta[0], meta[1], float(t.sum())))
                comm.send_backward(src, (t * 2).detach(), meta)
            rec["seen"] = np.array(sorted(seen), dtype=np.float64).reshape(-1, 4)
        dist.barrier()
    elif mode in ("adamw_lazy", "adamw_device"):
        # an AdamW outer optimizer (src/utils.py:60-61) on the sharded exchange: AdamW reads
        # .grad (a collective gather of the reduce-scattered slices, every rank in the same
        # order) and writes θ in place; against the reference's calls on a plain deepcopy
        # outer model with per-tensor all_reduce / n (src/comm.py:117-123), in this process
        import copy

        os.environ["DILOCO_OUTER_BUCKET_ELEMS"] = "4096"
        n = len(world_.dp_ranks)
        if n > 2:  # AdamW's g / sqrt(v) amplifies any change of sum order: the rank-order form
            import diloco_amd.comm as comm_mod

            comm_mod.DP_EXCHANGE = "a2a"
        inner = _micro_module(theta0, shapes)
        ref_inner = copy.deepcopy(inner)
        ref_outer = copy.deepcopy(ref_inner)
        outer = get_outer_model(inner, placement="device" if mode == "adamw_device" else None)
        cfg = _Cfg(type="AdamW", lr=0.01, weight_decay=0.1, betas=(0.9, 0.95))
        opt, ref_opt = get_optimizer(outer, cfg), get_optimizer(ref_outer, cfg)
        comm = TrainingComm(world_, (1, 1, 32), None)

        def host(ts):
            return np.concatenate([t.detach().numpy().reshape(-1) for t in ts])

        for s in range(1, 4):
            vals = synth.inner_tree([p.detach().numpy().reshape(-1).copy()
                                     for p in ref_outer.parameters()], s, dp_rank)
            with torch.no_grad():
                for p, q, v in zip(inner.parameters(), ref_inner.parameters(), vals):
                    p.copy_(torch.from_numpy(v).view(p.shape))
                    q.copy_(p)
            compute_pseudo_gradient(inner, outer)
            comm.sync_gradients(outer)
            opt.step()
            sync_inner_model(outer, inner)
            for po, pi in zip(ref_outer.parameters(), ref_inner.parameters()):
                po.grad = po.data - pi.data
                if n <= 2:
                    dist.all_reduce(po.grad, op=dist.ReduceOp.SUM)
                else:  # Σ in rank order, fp32, left to right
                    parts = [torch.empty_like(po.grad) for _ in range(n)]
                    dist.all_gather(parts, po.grad)
                    po.grad = parts[0].clone()
                    for q in parts[1:]:
                        po.grad += q
                po.grad /= n
            ref_opt.step()
            with torch.no_grad():
                for po, pi in zip(ref_outer.parameters(), ref_inner.parameters()):
                    pi.copy_(po)
            rec[f"theta_s{s}"] = host(outer.parameters())
            rec[f"inner_s{s}"] = host(inner.parameters())
            rec[f"avg_s{s}"] = host(p.grad for p in outer.parameters())
            rec[f"exp_avg_sq_s{s}"] = host(opt.state[p]["exp_avg_sq"] for p in outer.parameters())
            rec[f"ref_theta_s{s}"] = host(ref_outer.parameters())
            rec[f"ref_avg_s{s}"] = host(p.grad for p in ref_outer.parameters())
            rec[f"ref_exp_avg_sq_s{s}"] = host(ref_opt.state[p]["exp_avg_sq"]
                                               for p in ref_outer.parameters())
    elif mode in ("lone_read_default", "lone_read_sharded", "lone_read_device"):
        # after an outer step, rank 0 alone reads the outer optimizer's
        # state_dict() and .grad -- in the reference local CPU tensors (src/utils.py:218-221,
        # torch SGD state at src/train.py:267). Default placement (replicated exchange): the
        # reference's values, and the peers go on to the next step. Sharded (opted in on the
        # host placement; the device placement's default): the read is a collective its peer
        # does not make -> RuntimeError within the deadline, and the peer's late read of the
        # same values raises too instead of entering an all_gather alone.
        import time

        os.environ["DILOCO_COLLECTIVE_READ_TIMEOUT"] = "3"
        sharded = mode != "lone_read_default"
        inner = _micro_module(theta0, shapes)
        outer = get_outer_model(inner, placement="device" if mode == "lone_read_device" else None,
                                exchange="sharded" if mode == "lone_read_sharded" else None)
        from diloco_amd.utils import outer_mirror

        m = outer_mirror(outer)
        rec["exchange"] = np.array(getattr(m, "dev", m).exchange)
        opt = get_optimizer(outer, _Cfg(type="SGD", lr=0.7, momentum=0.9, nesterov=True))
        comm = TrainingComm(world_, (1, 1, 32), None)

        def host(ts):
            return np.concatenate([t.detach().numpy().reshape(-1) for t in ts])

        def outer_step(s):  # src/train.py:263-269, nothing read in between
            vals = synth.inner_tree([p.detach().numpy().reshape(-1).copy()
                                     for p in outer.parameters()], s, dp_rank)
            with torch.no_grad():
                for p, v in zip(inner.parameters(), vals):
                    p.copy_(torch.from_numpy(v).view(p.shape))
            compute_pseudo_gradient(inner, outer)
            comm.sync_gradients(outer)
            opt.step()
            sync_inner_model(outer, inner)

        outer_step(1)
        reads = (("state_dict", lambda: host(st["momentum_buffer"]
                                            for st in opt.state_dict()["state"].values())),
                 ("grad", lambda: host(p.grad for p in outer.parameters())))
        if dp_rank == 0 or sharded:
            if dp_rank != 0:
                time.sleep(7.0)  # past rank 0's two deadlines: the same reads, late
            for name, read in reads:
                t0 = time.time()
                try:
                    rec[f"{name}_s1"] = read()
                    rec[f"{name}_outcome"] = np.array("values")
                except RuntimeError as e:
                    rec[f"{name}_outcome"] = np.array("raised")
                    rec[f"{name}_msg"] = np.array(str(e))
                rec[f"{name}_secs"] = np.float64(time.time() - t0)
        if not sharded:  # the group is intact: a second step, read on every rank
            outer_step(2)
            rec["theta_s2"] = host(outer.parameters())
            rec["grad_s2"] = host(p.grad for p in outer.parameters())
    elif mode == "outputs":
        comm = TrainingComm(world_, (1, 1, 4), None)
        o = Outputs(step=3, tokens=100 * (rank + 1), num_micro_batches=rank, time=1.0 + rank,
              loss=0.0 if rank == 0 else 2.0 * rank, lr=None, norm=0.5, micro_step_time=0.1)
        agg = comm.sync_outputs(o)
        rec["agg"] = np.array([agg.tokens, agg.num_micro_batches, agg.time, agg.loss, agg.norm])
    np.savez(os.path.join(out, f"{mode}_r{rank}.npz"), **rec)
    dist.barrier()
    dist.destroy_process_group()


def _run(mode, world, num_stages=1):
    out = tempfile.mkdtemp(prefix="dl_gloo_")
    # forked workers: CPU only (no HIP state to inherit), and each skips re-importing torch --
    # the suite's time was mostly spawned children starting up (7.7 -> 3.2 min serial)
    mp.start_processes(_worker, args=(world, _free_port(), mode, num_stages, out), nprocs=world,
                       join=True, start_method="fork")
    return [dict(np.load(os.path.join(out, f"{mode}_r{r}.npz"))) for r in range(world)]


@pytest.mark.parametrize("mode", ["dropin", "dropin_device", "dropin_device_quiet",
                                  "dropin_device_quiet_buckets", "dropin_device_quiet_replicated",
                                  "dropin_device_quiet_a2a", "dropin_device_a2a_dp",
                                  "dropin_a2a_dp", "dropin_device_momentum_first",
                                  "dropin_device_eager_a2a_dp", "dropin_sync", "dropin_quiet",
                                  "dropin_quiet_sharded",
                                  "dropin_sync_a2a_dp",
                                  "dropin_device_eager", "dropin_deferred", "engine",
                                  "engine_ar", "engine_a2a", "dropin_host"])
def test_two_peers_match_reference_bit_exact(mode):
    g = load_npz("micro_n2.npz")
    recs = _run(mode, 2)
    for rec in recs:
        for s in (1, 2):
            for k in ("theta", "buf"):
                assert rec[f"{k}_s{s}"].tobytes() == g[f"{k}_s{s}"].tobytes(), (mode, k, s)
            assert rec[f"inner_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()
            if mode.startswith("dropin"):
                assert rec[f"avg_s{s}"].tobytes() == g[f"avg_s{s}"].tobytes()
    if mode.startswith("dropin") and "delta_s1" in recs[0]:
        assert recs[0]["delta_s1"].tobytes() == g["delta_s1_r0"].tobytes()
        assert recs[1]["delta_s1"].tobytes() == g["delta_s1_rlast"].tobytes()
    if "sharded_step" in recs[0]:  # which exchange ran: the device placement's default is
        # sharded, the host placement's replicated (reads local)
        want = ((mode.startswith("dropin_device") and not mode.endswith("_replicated"))
                or mode.endswith("_sharded"))
        assert all(bool(r["sharded_step"].all()) == want for r in recs), mode


@pytest.mark.parametrize("mode", ["dropin_device_quiet_a2a", "dropin_device_a2a_dp",
                                  "dropin_a2a_dp", "dropin_device_eager_a2a_dp",
                                  "dropin_sync_a2a_dp"])
@pytest.mark.parametrize("world", [4, 8])
def test_dropin_ordered_exchange_is_bit_exact_at_any_n(mode, world):
    """The outer model's ordered exchange (get_outer_model(..., exchange="a2a"), or
    DILOCO_DP_EXCHANGE=a2a behind TrainingComm.sync_gradients, host and device placements,
    fused and eager): every replica's .grad, θ, momentum and inner params bit-identical to the
    oracle's rank-order restatement at 4 and 8 peers (the reduce-scatter / all_reduce order
    is the transport's)."""
    exp = expected_rank_order(world)
    for rec in _run(mode, world):
        for s in (1, 2):
            for k in ("theta", "buf", "avg"):
                assert rec[f"{k}_s{s}"].tobytes() == exp[f"{k}_s{s}"].tobytes(), (mode, k, s)
            assert rec[f"inner_s{s}"].tobytes() == exp[f"theta_s{s}"].tobytes(), (mode, s)


@pytest.mark.parametrize("mode,world", [("dropin", 4), ("engine", 4), ("engine_ar", 4),
                                        ("dropin", 8), ("engine", 8), ("dropin_host", 4),
                                        ("dropin_device_quiet", 4),
                                        ("dropin_device_quiet_buckets", 4),
                                        ("dropin_device_quiet_buckets", 8),
                                        ("dropin_device_momentum_first", 8),
                                        ("dropin_quiet", 8), ("dropin_quiet_sharded", 8),
                                        ("dropin_sync", 4),
                                        ("dropin_device_quiet_replicated", 4)])
def test_four_and_eight_peers_match_reference_normwise(mode, world):
    """4 and 8 DP peers (8: the north star's DP = 8) against the reference's own gloo run."""
    from diloco_amd.trees import get_tree

    numels = get_tree("micro").numels()
    g = load_npz(f"micro_n{world}.npz")
    recs = _run(mode, world)
    for rec in recs:
        for s in (1, 2):
            for k in ("theta", "buf"):
                for a, b in zip(split(rec[f"{k}_s{s}"], numels), split(g[f"{k}_s{s}"], numels)):
                    assert normwise_ok(a, b, 1e-6), (mode, k, s)
    for s in (1, 2):  # every replica holds the same averaged state
        assert all(r[f"theta_s{s}"].tobytes() == recs[0][f"theta_s{s}"].tobytes() for r in recs)


def test_lone_read_on_the_default_placement_is_local():
    """on get_outer_model's default placement rank 0 alone reads the outer
    optimizer's state_dict() and .grad after an outer step; both are the reference's values
    (micro_n2.npz: the momentum and the average after step 1), and the two ranks then make
    a second step that is still the reference's."""
    g = load_npz("micro_n2.npz")
    r0, r1 = _run("lone_read_default", 2)
    assert str(r0["exchange"]) == "replicated"
    assert str(r0["state_dict_outcome"]) == "values" and str(r0["grad_outcome"]) == "values"
    assert r0["state_dict_s1"].tobytes() == g["buf_s1"].tobytes()
    assert r0["grad_s1"].tobytes() == g["avg_s1"].tobytes()
    assert "state_dict_outcome" not in r1  # rank 1 read nothing
    for r in (r0, r1):
        assert r["theta_s2"].tobytes() == g["theta_s2"].tobytes()
        assert r["grad_s2"].tobytes() == g["avg_s2"].tobytes()


@pytest.mark.parametrize("mode", ["lone_read_sharded", "lone_read_device"])
def test_lone_collective_read_raises_within_the_deadline(mode):
    """Under the sharded exchange (opted in on the host placement; the device placement's
    default) the same lone read is a collective its peer does not make: it raises
    RuntimeError on rank 0 within the 3 s deadline (DILOCO_COLLECTIVE_READ_TIMEOUT) instead of
    hanging, and rank 1's later reads of the same values raise at once instead of entering an
    all_gather alone."""
    r0, r1 = _run(mode, 2)
    assert str(r0["exchange"]) == "sharded"
    for name in ("state_dict", "grad"):
        assert str(r0[f"{name}_outcome"]) == "raised", name
        assert "collective over the DP group" in str(r0[f"{name}_msg"])
        assert 2.5 <= float(r0[f"{name}_secs"]) < 8.0, float(r0[f"{name}_secs"])
        assert str(r1[f"{name}_outcome"]) == "raised", name
        assert float(r1[f"{name}_secs"]) < 2.0, float(r1[f"{name}_secs"])


def test_sharded_engine_checkpoint_resume_two_peers():
    g = load_npz("micro_n2.npz")
    for rec in _run("engine_resume", 2):
        assert rec["theta_s2"].tobytes() == g["theta_s2"].tobytes()
        assert rec["buf_s2"].tobytes() == g["buf_s2"].tobytes()


def test_two_stages_reduce_within_their_dp_groups():
    """World(num_stages=2) on 4 ranks: stage = rank % 2, DP groups {0,2} and {1,3}
    (src/world.py:96-97); each group's outer step equals the 2-peer reference run."""
    g = load_npz("micro_n2.npz")
    recs = _run("dropin", 4, num_stages=2)
    for rec in recs:
        for s in (1, 2):
            assert rec[f"theta_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()
            assert rec[f"avg_s{s}"].tobytes() == g[f"avg_s{s}"].tobytes()


@pytest.mark.parametrize("world", [2, 4])
def test_gradsync_equals_per_tensor_allreduce(world):
    recs = _run("gradsync", world)
    for rec in recs:
        if world == 2:
            assert rec["got"].tobytes() == rec["ref"].tobytes()
        else:
            assert normwise_ok(rec["got"], rec["ref"], 1e-6)


def test_device_p2p_transport_protocol():
    """Header/payload split of the device p2p transport on 4 ranks / 2 stages: every forward
    message reaches the rank its sender drew, with its metadata and payload; every backward
    reply returns to its sender (src is the header's rank)."""
    recs = _run("p2p_device", 4, num_stages=2)
    base = float(np.arange(32).sum())
    for r in (0, 2):  # stage 0: K replies each, payload doubled
        got = recs[r]["got"]
        assert len(got) == 5 and set(got[:, 1]) == {r}
        assert sorted(got[:, 2]) == [0, 1, 2, 3, 4]
        for src, root, i, tot in got:
            assert src in (1, 3) and tot == 2 * (base + 32 * (1000 * r + i))
    seen = np.concatenate([recs[1]["seen"], recs[3]["seen"]])
    assert len(seen) == 10
    for src, root, i, tot in seen:
        assert src == root and tot == base + 32 * (1000 * src + i)


def test_single_peer_host_dropin_matches_reference():
    """--device cpu with one DP peer (BASELINE config #1's reference path at n = 1): the
    product's host semantics, no kernel backend, byte-equal to micro_n1.npz."""
    g = load_npz("micro_n1.npz")
    rec = _run("dropin_host", 1)[0]
    for s in (1, 2):
        assert rec[f"delta_s{s}"].tobytes() == g[f"delta_s{s}_r0"].tobytes()
        assert rec[f"avg_s{s}"].tobytes() == g[f"delta_s{s}_r0"].tobytes()  # n = 1: no sync
        for k in ("theta", "buf"):
            assert rec[f"{k}_s{s}"].tobytes() == g[f"{k}_s{s}"].tobytes(), (k, s)
        assert rec[f"inner_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()


def test_sync_outputs_aggregates_like_reference():
    recs = _run("outputs", 2)
    # tokens: 100+200; micro batches: ignore 0 -> 1; time mean(1,2); loss ignores 0 -> 2.0;
    # norm mean(0.5, 0.5)
    assert recs[0]["agg"].tolist() == [300, 1, 1.5, 2.0, 0.5]
    assert recs[1]["agg"].tolist() == recs[0]["agg"].tolist()


@pytest.mark.parametrize("world", [2, 4])
def test_int8_wire_exchange_matches_oracle(world):
    """all_to_all -> rank-order reduce -> all_gather over a real process group: every replica
    ends bit-identical to the oracle's restatement of the codec (deterministic at any n)."""
    exp = expected_q8(world)
    for rec in _run("engine_q8", world):
        for s in (1, 2):
            assert rec[f"theta_s{s}"].tobytes() == exp[f"theta_s{s}"].tobytes(), s
            assert rec[f"inner_s{s}"].tobytes() == exp[f"theta_s{s}"].tobytes(), s
    # and the codec is close to the exact fp32 average
    g = load_npz(f"micro_n{world}.npz")
    err = np.abs(exp["theta_s1"] - g["theta_s1"]).max() / np.abs(g["theta_s1"] - g["theta0"]).max()
    assert err < 2e-2


@pytest.mark.parametrize("world", [4, 8])
def test_a2a_exchange_is_bit_exact_against_rank_order_oracle(world):
    """exchange="a2a" over a real process group: the all_to_all hands every peer the n copies
    of its shard and the reduce sums them in rank order, so every replica ends bit-identical
    to the oracle's rank-order restatement at any n (the reduce-scatter's sum order is the
    transport's, normwise only) -- and still within 1e-6 normwise of the reference's gloo run."""
    from diloco_amd.trees import get_tree

    exp = expected_rank_order(world)
    recs = _run("engine_a2a", world)
    for rec in recs:
        for s in (1, 2):
            for k in ("theta", "buf"):
                assert rec[f"{k}_s{s}"].tobytes() == exp[f"{k}_s{s}"].tobytes(), (k, s)
            assert rec[f"inner_s{s}"].tobytes() == exp[f"theta_s{s}"].tobytes(), s
    numels = get_tree("micro").numels()
    g = load_npz(f"micro_n{world}.npz")
    for s in (1, 2):
        for a, b in zip(split(exp[f"theta_s{s}"], numels), split(g[f"theta_s{s}"], numels)):
            assert normwise_ok(a, b, 1e-6), s


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gradsync_a2a_is_bit_exact_against_rank_order_oracle(world):
    """GradSync(exchange="a2a"): all_to_all -> rank-order average -> all_gather; every rank's
    grads end equal to oracle.sum_avg of all ranks' grads, bit for bit, at any n."""
    from oracle import oracle

    sizes = (1, 3, 5000, 64, 4097)
    grads = []
    for r in range(world):
        g = torch.Generator().manual_seed(100 + r)
        grads.append(np.concatenate([torch.randn(n, generator=g).numpy() for n in sizes]))
    want = oracle.sum_avg(grads)
    for rec in _run("gradsync_a2a", world):
        assert rec["got"].tobytes() == want.tobytes()
    if world == 4:  # the same through TrainingComm.sync_gradients (DILOCO_DP_EXCHANGE=a2a)
        for rec in _run("dpsync_a2a", world):
            assert rec["got"].tobytes() == want.tobytes()


@pytest.mark.parametrize("mode", ["dropin_device_bf16", "dropin_device_bf16_eager"])
def test_dropin_device_bf16_wire_two_peers(mode):
    """BASELINE config #5 behind the reference's calls (get_outer_model(..., wire="bf16")): the
    deltas cross the DP exchange in bf16 and the SGD reads them from the wire. Two peers,
    2 outer steps, fused (nothing read between the calls) and eager: θ, momentum, the inner
    params and .grad (the codec's decoded average) bit-exact against the restatement of the
    codec (tests/expect.expected_bf16_allreduce), every replica identical."""
    exp = expected_bf16_allreduce(2)
    recs = _run(mode, 2)
    for rec in recs:
        for s in (1, 2):
            for k in ("theta", "buf", "avg"):
                assert rec[f"{k}_s{s}"].tobytes() == exp[f"{k}_s{s}"].tobytes(), (mode, k, s)
            assert rec[f"inner_s{s}"].tobytes() == exp[f"theta_s{s}"].tobytes(), (mode, s)


@pytest.mark.parametrize("mode", ["dropin_device_int8", "dropin_device_int8_eager",
                                  "dropin_int8"])
@pytest.mark.parametrize("world", [2, 4])
def test_dropin_int8_wire_matches_codec_restatement(mode, world):
    """The int8 wire behind the reference's calls (get_outer_model(..., wire="int8"), SURVEY
    §8f row 4): per bucket dl_delta_q8 -> all_to_all -> dl_q8_reduce (rank order) ->
    all_gather, the SGD reading the averaged slots (fused) or the decoded .grad (eager); the
    device placement and the default host placement. .grad (the decoded average), θ, the
    momentum and the inner params bit-identical to the oracle's restatement of the codec
    (tests/expect.expected_q8) at 2 and 4 peers, in several buckets."""
    exp = expected_q8(world)
    for rec in _run(mode, world):
        for s in (1, 2):
            for k in ("theta", "buf", "avg"):
                assert rec[f"{k}_s{s}"].tobytes() == exp[f"{k}_s{s}"].tobytes(), (mode, k, s)
            assert rec[f"inner_s{s}"].tobytes() == exp[f"theta_s{s}"].tobytes(), (mode, s)


@pytest.mark.parametrize("mode", ["adamw_lazy", "adamw_device"])
@pytest.mark.parametrize("world", [2, 3])
def test_dropin_adamw_outer_optimizer_on_the_sharded_exchange(mode, world):
    """An AdamW outer optimizer (the reference's get_optimizer allows it, src/utils.py:60-61)
    on the default lazy host and the device outer model, several buckets: three outer steps
    against the reference's calls on a plain deepcopy outer model in the same process, byte for
    byte -- at 2 peers the default sharded exchange against per-tensor all_reduce / n; at 3
    the rank-order exchange (DILOCO_DP_EXCHANGE=a2a) against a rank-order fp32 sum / n, since
    AdamW's g / sqrt(v) turns any change of summation order into O(lr) differences where g
    nearly cancels. θ equal across ranks and to the inner params."""
    recs = _run(mode, world)
    for rec in recs:
        for s in (1, 2, 3):
            assert rec[f"inner_s{s}"].tobytes() == rec[f"theta_s{s}"].tobytes(), (mode, s)
            assert rec[f"theta_s{s}"].tobytes() == recs[0][f"theta_s{s}"].tobytes(), (mode, s)
            for k in ("theta", "avg", "exp_avg_sq"):
                assert rec[f"{k}_s{s}"].tobytes() == rec[f"ref_{k}_s{s}"].tobytes(), (mode, k, s)
