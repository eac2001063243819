"""The drop-in surface on the GPU: the reference's call sequence of src/train.py:261-269 with
diloco_amd's get_outer_model / compute_pseudo_gradient / TrainingComm.sync_gradients /
get_optimizer(...).step() / sync_inner_model, HIP kernels underneath, compared bit-exact with
the reference's own outputs (tests/golden/micro_n{1,2}.npz).

Two-peer cases run two processes on the one GPU of the box. RCCL refuses two ranks on one
device, so these use a gloo DP group on the device tensors (DILOCO_DP_BACKEND=gloo); the
kernels are the product's HIP kernels. The RCCL transport itself runs in bench.py at N > 1.
"""
import os
import socket
import sys
import tempfile
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO, inner_tree_device_verified, load_json, load_npz
from conftest import spin as conftest_spin
from gpu_platform import gpu_state as _gpu_state

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Cfg:
    def __init__(self, **kw):
        self.__dict__.update(kw)


SGD_CFG = _Cfg(type="SGD", lr=0.7, momentum=0.9, nesterov=True)


def _module(values, shapes, device):
    m = torch.nn.Module()
    m.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.from_numpy(v.copy()).view(s))
                                   for v, s in zip(values, shapes)])
    return m.to(device)


def _flat(ts):
    return np.concatenate([t.detach().cpu().numpy().reshape(-1) for t in ts])


def _outer_steps(rank, n, steps=2, stock_sgd=False, host_shift=0.0, placement=None,
                 write_back=None, quiet=False, fused=None, wire=None, spin=0, exchange=None):
    """The reference's outer step sequence with the drop-in functions (this process = DP
    rank `rank` of `n`; the default process group must exist). quiet: nothing is read between
    the four calls (src/train.py:261-269 reads nothing), so a fused device outer model defers
    the delta and the /n into its one SGD pass; the values are read after sync_inner_model.
    spin: a slow producer -- a spin kernel of that many ms queued on the caller's stream
    right before sync_gradients, so every bucket's pack (and with it the data each collective
    reads) is still far from done when the collectives are issued."""
    from diloco_amd import synth
    from diloco_amd.comm import TrainingComm
    from diloco_amd.trees import get_tree
    from diloco_amd.utils import (compute_pseudo_gradient, flush_outer_model, get_optimizer,
                                  get_outer_model, sync_inner_model)
    from diloco_amd.world import World

    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    inner = _module(synth.outer_tree(spec.numels(), spec.init_spec()), shapes, "cpu")
    # src/train.py:382: before the inner model moves
    outer = get_outer_model(inner, placement, write_back=write_back, fused=fused, wire=wire,
                            exchange=exchange)
    deferred = write_back == "deferred"
    inner = inner.to("cuda:0")
    if placement == "device":
        # built while the inner model was on the CPU: the outer model waits for the first
        # compute_pseudo_gradient to name its device (never the current device, which the
        # reference does not set); the optimizer below is built on these very Parameters
        assert not any(p.is_cuda for p in outer.parameters())
    if stock_sgd:
        opt = torch.optim.SGD(outer.parameters(), lr=0.7, momentum=0.9, nesterov=True)
    else:
        opt = get_optimizer(outer, SGD_CFG)
        assert type(opt).__name__ == "OuterSGD"
    comm = TrainingComm(World.from_default_group(1), (1, 1, 32), None)
    rec = {}
    for s in range(1, steps + 1):
        prev = [p.detach().cpu().numpy().reshape(-1).copy() for p in outer.parameters()]
        vals = synth.inner_tree(prev, s, rank)
        with torch.no_grad():
            for p, v in zip(inner.parameters(), vals):
                p.copy_(torch.from_numpy(v).view(p.shape))
        # deferred write-back: outer step 1 flushes after every call, step 2 reads the host
        # tensors only after sync_inner_model's write-back (waited for by the flush)
        mid = not quiet and (not deferred or s == 1)
        compute_pseudo_gradient(inner, outer)
        if placement == "device":  # the same Parameter objects, now in the inner model's HBM
            assert all(p.device == torch.device("cuda", 0) for p in outer.parameters())
            assert all(map(lambda a, b: a is b, opt.param_groups[0]["params"],
                           outer.parameters()))
        if spin:
            conftest_spin(spin)
        t_sync = time.perf_counter()
        if deferred and mid:
            flush_outer_model(outer)
        if mid:
            rec[f"delta_s{s}"] = _flat(p.grad for p in outer.parameters())
        comm.sync_gradients(outer)
        if spin:  # host time of the call that issued every bucket's collective
            rec[f"sync_host_ms_s{s}"] = np.float64((time.perf_counter() - t_sync) * 1e3)
        if deferred and mid:
            flush_outer_model(outer)
        if mid:
            rec[f"avg_s{s}"] = _flat(p.grad for p in outer.parameters())
        opt.step()
        if deferred and mid:
            flush_outer_model(outer)
        if mid:
            rec[f"theta_s{s}"] = _flat(outer.parameters())
            rec[f"buf_s{s}"] = _flat(opt.state[p]["momentum_buffer"] for p in outer.parameters())
        sync_inner_model(outer, inner)
        if not mid:
            if deferred:  # quiet: reading .grad completes the fused model's pending work
                flush_outer_model(outer)
            rec[f"delta_s{s}"] = rec[f"avg_s{s}"] = _flat(p.grad for p in outer.parameters())
            rec[f"theta_s{s}"] = _flat(outer.parameters())
            rec[f"buf_s{s}"] = _flat(opt.state[p]["momentum_buffer"] for p in outer.parameters())
        torch.cuda.synchronize()
        rec[f"inner_s{s}"] = _flat(inner.parameters())
        if host_shift and s == 1:
            # a host-side in-place update between outer steps must reach the device mirror
            with torch.no_grad():
                for p in outer.parameters():
                    p.add_(host_shift)
    return rec


def _init_single():
    if not dist.is_initialized():
        f = tempfile.mktemp(prefix="dl_pg_")
        dist.init_process_group("gloo", init_method=f"file://{f}", rank=0, world_size=1)


@pytest.mark.parametrize("stock_sgd,placement,write_back,quiet,fused", [
    (False, "host", "sync", False, None), (True, "host", "sync", False, None),
    (False, "device", "sync", False, True), (False, "device", "sync", True, True),
    (False, "device", "sync", False, False), (True, "device", "sync", True, True),
    (False, "host", "deferred", False, None), (False, "host", "lazy", False, None),
    (False, "host", "lazy", True, None), (True, "host", "lazy", True, None),
    (False, "host", "lazy", True, False)])
def test_dropin_single_peer_matches_reference(stock_sgd, placement, write_back, quiet, fused):
    """The reference's call sequence, outer model on the host (its placement) or in HBM
    (placement="device"); torch's own CPU SGD on the host outer model as
    well (the mirror must see its in-place updates); the host placement with the deferred
    write-back (side-stream DMAs issued by sync_inner_model) and with the lazy one (the
    default: the step on the HBM twin, host tensors refreshed when read)."""
    _init_single()
    g = load_npz("micro_n1.npz")
    rec = _outer_steps(0, 1, stock_sgd=stock_sgd, placement=placement, write_back=write_back,
                       quiet=quiet, fused=fused)
    for s in (1, 2):
        assert rec[f"delta_s{s}"].tobytes() == g[f"delta_s{s}_r0"].tobytes()
        assert rec[f"avg_s{s}"].tobytes() == g[f"delta_s{s}_r0"].tobytes()  # n=1: no sync
        assert rec[f"theta_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()
        assert rec[f"buf_s{s}"].tobytes() == g[f"buf_s{s}"].tobytes()
        assert rec[f"inner_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()


def test_dropin_host_writes_are_seen_by_the_device_mirror():
    """θ_outer changed on the host between outer steps (version counter bump) -> re-upload."""
    from conftest import split
    from diloco_amd import synth
    from diloco_amd.trees import get_tree
    from oracle import oracle

    _init_single()
    g = load_npz("micro_n1.npz")
    rec = _outer_steps(0, 1, host_shift=0.25)
    numels = get_tree("micro").numels()
    st = oracle.OuterState([(t + np.float32(0.25)).astype(np.float32)
                            for t in split(g["theta_s1"], numels)])
    st.buf = [b.copy() for b in split(g["buf_s1"], numels)]
    st.steps = 1
    st.step([synth.inner_tree(st.theta, 2, 0)])
    assert rec["theta_s2"].tobytes() == np.concatenate(st.theta).tobytes()
    assert rec["inner_s2"].tobytes() == np.concatenate(st.theta).tobytes()


@pytest.mark.parametrize("pin", [False, True])
def test_outer_params_stay_host_tensors_with_reference_layout(pin, monkeypatch):
    """The default host outer model keeps CPU tensors of the reference's shapes; its arenas
    are pageable (as the reference's deepcopy(inner).to("cpu") is) unless DILOCO_HOST_PIN=1."""
    from diloco_amd import synth
    from diloco_amd.trees import get_tree
    from diloco_amd.utils import compute_pseudo_gradient, get_outer_model

    monkeypatch.setenv("DILOCO_HOST_PIN", "1" if pin else "0")
    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    inner = _module(synth.outer_tree(spec.numels(), spec.init_spec()), shapes, "cpu")
    outer = get_outer_model(inner)
    inner = inner.to("cuda:0")
    compute_pseudo_gradient(inner, outer)
    for p, q in zip(outer.parameters(), inner.parameters()):
        assert p.device.type == "cpu" and p.grad.device.type == "cpu"
        assert p.shape == q.shape and p.grad.shape == q.shape
        assert p.is_pinned() == pin


def _worker(rank, world, port, mode, out):
    for p in (PKG, REPO, os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["DILOCO_DP_BACKEND"] = "gloo"
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    rec = {}
    if mode in ("dropin", "dropin_device", "dropin_deferred", "dropin_device_quiet",
                "dropin_device_bf16", "dropin_device_quiet_buckets", "dropin_quiet_buckets",
                "dropin_sync", "dropin_device_int8", "dropin_int8",
                "dropin_quiet_buckets_sharded"):
        if "_quiet_buckets" in mode or "int8" in mode:  # several buckets: bucket b's
            os.environ["DILOCO_OUTER_BUCKET_ELEMS"] = "4096"  # waits for b's collective only
        rec = _outer_steps(rank, world,
                           placement="device" if mode.startswith("dropin_device") else None,
                           write_back="deferred" if mode == "dropin_deferred" else
                           "sync" if mode == "dropin_sync" else None,
                           quiet=mode in ("dropin_device_quiet", "dropin_device_bf16",
                                          "dropin_device_quiet_buckets", "dropin_quiet_buckets",
                                          "dropin_device_int8", "dropin_quiet_buckets_sharded"),
                           exchange="sharded" if mode.endswith("_sharded") else None,
                           wire="bf16" if mode == "dropin_device_bf16" else
                           "int8" if "int8" in mode else None)
    elif mode.startswith("slow_producer"):
        # the reference's calls over two gloo processes with no host wait anywhere, every
        # bucket's collective issued while a spin kernel still holds the packs back on the
        # caller's stream; bucket b's SGD pass waits for bucket b's Work only.
        # "_unordered": the control -- the packs run on a side stream behind the spin, which
        # the collectives (ordered behind the caller's stream) do not wait for
        os.environ["DILOCO_OUTER_BUCKET_ELEMS"] = "4096"
        spin = 200  # ms
        if mode.endswith("_unordered"):
            from diloco_amd.kernels import default_kernels

            k = default_kernels()
            orig, side, held = k.delta_pack, torch.cuda.Stream(), [False]

            def delta_pack_on_side(*a):
                with torch.cuda.stream(side):
                    if not held[0]:
                        conftest_spin(spin)
                        held[0] = True
                    orig(*a)
            k.delta_pack = delta_pack_on_side
            spin = 0
        rec = _outer_steps(rank, world, placement="host" if "_host" in mode else "device",
                           quiet=True, spin=spin)
    elif mode in ("engine", "engine_ar"):
        from diloco_amd import synth
        from diloco_amd.outer import OuterSync
        from diloco_amd.trees import get_tree

        spec = get_tree("micro")
        shapes = [s for _, s in spec.params()]
        params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, "cuda:0"), shapes)]
        # engine: reduce-scatter -> shard SGD -> all-gather (the n > 1 default); engine_ar:
        # all-reduce -> full SGD on each replica
        eng = OuterSync(params, world_size=world, bucket_cap_elems=4096,
                        shard=None if mode == "engine" else False)
        assert eng.sharded == (mode == "engine")
        for s in (1, 2):
            th = [t.reshape(-1) for t in eng.unpacked(eng.theta)]
            synth.inner_tree_device(th, s, rank, out=[p.view(-1) for p in params])
            eng.step()
            torch.cuda.synchronize()
            rec[f"theta_s{s}"] = _flat(eng.unpacked(eng.theta))
            rec[f"buf_s{s}"] = _flat(eng.unpacked(eng.momentum_full()))
            rec[f"inner_s{s}"] = _flat(params)
    elif mode in ("engine_xgmi", "engine_xgmi_inner"):
        # the direct exchange: wires and θ IPC-mapped between the processes (same GPU here),
        # one dl_xgmi_reduce_sgd per rank between two barriers
        from diloco_amd import synth
        from diloco_amd.outer import OuterSync
        from diloco_amd.trees import get_tree

        spec = get_tree("micro")
        shapes = [s for _, s in spec.params()]
        params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, "cuda:0"), shapes)]
        exchange = "xgmi" if mode == "engine_xgmi" else "xgmi_inner"
        eng = OuterSync(params, world_size=world, bucket_cap_elems=4096, exchange=exchange)
        assert eng.xgmi and eng.tree.total % (64 * world) == 0
        if exchange == "xgmi_inner":  # the params now live in the arena the peers read
            base = eng.inner_arena.data_ptr()
            assert all(base <= p.data_ptr() < base + 4 * eng.tree.total for p in params)
        for s in (1, 2):
            th = [t.reshape(-1) for t in eng.unpacked(eng.theta)]
            synth.inner_tree_device(th, s, rank, out=[p.view(-1) for p in params])
            eng.step()
            torch.cuda.synchronize()
            rec[f"theta_s{s}"] = _flat(eng.unpacked(eng.theta))
            rec[f"buf_s{s}"] = _flat(eng.unpacked(eng.momentum_full()))
            rec[f"inner_s{s}"] = _flat(params)
        eng.close()
    elif mode == "p2p":
        # device p2p transport with HIP framing: stage 0 -> stage 1 forward,
        # replies backward; payload staged through host memory (gloo data groups: RCCL refuses
        # two ranks on one GPU)
        os.environ["DILOCO_P2P_BACKEND"] = "gloo"
        from diloco_amd.comm import TrainingComm
        from diloco_amd.world import World

        w = World.from_default_group(2)
        shape = (2, 16, 64)
        comm = TrainingComm(w, shape, None, transport="device", device=torch.device("cuda", 0))
        K = 4
        g = torch.Generator().manual_seed(5)
        payloads = [torch.randn(shape, generator=g) for _ in range(K)]
        if rank == 0:
            for i, t in enumerate(payloads):
                dt = torch.bfloat16 if i % 2 else torch.float32  # bf16 promotes to fp32
                comm.send_forward(t.to("cuda:0", dt), (7, i))
            back = [comm.recv_backward() for _ in range(K)]
            rec["back_src"] = np.array([b[0] for b in back])
            rec["back_meta"] = np.array([b[2] for b in back])
            rec["back"] = np.stack([b[1].detach().cpu().numpy() for b in back])
        else:
            fwd = [comm.recv_forward() for _ in range(K)]
            for src, t, meta in fwd:
                assert t.is_cuda and t.requires_grad and tuple(t.shape) == shape
                comm.send_backward(src, t.detach() * 3, meta)
            rec["fwd_src"] = np.array([f[0] for f in fwd])
            rec["fwd_meta"] = np.array([f[2] for f in fwd])
            rec["fwd"] = np.stack([f[1].detach().cpu().numpy() for f in fwd])
        rec["want"] = np.stack([(t.to(torch.bfloat16).float() if i % 2 else t).numpy()
                                for i, t in enumerate(payloads)])
        time.sleep(0.5)  # let the peer's last send complete before teardown
    elif mode == "dp":
        from diloco_amd.comm import TrainingComm
        from diloco_amd.world import World

        g = torch.Generator().manual_seed(100 + rank)
        m = torch.nn.Module()
        m.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.zeros(n)) for n in
                                       (1, 3, 5000, 64, 4097, 70000)]).to("cuda:0")
        for i, p in enumerate(m.parameters()):
            if i != 1:  # one missing gradient: zero-filled (src/comm.py:121)
                p.grad = torch.randn(p.numel(), generator=g).to("cuda:0")
        ref = [p.grad.clone() if p.grad is not None else torch.zeros_like(p)
               for p in m.parameters()]
        for r in ref:
            dist.all_reduce(r, op=dist.ReduceOp.SUM)
            r /= world
        TrainingComm(World.from_default_group(1), (1, 1, 4), None).sync_gradients(m)
        torch.cuda.synchronize()
        rec["got"] = _flat(p.grad for p in m.parameters())
        rec["ref"] = _flat(ref)
    elif mode == "dp_t125":
        # the per-step DP sync (src/train.py:249-251 -> src/comm.py:117-123) on device grads of
        # the full T125 shapes: GradSync (dl_gather -> all_reduce -> dl_unpack_avg, 256 MiB
        # buckets) against torch's own per-tensor all_reduce + /n of the same grads
        from diloco_amd import synth
        from diloco_amd.comm import TrainingComm
        from diloco_amd.trees import get_tree
        from diloco_amd.world import World

        spec = get_tree("t125")
        m = torch.nn.Module()
        m.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.zeros(sh, device="cuda:0"))
                                       for _, sh in spec.params()])
        grads = synth.inner_tree_device(synth.outer_tree_device(spec, "cuda:0"), 3, rank)
        for p, g in zip(m.parameters(), grads):
            p.grad = g.view(p.shape)
        ref = [p.grad.clone() for p in m.parameters()]
        for r in ref:
            dist.all_reduce(r, op=dist.ReduceOp.SUM)
            r /= world
        comm = TrainingComm(World.from_default_group(1), (1, 1, spec.n_embd), None)
        comm.sync_gradients(m)
        torch.cuda.synchronize()
        if world <= 2:
            bad = [i for i, (p, r) in enumerate(zip(m.parameters(), ref))
                   if not torch.equal(p.grad, r)]
        else:  # a bucket's all_reduce and a tensor's may add the peers in different orders
            from conftest import normwise_ok

            bad = [i for i, (p, r) in enumerate(zip(m.parameters(), ref))
                   if not normwise_ok(p.grad.cpu().numpy(), r.cpu().numpy(), 1e-6)]
        rec["bad"] = np.array(bad or [-1])
        rec["n"] = np.int64(len(ref))
    elif mode in ("adamw_lazy", "adamw_device"):
        rec = _adamw_outer_steps(rank, world, mode == "adamw_device")
    elif mode == "dropin_device_t13b_bf16_n8":
        rec = _bf16_dropin_codec_check(rank, world)
    elif mode in ("dropin_device_t125", "dropin_device_t125_bf16", "dropin_device_t13b",
                  "dropin_device_t13b_n8", "dropin_host_t125"):
        rec = _full_size_dropin_two_peers(rank, world,
                                          wire="bf16" if mode.endswith("bf16") else "f32",
                                          tree="t1.3b" if "t13b" in mode else "t125",
                                          placement="device" if "device" in mode else None)
    np.savez(os.path.join(out, f"{mode}_r{rank}.npz"), **rec)
    dist.barrier()
    dist.destroy_process_group()


def _adamw_outer_steps(rank, world, device, steps=3):
    """An AdamW outer optimizer (src/utils.py:60-61) through the four calls with the HIP
    kernels in several buckets (each placement's default exchange); beside it, in this process, the
    reference's calls on a plain deepcopy outer model with per-tensor all_reduce / n -- on the
    CPU as the reference places it, or in HBM beside the device placement (torch's AdamW
    rounds differently on the GPU, and that optimizer is torch's in both)."""
    import copy

    from diloco_amd import synth
    from diloco_amd.comm import TrainingComm
    from diloco_amd.trees import get_tree
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)
    from diloco_amd.world import World

    os.environ["DILOCO_OUTER_BUCKET_ELEMS"] = "4096"
    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    theta0 = synth.outer_tree(spec.numels(), spec.init_spec())
    inner = _module(theta0, shapes, "cpu")
    ref_outer = copy.deepcopy(inner).to("cuda:0" if device else "cpu")
    outer = get_outer_model(inner, "device" if device else None)
    inner = inner.to("cuda:0")
    ref_inner = copy.deepcopy(inner)
    cfg = _Cfg(type="AdamW", lr=0.01, weight_decay=0.1, betas=(0.9, 0.95))
    opt = get_optimizer(outer, cfg)
    assert type(opt) is torch.optim.AdamW
    # torch picks its single-tensor AdamW for the outer model's Parameter subclasses; on plain
    # device tensors it would pick the foreach form, which rounds differently
    ref_opt = torch.optim.AdamW(ref_outer.parameters(), lr=cfg.lr, betas=cfg.betas,
                                weight_decay=cfg.weight_decay, foreach=False)
    comm = TrainingComm(World.from_default_group(1), (1, 1, 32), None)
    rec = {}
    for s in range(1, steps + 1):
        vals = synth.inner_tree([p.detach().cpu().numpy().reshape(-1).copy()
                                 for p in ref_outer.parameters()], s, rank)
        with torch.no_grad():
            for p, q, v in zip(inner.parameters(), ref_inner.parameters(), vals):
                p.copy_(torch.from_numpy(v).view(p.shape))
                q.copy_(p)
        compute_pseudo_gradient(inner, outer)
        comm.sync_gradients(outer)
        opt.step()
        sync_inner_model(outer, inner)
        for po, pi in zip(ref_outer.parameters(), ref_inner.parameters()):  # src/utils.py:221
            po.grad = po.data - pi.data.to(po.device)
            dist.all_reduce(po.grad, op=dist.ReduceOp.SUM)  # src/comm.py:122-123
            po.grad /= world
        ref_opt.step()
        with torch.no_grad():
            for po, pi in zip(ref_outer.parameters(), ref_inner.parameters()):
                pi.copy_(po)
        torch.cuda.synchronize()
        rec[f"theta_s{s}"] = _flat(outer.parameters())
        rec[f"inner_s{s}"] = _flat(inner.parameters())
        rec[f"avg_s{s}"] = _flat(p.grad for p in outer.parameters())
        rec[f"exp_avg_sq_s{s}"] = _flat(opt.state[p]["exp_avg_sq"] for p in outer.parameters())
        rec[f"ref_theta_s{s}"] = _flat(ref_outer.parameters())
        rec[f"ref_avg_s{s}"] = _flat(p.grad for p in ref_outer.parameters())
        rec[f"ref_exp_avg_sq_s{s}"] = _flat(ref_opt.state[p]["exp_avg_sq"]
                                            for p in ref_outer.parameters())
    return rec


def _pack_probe(m, picks):
    """Snapshots of the packed wire over the sampled tensors, taken right after each bucket's
    pack on the same stream: this rank's own delta as it entered the exchange. Compared with
    the exact delta after the step, a mismatch localises a failure to the pack (inputs
    verified before it) rather than the exchange; it fails the test like any other (DESIGN
    §5)."""
    snaps = {}
    k = m.k
    orig = k.delta_pack

    def delta_pack(tree, b, slot, theta, wire):
        orig(tree, b, slot, theta, wire)
        if tree is not m.tree:
            return
        blo, bhi = tree.bucket_ranges[b] if b >= 0 else (0, tree.total)
        for t, lo, cnt in picks:
            o = m.offs[t] + lo
            if blo <= o < bhi:
                snaps[t] = wire[o:o + cnt].clone()
    k.delta_pack = delta_pack
    return snaps


def _lost_pack(snaps, t, own, bf16):
    """Elements of tensor t's packed own delta that differ from the exact one."""
    from oracle import oracle

    got = snaps[t].float().cpu().numpy() if bf16 else snaps[t].cpu().numpy()
    want = oracle.bf16_round(own) if bf16 else own
    return int(np.count_nonzero(got.view(np.int32) != np.asarray(want, np.float32).view(np.int32)))


def _bf16_dropin_codec_check(rank, world, steps=2, tree="t1.3b"):
    """Config #5 (1.3B, bf16 wire, SGD fused into the unpack) through the reference's four calls
    with `world` processes: the exchange's bf16 partial sums come in gloo's order, so instead of
    a bit pattern each outer step checks, on sampled tensors (a wte window, block 0, the last
    tensor) and from the θ / momentum the device held before the step, that (1) `.grad` (the
    decoded average) is within the codec's a-priori bound (diloco_amd.outer.bf16_codec_bound,
    replicated bf16 all-reduce in any order) of the fp32 average of the same deltas, and (2) θ,
    the momentum and the inner params are torch's SGD-Nesterov applied to exactly that `.grad`
    (bit-exact: the SGD pass consumes the decoded average). Returns mismatches, the worst
    error / bound and a digest of the values for the replicas to be compared bit for bit."""
    import hashlib

    from diloco_amd import synth
    from diloco_amd.comm import TrainingComm
    from diloco_amd.outer import bf16_codec_bound
    from diloco_amd.trees import get_tree
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)
    from diloco_amd.world import World
    from oracle import oracle
    from test_configs_gpu import _picks, _slice_inputs

    F32 = np.float32
    spec = get_tree(tree)
    picks = _picks(False, spec)
    shapes = [sh for _, sh in spec.params()]
    inner = torch.nn.Module()
    inner.ps = torch.nn.ParameterList(
        [torch.nn.Parameter(x.view(sh)) for x, sh in zip(synth.outer_tree_device(spec, "cuda:0"),
                                                          shapes)])
    outer = get_outer_model(inner, "device", wire="bf16")
    opt = get_optimizer(outer, SGD_CFG)
    comm = TrainingComm(World.from_default_group(1), (1, 1, spec.n_embd), None)
    snaps = _pack_probe(outer._diloco_mirror, picks)
    bad, worst, digest = [], 0.0, hashlib.sha256()
    lost = []
    ops, ips = list(outer.parameters()), list(inner.parameters())

    def window(x, t, lo, m):
        return x.detach().view(-1)[lo:lo + m].cpu().numpy()

    for s in range(1, steps + 1):
        before = {(t, lo): (window(ops[t], t, lo, m),
                            None if s == 1 else window(opt.state[ops[t]]["momentum_buffer"], t, lo, m))
                  for t, lo, m in picks}
        th = [p.detach().view(-1) for p in ops]
        inner_tree_device_verified(th, s, rank, [p.data.view(-1) for p in ips])
        compute_pseudo_gradient(inner, outer)
        comm.sync_gradients(outer)
        opt.step()
        sync_inner_model(outer, inner)
        torch.cuda.synchronize()
        for t, lo, m in picks:
            th0, buf0 = before[(t, lo)]
            d = [oracle.delta(th0, x) for x in _slice_inputs(t, lo, m, s, world, th0)]
            nl = _lost_pack(snaps, t, d[rank], True)
            if nl:
                lost.append((s, t, nl))
            g32 = oracle.sum_avg(d)
            bound = bf16_codec_bound(np.sum(np.abs(d), axis=0, dtype=np.float64), world,
                                     "rccl").astype(F32)
            g = window(ops[t].grad, t, lo, m)
            err = np.abs(g.astype(np.float64) - g32)
            if not np.all(err <= bound):
                i = int(np.argmax(err / np.maximum(bound, 1e-38)))
                over = np.flatnonzero(err > bound)
                # per bad element: the rank whose delta, left out, explains the sum
                gn = g.astype(np.float64) * world
                dd = np.stack(d).astype(np.float64)[:, over]
                miss = np.argmin(np.abs((dd.sum(0) - gn[over])[None, :] - dd), axis=0)
                runs = np.split(over, np.flatnonzero(np.diff(over) != 1) + 1)
                bad.append(f"step {s} tensor {t} codec bound: {over.size} of {m} elements, "
                           f"missing ranks {sorted(set(miss.tolist()))}, runs "
                           f"{[(int(lo + r[0]), int(r.size)) for r in runs[:6]]}"
                           f"{'...' if len(runs) > 6 else ''} ({len(runs)} runs); element "
                           f"{lo + i} g {g[i]!r} fp32 avg {g32[i]!r} bound {bound[i]!r}")
            worst = max(worst, float((err / np.maximum(bound, 1e-38)).max()))
            th_exp, buf_exp = th0.copy(), (np.empty_like(th0) if buf0 is None else buf0.copy())
            oracle.sgd(th_exp, buf_exp, g, 0.7, 0.9, True, s == 1)
            for k, got in (("theta", window(ops[t], t, lo, m)),
                           ("buf", window(opt.state[ops[t]]["momentum_buffer"], t, lo, m)),
                           ("inner", window(ips[t], t, lo, m))):
                digest.update(got.tobytes())
                want = buf_exp if k == "buf" else th_exp
                if got.tobytes() != want.tobytes():
                    bad.append(f"step {s} tensor {t} {k}")
            digest.update(g.tobytes())
    return {"bad": np.array(bad or ["none"]), "checked": np.int64(len(picks) * steps),
            "worst": np.float64(worst), "digest": np.array(digest.hexdigest()),
            "lost_pack": np.array(lost or [(-1, -1, 0)]), "gpu": np.array(repr(_gpu_state()))}


def _full_size_dropin_two_peers(rank, world, steps=2, wire="f32", tree="t125",
                                placement="device"):
    """This process = DP rank `rank` of `world` on a full tree (T125, or T1.3B in 25 buckets):
    the reference's four calls (src/train.py:263-269, nothing read in between) on the fused
    device outer model, the exchange over the gloo DP group in 256 MiB buckets. Checked in the
    worker against the C oracle on sampled tensors (wte whole on T125, a 4 Mi-element window of
    it on T1.3B, the first block, the last tensor): θ, the momentum,
    the inner params and `.grad` (the average) after each outer step; returns the mismatches.
    Bit-exact at two peers; beyond, gloo's summation order differs from the oracle's rank
    order, so per tensor |got - oracle| <= 1e-6 * max|oracle|, and every rank's
    values are returned as a digest for the replicas to be compared bit for bit.
    wire="bf16" (config #5's codec behind the same calls): the oracle's restatement of the
    codec -- each delta rounded to bf16 (RNE), the partial sums rounded to bf16 in rank order,
    the average = sum / n in fp32. placement=None: get_outer_model's default -- the reference's
    CPU outer model stepped on its HBM twin (write_back="lazy"); θ, .grad and the momentum are
    then read as the CPU tensors the reference holds."""
    from diloco_amd import synth
    from diloco_amd.comm import TrainingComm
    from diloco_amd.trees import get_tree
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)
    from diloco_amd.world import World
    from oracle import oracle
    import hashlib

    from conftest import normwise_ok
    from test_configs_gpu import _picks, _slice_inputs

    F32 = np.float32
    spec = get_tree(tree)
    picks = _picks(tree == "t125", spec)
    init = spec.init_spec()
    exp = {}
    for t, lo, m in picks:  # the oracle on the sampled tensors: θ, buf and g per step
        b, sc = init[t]
        th = (F32(b) + synth.uniform(synth.OUTER_SEED, t, m, start=lo) * F32(sc)).astype(F32)
        buf = np.empty_like(th)
        for s in range(1, steps + 1):
            d = [oracle.delta(th, x) for x in _slice_inputs(t, lo, m, s, world, th)]
            if wire == "bf16":
                acc = oracle.bf16_round(d[0])
                for dr in d[1:]:
                    acc = oracle.bf16_round((acc + oracle.bf16_round(dr)).astype(F32))
                g = (acc / F32(world)).astype(F32)
            else:
                g = oracle.sum_avg(d)
            oracle.sgd(th, buf, g, 0.7, 0.9, True, s == 1)
            exp[(t, s)] = (th.copy(), buf.copy(), g)
    shapes = [sh for _, sh in spec.params()]
    inner = torch.nn.Module()
    inner.ps = torch.nn.ParameterList(
        [torch.nn.Parameter(x.view(sh)) for x, sh in zip(synth.outer_tree_device(spec, "cuda:0"),
                                                          shapes)])
    outer = get_outer_model(inner, placement, wire=wire)  # fused (the default)
    dm = getattr(outer._diloco_mirror, "dev", outer._diloco_mirror)  # the lazy host's HBM twin
    assert dm.fused
    assert dm.tree.n_buckets == (25 if tree == "t1.3b" else 2)
    if placement is None:
        assert all(p.device.type == "cpu" for p in outer.parameters())
    opt = get_optimizer(outer, SGD_CFG)
    comm = TrainingComm(World.from_default_group(1), (1, 1, spec.n_embd), None)
    snaps = _pack_probe(dm, picks)
    bad, lost = [], []
    digest = hashlib.sha256()
    for s in range(1, steps + 1):
        # this rank's own delta as the pack must produce it, from the θ the device holds before
        # the step (beyond two peers θ differs from the oracle's rank-order chain in the last
        # bits -- gloo's sum order -- so the chain's delta is not the pack's bit pattern)
        own = {t: oracle.delta(th0, _slice_inputs(t, lo, m, s, world, th0)[rank])
               for t, lo, m in picks
               for th0 in [list(outer.parameters())[t].detach().view(-1)[lo:lo + m].cpu().numpy()]}
        # θ on the device (the default placement's outer parameters are CPU tensors)
        th = [p.detach().view(-1).to("cuda:0") for p in outer.parameters()]
        inner_tree_device_verified(th, s, rank, [p.data.view(-1) for p in inner.parameters()])
        del th
        compute_pseudo_gradient(inner, outer)
        comm.sync_gradients(outer)
        opt.step()
        sync_inner_model(outer, inner)
        torch.cuda.synchronize()
        ops, ips = list(outer.parameters()), list(inner.parameters())
        for t, lo, m in picks:
            nl = _lost_pack(snaps, t, own[t], wire == "bf16")
            if nl:
                lost.append((s, t, nl))
            want_th, want_buf, want_g = exp[(t, s)]
            got = {"theta": ops[t].detach().view(-1)[lo:lo + m],
                   "buf": opt.state[ops[t]]["momentum_buffer"].view(-1)[lo:lo + m],
                   "inner": ips[t].detach().view(-1)[lo:lo + m],
                   "grad": ops[t].grad.view(-1)[lo:lo + m]}
            for k, want in (("theta", want_th), ("buf", want_buf), ("inner", want_th),
                            ("grad", want_g)):
                g = got[k].cpu().numpy()
                digest.update(g.tobytes())
                ok = (g.tobytes() == want.tobytes() if world <= 2
                      else normwise_ok(g, want, 1e-6))
                if not ok:
                    bad.append(f"step {s} tensor {t} {k}")
    return {"bad": np.array(bad or ["none"]), "checked": np.int64(len(picks) * steps),
            "digest": np.array(digest.hexdigest()),
            "lost_pack": np.array(lost or [(-1, -1, 0)]), "gpu": np.array(repr(_gpu_state()))}


# Hardware queues per rank process when eight ranks share the one GPU: each process's queues
# (torch's streams up to GPU_MAX_HW_QUEUES, gloo's high-priority copy stream, one more) enter
# the firmware scheduler's runlist, which has num_cp_queues = 24 slots. At the default 4 the
# eight ranks hold 48 and the scheduler time-slices them, remapping processes to new VMIDs
# mid-step; at 1 they hold 24 and no remap happens (profiles/r06_platform_probes.txt
# I / J). One process per GPU, the product's shape, holds at most 6.
EIGHT_PEER_HW_QUEUES = "1"


def _run(mode, world=2):  # noqa: D401
    out = tempfile.mkdtemp(prefix="dl_gpu_")
    prev = os.environ.get("GPU_MAX_HW_QUEUES")
    if world > 2:  # the spawned ranks read it at their HIP initialisation
        os.environ["GPU_MAX_HW_QUEUES"] = EIGHT_PEER_HW_QUEUES
    try:
        mp.spawn(_worker, args=(world, _free_port(), mode, out), nprocs=world, join=True)
    finally:
        if prev is None:
            os.environ.pop("GPU_MAX_HW_QUEUES", None)
        else:
            os.environ["GPU_MAX_HW_QUEUES"] = prev
    return [dict(np.load(os.path.join(out, f"{mode}_r{r}.npz"))) for r in range(world)]


def _check_eight_peers(recs):
    """Config #4 / #5 with eight processes: every rank's checks clean, its own packed delta
    exact (a lost pack is a failure, not a retry), all replicas bit-identical."""
    info = [f"rank {r}: GPU state {str(rec.get('gpu', ''))}" for r, rec in enumerate(recs)]
    path = os.environ.get("DILOCO_TEST_RECORD")  # the record scripts keep the GPU's state
    if path:
        import json

        with open(path, "a") as f:
            f.write(json.dumps({"test": os.environ.get("PYTEST_CURRENT_TEST", ""),
                                "ranks": [str(rec.get("gpu", "")) for rec in recs]}) + "\n")
    for r, rec in enumerate(recs):
        assert rec["checked"] == 22
        assert int(rec["lost_pack"][0][0]) < 0, (r, rec["lost_pack"].tolist(), info)
        assert list(rec["bad"]) == ["none"], (r, list(rec["bad"])[:10], info)
    assert len({str(rec["digest"]) for rec in recs}) == 1


@pytest.mark.parametrize("mode", ["dropin", "dropin_device", "dropin_device_quiet",
                                  "dropin_device_quiet_buckets", "dropin_quiet_buckets",
                                  "dropin_quiet_buckets_sharded", "dropin_sync", "dropin_deferred",
                                  "engine", "engine_ar"])
def test_two_peers_on_gpu_match_reference(mode):
    """Two processes on the GPU, gloo DP group: dropin / dropin_quiet_buckets = the default
    placement (the CPU outer model on its HBM twin; its replicated exchange, several buckets in
    flight; _sharded: the opt-in sharded exchange on it), dropin_sync / dropin_deferred =
    host-authoritative write-backs, dropin_device* = the outer model in HBM (sharded by
    default); every value bit-exact vs the reference's 2-peer run."""
    g = load_npz("micro_n2.npz")
    for rec in _run(mode):
        for s in (1, 2):
            assert rec[f"theta_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes(), (mode, s)
            assert rec[f"buf_s{s}"].tobytes() == g[f"buf_s{s}"].tobytes(), (mode, s)
            assert rec[f"inner_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes(), (mode, s)
            if mode.startswith("dropin"):
                assert rec[f"avg_s{s}"].tobytes() == g[f"avg_s{s}"].tobytes()


@pytest.mark.parametrize("mode", ["slow_producer_device", "slow_producer_host",
                                  "slow_producer_unordered"])
def test_collectives_behind_a_slow_producer(mode):
    """Two processes, gloo DP group on the device tensors, no host synchronize anywhere: each
    step's packs queue behind a 200 ms spin kernel (dl_spin) while every bucket's collective
    (the device placement's reduce_scatter, the host placement's all_reduce) is issued --
    gloo's issuing call returns long
    before the spin ends, its staging copy ordered behind the caller's stream by an event
    (tools/gloo_sync_probe.py; `sync_host_ms_s*` records the issue time); the averages must be
    the reference's (micro_n2.npz, bit-exact), on both placements. The control runs the packs
    on a side stream the collectives are not ordered behind and must come out wrong: the
    producer side of the order is really exercised. (gloo's Work.wait() holds the host until
    the collective is done, where RCCL's only orders the stream: the consumer side is tested
    against a stream-ordered slow peer in tests/test_async_order_gpu.py.)"""
    recs = _run(mode)
    g = load_npz("micro_n2.npz")
    ok = all(recs[r][f"{k}_s{s}"].tobytes() == g[f"{k}_s{s}"].tobytes()
             for r in (0, 1) for s in (1, 2) for k in ("theta", "buf", "avg"))
    ok &= all(recs[r][f"inner_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()
              for r in (0, 1) for s in (1, 2))
    assert ok == (mode != "slow_producer_unordered"), mode
    if mode != "slow_producer_unordered":  # the calls returned before the producer finished
        assert all(float(recs[r][f"sync_host_ms_s{s}"]) < 150 for r in (0, 1) for s in (1, 2))


def test_t125_two_peers_dropin_device_bit_exact_vs_oracle():
    """BASELINE config #3 (T125, DP = 2, fp32) through the reference's own calls at full size:
    two processes, the fused device outer model (the bench's headline path at N > 1: per
    bucket dl_delta_pack -> all_reduce, then one dl_unpack_sgd pass with /n and the inner
    write), 2 outer steps. θ, momentum, inner and .grad bit-exact against the C oracle on wte
    (38.6 M elements, whole), the first block and the last tensor (src/comm.py:122-123,
    src/utils.py:221,226)."""
    for rec in _run("dropin_device_t125"):
        assert rec["checked"] == 22
        assert list(rec["bad"]) == ["none"], list(rec["bad"])[:10]


def test_t125_two_peers_dropin_default_placement_bit_exact_vs_oracle():
    """BASELINE config #3 on the outer model src/train.py gets: get_outer_model(inner) with
    its defaults (the CPU outer model, stepped on its HBM twin, its replicated exchange over
    the gloo DP group); θ, .grad and the momentum read as CPU tensors, and the inner params, bit-exact
    against the C oracle on the whole wte, block 0 and the last tensor after each of 2 steps."""
    recs = _run("dropin_host_t125")
    for r in recs:
        assert r["bad"].tolist() == ["none"], r["bad"][:8]
        assert int(r["checked"]) == 22
    assert recs[0]["digest"] == recs[1]["digest"]


def test_t125_two_peers_dp_grad_sync_matches_torch_all_reduce():
    """§8f row 1 at full T125 size, two processes: TrainingComm.sync_gradients on device grads
    (GradSync: dl_gather -> all_reduce per 256 MiB bucket -> dl_unpack_avg) equals torch's own
    per-tensor all_reduce(SUM) / n of the same grads, every one of the 148 tensors bit-exact."""
    for rec in _run("dp_t125"):
        assert rec["n"] == 148
        assert list(rec["bad"]) == [-1], list(rec["bad"])[:10]


def test_t125_eight_peers_dp_grad_sync_matches_torch_all_reduce():
    """The same with eight processes: every gradient within 1e-6 normwise of torch's own
    per-tensor all_reduce / n (the peers' summation order may differ between a 256 MiB bucket
    and a tensor)."""
    for rec in _run("dp_t125", 8):
        assert rec["n"] == 148
        assert list(rec["bad"]) == [-1], list(rec["bad"])[:10]


def test_t13b_two_peers_dropin_device_bit_exact_vs_oracle():
    """BASELINE config #4's 1.3B workload (25 buckets, each packed right before its collective,
    bucket b's SGD pass waiting for bucket b's exchange only) through the reference's four
    calls, two processes: θ, momentum, inner and .grad bit-exact against the C oracle on a wte
    window, block 0 and the last tensor after each of 2 outer steps."""
    for rec in _run("dropin_device_t13b"):
        assert rec["checked"] == 22
        assert list(rec["bad"]) == ["none"], list(rec["bad"])[:10]


def test_t13b_eight_peers_dropin_device_vs_oracle():
    """BASELINE config #4 itself (1.3B, DP = 8, 25 buckets pipelined) through the reference's
    four calls with eight processes on the one GPU (gloo DP group on the device tensors, ~21 GB
    of HBM each): θ, momentum, inner and .grad within 1e-6 normwise of the C oracle's
    rank-order result on a wte window, block 0 and the last tensor after each of 2 outer
    steps, and all eight replicas bit-identical."""
    _check_eight_peers(_run("dropin_device_t13b_n8", 8))


def test_t13b_eight_peers_dropin_device_bf16_wire_within_codec_bound():
    """BASELINE config #5 itself (1.3B, DP = 8, bf16 wire, SGD fused into the unpack) through
    the reference's four calls with eight processes on the one GPU: .grad within the codec's
    a-priori bound of the fp32 average, θ / momentum / inner exactly torch's SGD-Nesterov of
    that .grad, replicas bit-identical (see _bf16_dropin_codec_check)."""
    recs = _run("dropin_device_t13b_bf16_n8", 8)
    _check_eight_peers(recs)
    print(f"bf16 wire, 8 peers: worst codec error / bound {float(recs[0]['worst']):.3f}")


def test_t125_two_peers_dropin_device_bf16_wire_vs_codec_restatement():
    """BASELINE config #5's codec (bf16 wire, SGD fused into the unpack) through the
    reference's four calls at full T125 size, two processes: θ, momentum, inner and .grad (the
    decoded average) bit-exact against the oracle's restatement of the codec on wte (whole),
    block 0 and the last tensor after each of 2 outer steps."""
    for rec in _run("dropin_device_t125_bf16"):
        assert rec["checked"] == 22
        assert list(rec["bad"]) == ["none"], list(rec["bad"])[:10]


def test_two_peers_on_gpu_bf16_outer_wire():
    """Config #5's bf16 wire behind the reference's calls on the GPU (two processes, gloo DP
    group on device tensors): the HIP pack casts to bf16, the SGD pass reads the wire; θ,
    momentum, inner and .grad (decoded average) bit-exact against the codec's restatement."""
    from expect import expected_bf16_allreduce

    exp = expected_bf16_allreduce(2)
    for rec in _run("dropin_device_bf16"):
        for s in (1, 2):
            assert rec[f"theta_s{s}"].tobytes() == exp[f"theta_s{s}"].tobytes(), s
            assert rec[f"buf_s{s}"].tobytes() == exp[f"buf_s{s}"].tobytes(), s
            assert rec[f"avg_s{s}"].tobytes() == exp[f"avg_s{s}"].tobytes(), s
            assert rec[f"inner_s{s}"].tobytes() == exp[f"theta_s{s}"].tobytes(), s


@pytest.mark.parametrize("exchange", ["xgmi", "xgmi_inner"])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_direct_exchange_between_processes(world, exchange):
    """exchange='xgmi' (peers' wires) and 'xgmi_inner' (peers' inner arenas, no wire) with
    `world` processes on the one GPU (IPC between processes of one device; across devices the
    same code reads over xGMI): every replica equals the oracle's rank-order sum + SGD
    bit-exact at any n, and the reference bit-exact at n = 2, normwise at n = 4, 8."""
    from diloco_amd import synth
    from diloco_amd.trees import get_tree
    from oracle import oracle

    recs = _run(f"engine_{exchange}", world)
    spec = get_tree("micro")
    st = oracle.OuterState(synth.outer_tree(spec.numels(), spec.init_spec()))
    for s in (1, 2):
        st.step([synth.inner_tree(st.theta, s, r) for r in range(world)])
        want_th = np.concatenate(st.theta)
        want_buf = np.concatenate(st.buf)
        for rec in recs:
            assert rec[f"theta_s{s}"].tobytes() == want_th.tobytes(), s
            assert rec[f"buf_s{s}"].tobytes() == want_buf.tobytes(), s
            assert rec[f"inner_s{s}"].tobytes() == want_th.tobytes(), s
        g = load_npz(f"micro_n{world}.npz")
        if world == 2:
            assert want_th.tobytes() == g[f"theta_s{s}"].tobytes()
        else:  # the reference's gloo sum order differs: normwise
            from conftest import normwise_ok, split

            for k, got in (("theta", want_th), ("buf", want_buf)):
                for a, b in zip(split(got, spec.numels()), split(g[f"{k}_s{s}"], spec.numels())):
                    assert normwise_ok(a, b, 1e-6), (k, s)


def test_device_p2p_transport_on_gpu():
    """HIP-framed activations through the device p2p transport, 2 ranks / 2 stages: payloads
    (fp32 and bf16-promoted) and metadata arrive intact, replies return to the sender."""
    r0, r1 = _run("p2p")
    want = r1["want"]
    assert r1["fwd_src"].tolist() == [0] * 4
    assert r1["fwd_meta"].tolist() == [[7, i] for i in range(4)]
    assert r1["fwd"].tobytes() == want.tobytes()
    assert r0["back_src"].tolist() == [1] * 4
    assert r0["back_meta"].tolist() == [[7, i] for i in range(4)]
    assert np.array_equal(r0["back"], want * 3)


def test_dp_sync_of_device_grads_two_peers():
    for rec in _run("dp"):
        assert rec["got"].tobytes() == rec["ref"].tobytes()


def test_serializer_matches_reference_fixture():
    from diloco_amd.serializer import Serializer

    for case in load_json("serializer.json"):
        dtype = getattr(torch, case["dtype"])
        x = torch.tensor(case["x"], dtype=torch.float32).to(dtype).view(case["shape"]).cuda()
        s = Serializer(tuple(case["shape"]))
        assert list(s.shape) == case["serializer_shape"]
        y = s.serialize(x, tuple(case["meta"]))
        assert list(y.shape) == case["out_shape"] and str(y.dtype).split(".")[-1] == case["out_dtype"]
        assert y[0].flatten()[:2].tolist() == case["meta_plane"]
        assert y[1].flatten().tolist() == case["payload"]
        t, m = s.deserialize(y)
        assert list(t.shape) == case["deser_shape"] and list(m) == case["deser_meta"]
        assert torch.equal(t, y[1])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64])
def test_serializer_device_frame_keeps_autograd_and_promotes_like_cat(dtype):
    """src/serializer.py:15 is torch.cat([meta_plane, tensor]): the frame's dtype is the
    promotion of fp32 with the payload's (fp64 stays fp64) and it keeps the payload's graph.
    The HIP frame equals the host restatement of that cat bit for bit and backpropagates
    plane 1's gradient to the payload in its own dtype."""
    from diloco_amd.serializer import Serializer

    g = torch.Generator().manual_seed(11)
    x0 = torch.randn(3, 5, 7, generator=g, dtype=torch.float64).to(dtype)
    x = x0.clone().cuda().requires_grad_(True)
    s = Serializer((3, 5, 7))
    y = s.serialize(x, (3, 1 << 20))
    ref = Serializer._frame_host(x0, (3, 1 << 20))  # torch.stack/cat on the host
    assert y.is_cuda and y.dtype == ref.dtype == torch.promote_types(torch.float32, dtype)
    assert y.requires_grad and y.grad_fn is not None
    assert torch.equal(y[1].detach().cpu(), ref[1])
    assert y[0].flatten()[:2].tolist() == [3.0, float(1 << 20)]
    w = torch.randn(3, 5, 7, generator=g, dtype=torch.float64).to(y.dtype).cuda()
    (y[1] * w).sum().backward()
    assert x.grad.dtype == dtype and torch.equal(x.grad.cpu(), w.to(dtype).cpu())
    with torch.no_grad():
        assert s.serialize(x, (0, 1)).grad_fn is None


def test_serializer_errors_and_large_payload():
    from diloco_amd.serializer import Serializer

    s = Serializer((1,))
    with pytest.raises(IndexError):
        s.serialize(torch.ones(1, device="cuda"), (0, 1))
    y = Serializer((4,)).serialize(torch.arange(4.0), (0, 1))  # host tensor: framed on the host
    assert y.device.type == "cpu" and y[1].tolist() == [0.0, 1.0, 2.0, 3.0]
    x = torch.randn(32, 1024, 768, device="cuda")  # the experiment's (mbs, seq, n_embd)
    y = Serializer(tuple(x.shape)).serialize(x, (5, 7))
    assert torch.equal(y[1], x) and y[0].flatten()[:2].tolist() == [5.0, 7.0]
    xb = torch.randn(3, 1001, device="cuda").to(torch.bfloat16)
    yb = Serializer((3, 1001)).serialize(xb, (1, 2))
    assert torch.equal(yb[1], xb.float())


@pytest.mark.parametrize("placement", ["device", None])
def test_t125_fused_device_dropin_bit_exact_vs_oracle(placement):
    """The reference's four calls at full T125 size (148 tensors, 124,475,904 params) on the
    fused device outer model, and on the default outer model (the CPU outer model stepped on
    its HBM twin, write_back="lazy"), nothing read in between: each outer step is one
    dl_delta_pack_sgd and sync_inner_model a verified no-op. θ, momentum, .grad and the inner
    params bit-exact vs the C oracle on every tensor after each of 2 outer steps (for the
    default placement: read on the CPU, i.e. after the lazy copies from HBM)."""
    from diloco_amd import synth
    from diloco_amd.comm import TrainingComm
    from diloco_amd.trees import get_tree
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)
    from diloco_amd.world import World
    from oracle import oracle

    _init_single()
    spec = get_tree("t125")
    shapes = [s for _, s in spec.params()]
    inner = torch.nn.Module()
    inner.ps = torch.nn.ParameterList(
        [torch.nn.Parameter(t.view(s)) for t, s in zip(synth.outer_tree_device(spec, "cuda:0"),
                                                       shapes)])
    outer = get_outer_model(inner, placement)
    assert outer._diloco_mirror.fused
    assert all(p.device.type == ("cuda" if placement else "cpu") for p in outer.parameters())
    opt = get_optimizer(outer, SGD_CFG)
    comm = TrainingComm(World.from_default_group(1), (1, 1, spec.n_embd), None)
    st = oracle.OuterState([p.detach().cpu().numpy().reshape(-1) for p in outer.parameters()])
    for s in (1, 2):
        synth.inner_tree_device([p.detach().view(-1).to("cuda:0") for p in outer.parameters()],
                                s, 0, out=[p.data.view(-1) for p in inner.parameters()])
        compute_pseudo_gradient(inner, outer)
        comm.sync_gradients(outer)
        opt.step()
        sync_inner_model(outer, inner)
        torch.cuda.synchronize()
        inner_host = [synth.values(synth.noise_seed(s, 0), t, x.size, 0.0, synth.NOISE_SCALE, add=x)
                      for t, x in enumerate(st.theta)]
        delta = st.step([inner_host])[0][0]
        for t, (p, q) in enumerate(zip(outer.parameters(), inner.parameters())):
            th = p.detach().cpu().numpy().reshape(-1)
            assert th.tobytes() == st.theta[t].tobytes(), (s, t)
            assert q.detach().cpu().numpy().reshape(-1).tobytes() == st.theta[t].tobytes()
            buf = opt.state[p]["momentum_buffer"].cpu().numpy().reshape(-1)
            assert buf.tobytes() == st.buf[t].tobytes(), (s, t)
            assert p.grad.cpu().numpy().reshape(-1).tobytes() == delta[t].tobytes(), (s, t)


def test_t13b_fused_device_dropin_vs_oracle_on_sampled_tensors():
    """The reference's four calls at the 1.3B workload (292 tensors, 1,313,722,368 params) on
    the fused device outer model, one peer, 2 outer steps, nothing read in between: θ, the
    momentum, .grad and the inner params bit-exact vs the C oracle on a 4 Mi window of wte,
    block 0's tensors and the last tensor (every step is elementwise, so a window is
    restated exactly from the counter-based inputs)."""
    import gc

    from diloco_amd import synth
    from diloco_amd.trees import get_tree
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)
    from oracle import oracle

    spec = get_tree("t1.3b")
    numels, init = spec.numels(), spec.init_spec()
    picks = [(0, 37_000_011, 4 << 20)] + [(t, 0, numels[t]) for t in range(1, 10)] + [
        (len(numels) - 1, 0, numels[-1])]
    shapes = [s for _, s in spec.params()]
    inner = torch.nn.Module()
    inner.ps = torch.nn.ParameterList(
        [torch.nn.Parameter(t.view(s)) for t, s in zip(synth.outer_tree_device(spec, "cuda:0"),
                                                       shapes)])
    outer = get_outer_model(inner, "device")
    assert outer._diloco_mirror.fused and outer._diloco_mirror.tree.n_buckets == 25
    opt = get_optimizer(outer, SGD_CFG)
    F32 = np.float32
    exp = {}
    for t, lo, m in picks:
        b, sc = init[t]
        exp[t] = [(F32(b) + synth.uniform(synth.OUTER_SEED, t, m, start=lo) * F32(sc)).astype(F32),
                  np.empty(m, dtype=F32)]
    ps, qs = list(outer.parameters()), list(inner.parameters())
    for s in (1, 2):
        synth.inner_tree_device([p.detach().view(-1) for p in ps], s, 0,
                                out=[q.data.view(-1) for q in qs])
        compute_pseudo_gradient(inner, outer)
        opt.step()
        sync_inner_model(outer, inner)
        torch.cuda.synchronize()
        for t, lo, m in picks:
            th, buf = exp[t]
            x = (F32(0.0) + synth.uniform(synth.noise_seed(s, 0), t, m, start=lo)
                 * F32(synth.NOISE_SCALE) + th).astype(F32)
            g = oracle.delta(th, x)
            oracle.sgd(th, buf, g, 0.7, 0.9, True, s == 1)
            got = ps[t].detach().reshape(-1)[lo:lo + m].cpu().numpy()
            assert got.tobytes() == th.tobytes(), (s, t)
            assert qs[t].detach().reshape(-1)[lo:lo + m].cpu().numpy().tobytes() == th.tobytes()
            mb = opt.state[ps[t]]["momentum_buffer"].reshape(-1)[lo:lo + m].cpu().numpy()
            assert mb.tobytes() == buf.tobytes(), (s, t)
            assert ps[t].grad.reshape(-1)[lo:lo + m].cpu().numpy().tobytes() == g.tobytes()
    outer._diloco_mirror.close()
    del outer, inner, opt, ps, qs
    gc.collect()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("placement", ["device", None])
def test_outer_model_deepcopies_and_pickles_with_the_hip_library(placement):
    """an outer model whose mirror holds the HIP library's tree handle (a ctypes
    pointer) deep-copies and pickles: the mirror stays behind, the copy's parameters are plain
    Parameters holding the current values (the device placement and the default lazy host
    placement, after a fused outer step)."""
    import copy
    import io

    from diloco_amd import synth
    from diloco_amd.trees import get_tree
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)

    g = load_npz("micro_n1.npz")
    spec = get_tree("micro")
    shapes = [s for _, s in spec.params()]
    inner = _module(synth.outer_tree(spec.numels(), spec.init_spec()), shapes, "cuda:0")
    outer = get_outer_model(inner, placement)
    opt = get_optimizer(outer, SGD_CFG)
    vals = synth.inner_tree([p.detach().cpu().numpy().reshape(-1) for p in outer.parameters()],
                            1, 0)
    with torch.no_grad():
        for p, v in zip(inner.parameters(), vals):
            p.copy_(torch.from_numpy(v).view(p.shape))
    compute_pseudo_gradient(inner, outer)
    opt.step()
    sync_inner_model(outer, inner)
    c = copy.deepcopy(outer)
    assert getattr(c, "_diloco_mirror", None) is None
    assert all(type(p) is torch.nn.Parameter for p in c.parameters())
    assert _flat(c.parameters()).tobytes() == g["theta_s1"].tobytes()
    bio = io.BytesIO()
    torch.save(outer, bio)  # the whole module object, mirror attribute included
    bio.seek(0)
    d = torch.load(bio, weights_only=False)  # our own file, written just above
    assert getattr(d, "_diloco_mirror", None) is None
    assert _flat(d.parameters()).tobytes() == g["theta_s1"].tobytes()
    bio = io.BytesIO()
    torch.save(opt.state_dict(), bio)
    bio.seek(0)
    st = torch.load(bio, weights_only=True)["state"]
    assert _flat(st[i]["momentum_buffer"] for i in range(len(st))).tobytes() == g["buf_s1"].tobytes()


@pytest.mark.parametrize("mode", ["dropin_device_int8", "dropin_int8"])
def test_dropin_int8_wire_two_peers_on_gpu(mode):
    """The int8 wire behind the reference's calls on the GPU (two processes, gloo DP group,
    several buckets): the device placement with nothing read between the calls (the SGD reads
    the averaged slots, dl_unpack_sgd_q8) and the default host placement read after every
    call (the slots decoded into .grad). .grad, θ, momentum and the inner params bit-exact vs
    the oracle's restatement of the codec (tests/expect.expected_q8)."""
    from expect import expected_q8

    exp = expected_q8(2)
    for rec in _run(mode):
        for s in (1, 2):
            for k in ("theta", "buf", "avg"):
                assert rec[f"{k}_s{s}"].tobytes() == exp[f"{k}_s{s}"].tobytes(), (mode, k, s)
            assert rec[f"inner_s{s}"].tobytes() == exp[f"theta_s{s}"].tobytes(), (mode, s)


@pytest.mark.parametrize("mode", ["adamw_lazy", "adamw_device"])
def test_dropin_adamw_outer_optimizer_two_peers_on_gpu(mode):
    """An AdamW outer optimizer (src/utils.py:60-61) on the default lazy host and the device
    outer model with the HIP kernels: two processes, several buckets (the host placement's
    replicated exchange, the device placement's sharded one: AdamW reading the gathered .grad),
    AdamW writing θ in place; three outer steps byte-equal to
    the reference's calls on a plain deepcopy outer model (per-tensor all_reduce / n) on the
    same device as the outer model's parameters."""
    recs = _run(mode)
    for rec in recs:
        for s in (1, 2, 3):
            assert rec[f"inner_s{s}"].tobytes() == rec[f"theta_s{s}"].tobytes(), (mode, s)
            for k in ("theta", "avg", "exp_avg_sq"):
                got, want = rec[f"{k}_s{s}"], rec[f"ref_{k}_s{s}"]
                assert got.tobytes() == want.tobytes(), (
                    mode, k, s, int((got != want).sum()), float(np.abs(got - want).max()))
