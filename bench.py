#!/usr/bin/env python3
"""Benchmark: DiLoCo outer step, device-resident, GB/s of parameters reduced.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--tree t125]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

One step = one outer step of src/train.py:261-269 over the whole synthetic tree on every rank,
made through the reference's own calls -- compute_pseudo_gradient -> TrainingComm.sync_gradients
-> outer_optimizer.step() -> sync_inner_model (diloco_amd's drop-in modules, train.py untouched)
-- on the outer model get_outer_model(inner) returns with its defaults (the reference's CPU
outer model, stepped on its HBM twin):
    N = 1  one dl_delta_pack_sgd (outer.grad = θ_outer - inner, Nesterov SGD, inner = θ)
    N > 1  the default placement's replicated exchange (round 6: .grad and the momentum stay
           local on every rank, as in the reference): per bucket dl_delta_pack -> RCCL
           all_reduce, then per bucket dl_unpack_sgd (/n, Nesterov SGD, inner = θ); the opt-in
           sharded form (reduce_scatter -> dl_shard_sgd -> all_gather(θ)) is a side leg
Same tree per rank at every N (weak scaling). value = 4 * params / t_step ("GB/s
params reduced": the bytes of ONE parameter tree reduced per DP step, max time over ranks);
N * 4 * params / t_step is "value_aggregate".

Rank 0 prints ONE compact JSON line (<= 4 KB: the headline, its roofline kernel, the CPU
baseline, one-number summaries of the side legs, parity ok/err, the exchange efficiency at
N > 1) and writes every leg's full record to a side file (--detail, default
gpurun_out/bench_detail_n<N>.json). A watchdog bounds the run (--deadline): the line is printed
whatever a side leg does; a heartbeat on stderr names the running leg every 20 s. A/B-only
measurements (copy / mix ceilings, the two-kernel and wire-less steps, RCCL setting variants)
live in tools/bench_ab.py.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import platform
import subprocess
import sys
import threading
import time
from datetime import timedelta

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "diloco-swarm_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from diloco_amd import _lib, synth  # noqa: E402
from diloco_amd.outer import OuterSync  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402

METRIC = "GB/s params reduced (device-resident), DiLoCo outer step @1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
XGMI_LINK_GBS = 153.0       # per link per direction; busBW peak (n-1)*153
LINE_MAX_BYTES = 4096       # the driver parses one stdout line; everything else -> detail file


def log(msg):
    """One stderr line per call, written whole (ranks share the stream), rank-tagged at N > 1."""
    ws = os.environ.get("WORLD_SIZE", "1")
    tag = f"[bench r{os.environ.get('RANK', '0')}/{ws}]" if ws != "1" else "[bench]"
    sys.stderr.write(f"{tag} {msg}\n")
    sys.stderr.flush()


def load_pmc(tree):
    """Per-launch HBM bytes from the committed rocprofv3 counter passes of the same kernels
    (tools/gpu_pmc.sh -> profiles/rNN_pmc_<tree>.json, FETCH_SIZE x2 gfx950 correction)."""
    files = sorted(glob.glob(os.path.join(HERE, "profiles", f"r*_pmc_{tree}.json")))
    if not files:
        return {}
    with open(files[-1]) as f:
        d = json.load(f)
    return {k: v["hbm_bytes"] for k, v in d.get("kernels", {}).items()}


def setup_dist(n_gpus):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={ws}; launch N>1 with torchrun")
    # DILOCO_BENCH_BACKEND=gloo rehearses the N > 1 code path with several ranks on one GPU
    # (RCCL refuses two ranks per device): the DP group is then gloo too. The driver's
    # multi-GPU runs use RCCL for it.
    backend = os.environ.get("DILOCO_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local %= max(1, torch.cuda.device_count())
        # the drop-in legs' DP group too (comm.dp_backend() reads it when the group is made)
        os.environ.setdefault("DILOCO_DP_BACKEND", "gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if ws > 1:
        # the process groups src/train.py runs with: a gloo default group (src/world.py:32-33)
        # and, for every device collective, the DP group TrainingComm's DPSync creates over it
        # (an RCCL subgroup, use_local_synchronization=True; dp_group() below). A hung
        # collective becomes an error after 5 minutes instead of the 10-minute default.
        dist.init_process_group("gloo", timeout=timedelta(minutes=5))
    return ws, rank, dev


_COMM: dict = {}


def training_comm(n_embd=768):
    """The run's TrainingComm for activations of width n_embd (src/train.py:291 makes one per
    run, for its model's shape), over the default group. One per width -- the shape is the
    pipeline's activation shape -- all sharing the first one's DPSync, so every leg's DP
    collectives run on the one DP group (one RCCL communicator) of the run."""
    c = _COMM.get(n_embd)
    if c is None:
        from diloco_amd.comm import TrainingComm
        from diloco_amd.world import World

        c = TrainingComm(World.from_default_group(1), (1, 1, n_embd), None)
        first = next(iter(_COMM.values()), None)
        if first is not None:
            c.dp = first.dp
        _COMM[n_embd] = c
    return c


def dp_group(dev):
    """The group of every device collective in the bench at N > 1: DPSync.dp_group, exactly
    the group TrainingComm.sync_gradients reduces over in src/train.py's wiring. None at one
    rank (no collective is made)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return None
    return training_comm().dp.dp_group(dev)


def _max_over_ranks(x, dev, ws):
    if ws == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64)  # host value, the gloo default group
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _sync(ws):
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()


def kernel_entry(bytes_per_launch, ms, traffic=None, bound="hbm", peak=HBM_PEAK_GBS, **kw):
    """A roofline record: algorithmic bytes per launch over the average launch duration."""
    ach = bytes_per_launch / (ms * 1e-3) / 1e9
    e = {"bound": bound, "achieved": round(ach, 1), "peak": peak, "unit": "GB/s",
         "frac": round(ach / peak, 4), "traffic": round(traffic) if traffic else None,
         "bytes_per_launch": int(bytes_per_launch), "avg_ms": round(ms, 5)}
    e.update(kw)
    return e


SCRUB_MIB = 512  # >= 2 x the 256 MiB Infinity Cache moved per scrub (read 512 + write 512)


class Scrubber:
    """Evicts the step's bytes from the Infinity Cache (and every L2) between cold steps: a
    default-policy dl_copy of SCRUB_MIB MiB, enqueued outside the timed events. In training H
    inner steps run between two outer steps, so the cold figure is the one a DiLoCo run sees."""

    def __init__(self, dev):
        n = (SCRUB_MIB << 20) // 4
        self.a = torch.ones(n, device=dev)
        self.b = torch.empty(n, device=dev)
        self.s = torch.cuda.current_stream(dev).cuda_stream

    def __call__(self):
        _lib.call("dl_copy", self.a.data_ptr(), self.b.data_ptr(), self.a.numel() * 4, 0, self.s)
        self.a, self.b = self.b, self.a

    def close(self):
        del self.a, self.b


# ---- the drop-in outer step (the headline) ------------------------------------------------------
def dropin_bpp(ws, exchange, wire="f32"):
    """HBM bytes per parameter of the fused device drop-in step (kernels only; RCCL's own
    traffic not counted): one peer dl_delta_pack_sgd (read θ, inner, m; write wire, θ, m,
    inner) 28; N > 1 dl_delta_pack 12 (bf16 wire 10) + sharded dl_shard_sgd 20/n + dl_scatter
    8; a2a adds the rank-order reduce (reads n slices = 4, writes 4/n); replicated
    dl_unpack_sgd with the inner write 24 (bf16 wire 22)."""
    if ws == 1:
        return 28.0
    if wire == "int8":  # dl_delta_q8 8 + slot, dl_q8_reduce (n + 1)/n slots, dl_unpack_sgd_q8
        sb = 4160.0 / 4096  # one 4160-B slot per 4096-element chunk
        return 8 + sb + (ws + 1) * sb / ws + sb + 24.0
    wb = 2 if wire == "bf16" else 4
    if wire == "bf16" or exchange == "replicated":
        return 8 + wb + wb + 20.0
    if exchange == "a2a":
        return 12 + 4 + 4.0 / ws + 20.0 / ws + 8
    return 12 + 20.0 / ws + 8



def _dropin_objects(spec, dev, rank, wire, bucket_elems, exchange, placement=None):
    """The objects src/train.py builds for the outer step (train.py:375-421): an inner model on
    the GPU, get_outer_model(inner) -- by default the reference's host placement, stepped on an
    HBM twin (write_back="lazy") -- get_optimizer(outer, nesterov cfg), TrainingComm."""
    from types import SimpleNamespace

    from diloco_amd.utils import get_optimizer, get_outer_model

    if not dist.is_initialized():
        import tempfile

        dist.init_process_group("gloo", init_method="file://" + tempfile.mktemp(prefix="dlpg"),
                                rank=0, world_size=1)
    shapes = [s for _, s in spec.params()]
    inner = torch.nn.Module()
    inner.ps = torch.nn.ParameterList(
        [torch.nn.Parameter(t.view(s)) for t, s in zip(synth.outer_tree_device(spec, dev), shapes)])
    knob, prev = "DILOCO_OUTER_BUCKET_ELEMS", os.environ.get("DILOCO_OUTER_BUCKET_ELEMS")
    if bucket_elems is not None:
        os.environ[knob] = str(int(bucket_elems))
    try:
        outer = get_outer_model(inner, placement, wire=wire, exchange=exchange)
    finally:
        if bucket_elems is not None:
            if prev is None:
                os.environ.pop(knob, None)
            else:
                os.environ[knob] = prev
    opt = get_optimizer(outer, SimpleNamespace(type="SGD", lr=0.7, momentum=0.9, nesterov=True))
    # one TrainingComm per run, as src/train.py:291 makes (its DP group -- an RCCL
    # communicator at N > 1 -- is created once and shared by every leg)
    comm = training_comm(spec.n_embd)
    # inner = θ_0 + this rank's noise (H inner steps' stand-in); later steps see inner = θ
    synth.inner_tree_device([p.data.view(-1) for p in inner.parameters()], 1, rank,
                            out=[p.data.view(-1) for p in inner.parameters()])
    return inner, outer, opt, comm


def run_dropin(spec, dev, ws, rank, steps, warmup, wire="f32", bucket_elems=None,
               exchange=None, cold=False, synced=False, placement=None):
    """The outer step through the reference's call surface, src/train.py:263-269, on the outer
    model get_outer_model returns (placement None: the default, the reference's CPU outer
    model stepped on its HBM twin; "device": the outer model in HBM; exchange None: that
    placement's default, DEFAULT_EXCHANGE): K steps back to back
    between barrier + synchronize (the four Python calls of step k+1 are issued while step k's
    kernels run). synced: a device synchronize after every step, as the reference's loop has
    around its outer step (src/train.py:244), so the calls' host time is exposed; each step is
    timed on its own and the value is the median step's (one host stall on a shared box moved a
    10-step mean from 0.68 to 5.3 ms; the mean stays in the record). cold (N = 1): then K more
    steps, each after an Infinity-Cache scrub outside the events."""
    from diloco_amd.utils import compute_pseudo_gradient, sync_inner_model

    inner, outer, opt, comm = _dropin_objects(spec, dev, rank, wire, bucket_elems, exchange,
                                              placement)

    issue, wait = [], []  # synced: per step, the four calls' host time and the synchronize's

    def one():
        t1 = time.perf_counter()
        compute_pseudo_gradient(inner, outer)
        comm.sync_gradients(outer)
        opt.step()
        sync_inner_model(outer, inner)
        if synced:
            t2 = time.perf_counter()
            torch.cuda.synchronize()
            issue.append(t2 - t1)
            wait.append(time.perf_counter() - t2)

    for _ in range(max(warmup, 1)):
        one()
    _sync(ws)
    del issue[:], wait[:]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    ev[0].record()
    per = []
    for _ in range(steps):
        t1 = time.perf_counter()
        one()
        per.append(time.perf_counter() - t1)
    ev[1].record()
    _sync(ws)
    dt = _max_over_ranks((time.perf_counter() - t0) / steps, dev, ws)
    loop_ms = ev[0].elapsed_time(ev[1]) / steps
    mean_ms = dt * 1e3
    if synced:  # every step ended with a synchronize: its own wall time is the step's
        dt = _max_over_ranks(float(np.median(per)), dev, ws)
    P = spec.total()
    mm = outer._diloco_mirror
    m = getattr(mm, "dev", mm)  # the lazy host placement steps on its HBM twin
    # the bf16 wire: RCCL's bf16 all_reduce; int8: its all_to_all + rank-order reduce
    ex = "replicated" if wire == "bf16" else "int8 a2a" if wire == "int8" else m.exchange
    bpp = dropin_bpp(ws, ex, wire)
    res = {"tree": spec.name, "params": P, "tensors": len(m.params), "padded": m.tree.total,
           "buckets": m.tree.n_buckets, "ms_per_step": dt * 1e3, "value": 4.0 * P / dt / 1e9,
           "value_aggregate": ws * 4.0 * P / dt / 1e9, "loop_gpu_ms_per_step": round(loop_ms, 5),
           "wire": wire, "exchange": ex if ws > 1 else "none (one peer)",
           "hbm_bytes_per_param": round(bpp, 3), "synced": synced,
           **({"mean_ms_per_step": round(mean_ms, 5), "timing": "median step (synced)",
               "steps_ms": _spread(per), "issue_ms": _spread(issue), "sync_wait_ms": _spread(wait)}
              if synced else {}),
           "placement": ("device" if mm is m else "host (write_back lazy: HBM twin)")}
    if ws == 1:
        # one kernel per step: its average launch duration is the timed loop's GPU span / K
        # (the rocprofv3 average of the same command agrees, profiles/), <= ms_per_step
        res["roofline"] = kernel_entry(28 * P, loop_ms, load_pmc(spec.name).get("delta_pack_sgd"),
                                       kernel="dl_delta_pack_sgd",
                                       timing="timed loop GPU span / K")
        if cold:
            scr = Scrubber(dev)
            cev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(steps)]
            for e in cev:
                scr()
                e[0].record()
                one()
                e[1].record()
            torch.cuda.synchronize()
            scr.close()
            c_ms = sum(e[0].elapsed_time(e[1]) for e in cev) / steps
            res["cold"] = {"step_ms": round(c_ms, 5), "value": 4.0 * P / (c_ms * 1e-3) / 1e9,
                           "note": "Infinity Cache scrubbed before each step (512 MiB copy "
                                   "outside the events); the four calls' event span"}
    else:
        res["roofline"] = exchange_roofline(m, ws, dev, steps, comm.dp.dp_group(dev))
    mm.close()
    del outer, opt, inner, m, mm
    torch.cuda.empty_cache()
    return res


def _spread(xs):
    """Median, mean, p90, max and the five slowest of a list of seconds, in ms."""
    if not xs:
        return None
    a = np.sort(np.asarray(xs) * 1e3)
    return {"median": round(float(np.median(a)), 4), "mean": round(float(a.mean()), 4),
            "p90": round(float(a[int(0.9 * (len(a) - 1))]), 4), "max": round(float(a[-1]), 4),
            "slowest": [round(float(x), 3) for x in a[-5:][::-1]]}


def exchange_roofline(m, ws, dev, steps, group):
    """The exchange of the drop-in step alone: the same collectives the step makes on the
    mirror's buffers (every bucket: sharded reduce_scatter + all_gather(θ); a2a all_to_all +
    all_gather; replicated all_reduce), back to back, max over ranks. Bus bytes per GPU:
    (n-1)/n of the wire + (n-1)/n of θ for the sharded forms, 2(n-1)/n of the wire for the
    all-reduce; peak (n-1) x 153 GB/s (one xGMI link per peer)."""
    rank = dist.get_rank(group)
    if m.wire == "int8":  # all_to_all + all_gather of every bucket's slots
        q = m._q8
        S = q["S"]
        recv = q["recv"][0]
        slot_bytes = sum(q["n"] * p[1] for p in q["plan"]) * S

        def once_q8():
            for b, (nch, mm, base, rb) in enumerate(q["plan"]):
                region = m._q8_region(q, b)
                dist.all_to_all_single(recv[:ws * mm * S], region, group=group)
                dist.all_gather_into_tensor(region, q["red"][rb * S:(rb + mm) * S], group=group)

        once_q8()
        _sync(ws)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = max(3, steps // 2)
        e0.record()
        for _ in range(reps):
            once_q8()
        e1.record()
        e1.synchronize()
        ms = _max_over_ranks(e0.elapsed_time(e1) / reps, dev, ws)
        return kernel_entry(2.0 * (ws - 1) / ws * slot_bytes, ms, bound="xgmi",
                            peak=(ws - 1) * XGMI_LINK_GBS,
                            kernel="rccl all_to_all + all_gather of the int8 slots")
    w = m.d_wire16 if m.wire == "bf16" else m.d_wire
    sharded = m.exchange != "replicated" and m.wire != "bf16"
    recv = torch.empty_like(w) if m.exchange == "a2a" else None
    frac = (ws - 1) / ws * m.tree.total
    bus = frac * (w.element_size() + 4) if sharded else 2.0 * frac * w.element_size()

    def once():
        for b, (lo, hi) in enumerate(m.tree.bucket_ranges):
            if not sharded:
                dist.all_reduce(w[lo:hi], group=group)
                continue
            a, e = m._own(b, ws, rank)
            if recv is not None:
                dist.all_to_all_single(recv[lo:hi], w[lo:hi], group=group)
            else:
                dist.reduce_scatter_tensor(w[a:e], w[lo:hi], group=group)
            dist.all_gather_into_tensor(m.d_theta[lo:hi], m.d_theta[a:e], group=group)

    reps = max(3, steps // 2)
    once()
    _sync(ws)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        once()
    e1.record()
    e1.synchronize()
    ms = _max_over_ranks(e0.elapsed_time(e1) / reps, dev, ws)
    name = ("rccl all_to_all + all_gather" if recv is not None else
            "rccl reduce_scatter + all_gather" if sharded else "rccl all_reduce")
    return kernel_entry(bus, ms, bound="xgmi", peak=(ws - 1) * XGMI_LINK_GBS,
                        kernel=name + " (all buckets, back to back)")


# ---- the engine (OuterSync) and the codec legs -----------------------------------------------
def build(spec, dev, rank, wire, cap, fuse=True, shard=None, exchange="rccl", keep_wire=False,
          group=None):
    shapes = [s for _, s in spec.params()]
    theta0 = synth.outer_tree_device(spec, dev)
    params = [t.view(s) for t, s in zip(theta0, shapes)]
    eng = OuterSync(params, lr=0.7, momentum=0.9, nesterov=True, wire_dtype=wire,
                    bucket_cap_elems=cap, fuse_single=fuse, shard=shard, exchange=exchange,
                    keep_wire=keep_wire, group=group if group is not None else dp_group(dev))
    # inner = θ_0 + this rank's noise (stands in for H inner steps)
    synth.inner_tree_device([p.view(-1) for p in params], 1, rank, out=[p.view(-1) for p in params])
    return eng


def run_engine(spec, dev, ws, rank, steps, warmup, wire, cap, fuse=True, shard=None,
               exchange="rccl", keep_wire=False):
    """OuterSync.step, K steps timed between barrier + synchronize. Roofline at N = 1: the
    one-pass kernel from the timed loop's span, or (two kernels: fuse=False) each kernel from
    an instrumented pass with events between them; at N > 1 the exchange's collectives."""
    eng = build(spec, dev, rank, wire, cap, fuse, shard, exchange, keep_wire)
    P = spec.total()
    for _ in range(max(warmup, 1)):  # >= 1: the timed steps run the steady-state SGD mode
        eng.step()
    _sync(ws)
    loop_ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    loop_ev[0].record()
    for _ in range(steps):
        eng.step()
    loop_ev[1].record()
    _sync(ws)
    dt = _max_over_ranks(time.perf_counter() - t0, dev, ws)
    loop_ms = loop_ev[0].elapsed_time(loop_ev[1]) / steps
    wb = 2 if wire == torch.bfloat16 else 4
    res = {"tree": spec.name, "params": P, "buckets": eng.tree.n_buckets,
           "ms_per_step": dt / steps * 1e3, "value": 4.0 * P / (dt / steps) / 1e9,
           "value_aggregate": ws * 4.0 * P / (dt / steps) / 1e9,
           "wire": "bf16" if wire == torch.bfloat16 else "f32",
           "variant": ("dl_delta_pack_sgd (one pass, wire kept)" if ws == 1 and fuse and keep_wire
                       else "dl_delta_sgd (one pass)" if ws == 1 and fuse
                       else "dl_delta_pack -> dl_unpack_sgd (tiled)" if ws == 1
                       else "all_to_all -> rank-order reduce + shard SGD -> all_gather" if eng.a2a
                       else "reduce_scatter -> shard SGD -> all_gather" if eng.sharded
                       else "all_reduce -> replicated SGD")}
    if ws == 1 and fuse:
        name = "delta_pack_sgd" if keep_wire else "delta_sgd"
        nbytes = (24 + (wb if keep_wire else 0)) * P
        pmc = load_pmc(spec.name) if wire == torch.float32 else {}
        res["roofline"] = kernel_entry(nbytes, loop_ms, pmc.get(name), kernel="dl_" + name,
                                       timing="timed loop GPU span / K")
    elif ws == 1:
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
        for e in ev:  # the kernels on the stream they run on, events between them
            e[0].record()
            eng.pseudo_gradient()
            e[1].record()
            eng.apply()
            eng.steps_done += 1
            e[2].record()
        torch.cuda.synchronize()
        first = sum(e[0].elapsed_time(e[1]) for e in ev) / steps
        second = sum(e[1].elapsed_time(e[2]) for e in ev) / steps
        ks = {"delta_pack": kernel_entry((8 + wb) * P, first, kernel="dl_delta_pack"),
              "unpack_sgd": kernel_entry((wb + 20) * P, second, kernel="dl_unpack_sgd")}
        res["kernels"] = ks
        res["roofline"] = dict(max(ks.values(), key=lambda k: k["avg_ms"]),
                               timing="instrumented pass (events between the kernels)")
    elif eng.xgmi:
        # the exchange kernel moves (n-1)/n·4P in (peers' inner / wire) and (n-1)/n·4P out
        # (θ stores); over the whole step time this is a lower bound on its xGMI rate
        bus = 2.0 * (ws - 1) / ws * 4 * eng.tree.total
        res["roofline"] = kernel_entry(bus, dt / steps * 1e3, bound="xgmi",
                                       peak=(ws - 1) * XGMI_LINK_GBS,
                                       kernel="dl_xgmi_delta_sgd (whole step, lower bound)")
    else:
        def collectives():
            for b in range(eng.tree.n_buckets):
                if eng.sharded:
                    eng.reduce_scatter(b, async_op=False)
                    eng.all_gather(b, async_op=False)
                else:
                    eng.all_reduce(b, async_op=False)

        collectives()
        _sync(ws)
        reps = max(3, steps // 2)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            collectives()
        e1.record()
        e1.synchronize()
        ms = _max_over_ranks(e0.elapsed_time(e1) / reps, dev, ws)
        frac = (ws - 1) / ws * eng.tree.total
        bus = frac * (wb + 4) if eng.sharded else 2.0 * frac * wb
        res["roofline"] = kernel_entry(bus, ms, bound="xgmi", peak=(ws - 1) * XGMI_LINK_GBS,
                                       kernel="the engine's collectives, back to back")
    eng.close()
    del eng
    torch.cuda.empty_cache()
    return res


def run_q8(spec, dev, ws, rank, steps, warmup, cap):
    """int8 wire: per-bucket dl_delta_q8 -> all_to_all -> dl_q8_reduce ->
    all_gather -> dl_unpack_sgd_q8; 1.016 B/param on the bus instead of 4. At one replica the
    exchange is skipped and the three kernels run once each over the whole tree (timed in place
    with events; roofline = the slowest)."""
    from diloco_amd.kernels import Q8_SLOT
    from diloco_amd.plan import SLOT_INNER

    eng = build(spec, dev, rank, torch.int8, cap)
    P = spec.total()
    for _ in range(max(warmup, 1)):
        eng.step()
    _sync(ws)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.step()
    _sync(ws)
    dt = _max_over_ranks(time.perf_counter() - t0, dev, ws)
    slot_bytes = eng.tree.n_chunks * Q8_SLOT
    res = {"tree": spec.name, "params": P, "buckets": eng.tree.n_buckets,
           "ms_per_step": dt / steps * 1e3, "value": 4.0 * P / (dt / steps) / 1e9,
           "value_aggregate": ws * 4.0 * P / (dt / steps) / 1e9, "wire": "int8",
           "wire_bytes_per_param": round(slot_bytes / P, 4),
           "bus_bytes_per_step": 2.0 * (ws - 1) / ws * slot_bytes}
    if ws == 1:
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        tot = [[], [], []]
        for _ in range(steps):
            ev[0].record()
            eng.k.delta_q8(eng.tree, -1, SLOT_INNER, eng.theta, eng.q_slots)
            ev[1].record()
            eng.k.q8_reduce(eng.q_slots, 1, eng.tree.n_chunks, 1, eng.q_slots)
            ev[2].record()
            eng.k.unpack_sgd_q8(eng.tree, -1, eng.q_slots, eng.theta, eng.mom, eng.lr,
                                eng.momentum, eng.nesterov, False, SLOT_INNER)
            ev[3].record()
            eng.steps_done += 1
            torch.cuda.synchronize()
            for i in range(3):
                tot[i].append(ev[i].elapsed_time(ev[i + 1]))
        pmc = load_pmc(spec.name)
        ks = {}
        for i, (name, nb) in enumerate((("delta_q8", 8 * P + slot_bytes),
                                        ("q8_reduce", 2 * slot_bytes),
                                        ("unpack_sgd_q8", slot_bytes + 20 * P))):
            t = torch.tensor(tot[i], dtype=torch.float64)
            ks[name] = kernel_entry(nb, float(t.mean()), pmc.get(name), kernel="dl_" + name,
                                    rel_std=round(float(t.std() / t.mean()), 4) if steps > 1 else 0)
        res["kernels"] = ks
        res["roofline"] = dict(max(ks.values(), key=lambda k: k["avg_ms"]))
    eng.close()
    del eng
    torch.cuda.empty_cache()
    return res


# ---- parity self-checks (one codec contract: diloco_amd.outer.bf16_codec_bound) ------------------
def _identical(t, ws):
    """Every replica holds bit-identical bytes of t (checksums compared by max over ranks)."""
    bits = t.view(torch.int32).to(torch.int64).sum()
    ck = torch.stack([bits, -bits])
    if ws > 1:
        dist.all_reduce(ck, op=dist.ReduceOp.MAX, group=dp_group(t.device))
    return bool(ck[0].item() == -ck[1].item())


def parity_f32(dev, ws, rank):
    """The HIP path (+ RCCL at N > 1) on the tiny tree with 3 buckets: the averaged deltas
    normwise <= 1e-6 of a plain torch fp32 statement of every rank's delta (the north-star
    tolerance), every replica bit-identical after the step."""
    spec = get_tree("tiny")
    eng = build(spec, dev, rank, torch.float32, 1 << 20, shard=False)
    for b in range(eng.tree.n_buckets):
        eng.pseudo_gradient(b)
        if ws > 1:
            eng.all_reduce(b, async_op=False)
    got = [t.reshape(-1) / ws for t in eng.unpacked(eng.wire)]
    theta0 = synth.outer_tree_device(spec, dev)
    acc = [torch.zeros_like(t) for t in theta0]
    for r in range(ws):  # every rank's inner, regenerated locally (counter-based)
        acc = [a + (t - i) for a, t, i in zip(acc, theta0, synth.inner_tree_device(theta0, 1, r))]
    worst = 0.0
    for g, a in zip(got, acc):
        ref = a / ws
        worst = max(worst, float((g - ref).abs().max()) / float(ref.abs().max().clamp_min(1e-30)))
    eng.apply()
    eng.steps_done += 1
    torch.cuda.synchronize()
    identical = _identical(eng.theta, ws)
    eng.close()
    return {"tree": "tiny", "err": worst, "tol": 1e-6, "replicas_identical": identical,
            "ok": bool(worst <= 1e-6 and identical)}


def codec_parity(spec, dev, ws, rank, cap, picks=None):
    """The bf16 wire's one error contract (config #5; diloco_amd.outer.bf16_codec_bound, as
    tests/test_configs_gpu.py holds it): one outer step through the real exchange -- the
    replicated RCCL bf16 all-reduce (the bf16 default) and the ordered exchange
    (exchange="a2a": bf16 slices summed in fp32 in rank order) -- against the fp32 statement
    of the same step in torch, element by element: |u_bf16 - u_fp32| over the per-element
    a-priori bound of the applied update, worst ratio <= 1 required. picks: the tensors checked
    (default all)."""
    from diloco_amd.outer import U_F32, bf16_codec_bound

    nt = len(spec.params())
    picks = list(range(nt)) if picks is None else picks
    out = {"tree": spec.name, "n": ws}
    for name, kw in (("rccl", dict(shard=False)), ("a2a", dict(shard=None, exchange="a2a"))):
        eng = build(spec, dev, rank, torch.bfloat16, cap, fuse=False, **kw)
        th0 = {t: eng.unpacked(eng.theta)[t].reshape(-1).clone() for t in picks}
        eng.step()
        torch.cuda.synchronize()
        th1 = eng.unpacked(eng.theta)
        worst_norm, worst_ratio = 0.0, 0.0
        for t in picks:
            x0 = th0[t]
            sabs = torch.zeros_like(x0)
            g = torch.zeros_like(x0)
            for r in range(ws):  # every peer's inner, regenerated (counter-based)
                inner = torch.empty_like(x0)
                synth.fill_device(inner, synth.noise_seed(1, r), t, 0.0, synth.NOISE_SCALE, add=x0)
                d = x0 - inner
                g += d  # rank order, fp32
                sabs += d.abs()
                del inner, d
            g /= ws
            u32 = 0.7 * (g + 0.9 * g)  # first Nesterov step: buf = g, u = g + m·buf
            ubf = x0 - th1[t].reshape(-1)
            err = (ubf - u32).abs()
            bound = (0.7 * 1.9 * bf16_codec_bound(sabs, ws, name)
                     + 4 * U_F32 * (x0.abs() + th1[t].reshape(-1).abs() + 2 * u32.abs()))
            worst_norm = max(worst_norm, float(err.max()) / max(float(u32.abs().max()), 1e-30))
            worst_ratio = max(worst_ratio, float((err / bound).max()))
        out[name] = {"normwise": worst_norm, "err_over_bound": round(worst_ratio, 4),
                     "identical": _identical(eng.theta, ws)}
        eng.close()
        del eng, th0, th1
        torch.cuda.empty_cache()
    out["err"] = max(out["rccl"]["err_over_bound"], out["a2a"]["err_over_bound"])
    out["ok"] = bool(out["err"] <= 1.0 and out["rccl"]["identical"] and out["a2a"]["identical"])
    return out


def parity_q8(dev, ws, rank):
    """int8 codec on the tiny tree (3 buckets): the averaged g every replica applies against the
    exact fp32 average, element by element, within the quantiser's own bound
        |g - avg| <= (1/n) Σ_r s_r/2 + s'/2,   s_r = amax_chunk(delta_r)/127,
        s' = amax_chunk(avg')/127 <= (amax_chunk(avg) + (1/n) Σ_r s_r/2)/127
    (plus 1e-5 relative slack for the fp32 sums); and every replica bit-identical after it."""
    from diloco_amd.kernels import Q8_SLOT

    spec = get_tree("tiny")
    eng = build(spec, dev, rank, torch.int8, 1 << 20)
    deq = []
    for b in range(eng.tree.n_buckets):
        eng.pseudo_gradient(b)
        nch, m, _ = eng.q8_plan[b]
        if ws > 1:
            eng.q8_exchange(b).wait()
        else:
            region = eng.q8_region(b)
            eng.k.q8_reduce(region, 1, m, 1, region)
        sl = eng.q8_region(b).view(-1, Q8_SLOT)[:nch]
        scale = sl[:, :4].contiguous().view(torch.float32)
        deq.append(sl[:, 64:].contiguous().view(torch.int8).float() * scale)
    deq = torch.cat(deq)  # [n_chunks, 4096], tree chunk order
    theta0 = synth.outer_tree_device(spec, dev)
    deltas = [[t - i for t, i in zip(theta0, synth.inner_tree_device(theta0, 1, r))]
              for r in range(ws)]

    def rows(x):  # one tensor -> its chunks, zero-padded to 4096
        k = -(-x.numel() // 4096)
        return torch.nn.functional.pad(x.reshape(-1), (0, k * 4096 - x.numel())).view(k, 4096)

    worst, c = 0.0, 0
    for t in range(len(theta0)):
        ref = deltas[0][t].clone()
        for r in range(1, ws):
            ref = ref + deltas[r][t]
        if ws > 1:
            ref = ref / ws
        R = rows(ref)
        k = R.shape[0]
        half_s = sum(rows(deltas[r][t]).abs().amax(1, keepdim=True) / 254 for r in range(ws)) / ws
        s2 = (R.abs().amax(1, keepdim=True) + half_s) / 127
        bound = (half_s + s2 / 2) * (1 + 1e-5) + 1e-30
        worst = max(worst, float(((deq[c:c + k] - R).abs() / bound).max()))
        c += k
    for b in range(eng.tree.n_buckets):
        eng.apply(b)
    eng.steps_done += 1
    torch.cuda.synchronize()
    identical = _identical(eng.theta, ws)
    eng.close()
    return {"tree": "tiny", "err": worst, "tol": 1.0, "replicas_identical": identical,
            "ok": bool(worst <= 1.0 and identical)}


def parity_sharded(dev, ws, rank, exchange="rccl"):
    """The engine's sharded step (exchange="a2a": all_to_all + rank-order reduce) against its
    replicated one (all-reduce -> dl_unpack_sgd) on the tiny tree, 2 outer steps: θ, momentum
    and inner normwise <= 1e-6 per tensor (bit-exact where the two sum in the same order),
    every replica bit-identical."""
    spec = get_tree("tiny")
    ea = build(spec, dev, rank, torch.float32, 1 << 20, shard=True, exchange=exchange)
    eb = build(spec, dev, rank, torch.float32, 1 << 20, shard=False)
    for s in (1, 2):
        for e in (ea, eb):
            if s > 1:
                th = [t.reshape(-1) for t in e.unpacked(e.theta)]
                synth.inner_tree_device(th, s, rank, out=[p.view(-1) for p in e.params])
            e.step()
    torch.cuda.synchronize()
    worst, exact = 0.0, True
    for x, y in ((ea.theta, eb.theta), (ea.momentum_full(), eb.momentum_full())):
        exact &= bool(torch.equal(x, y))
        for a, b in zip(ea.unpacked(x), eb.unpacked(y)):
            worst = max(worst, float((a - b).abs().max()) / float(b.abs().max().clamp_min(1e-30)))
    inner_ok = all(torch.equal(p, t) for p, t in zip(ea.params, ea.unpacked(ea.theta)))
    identical = _identical(ea.theta, ws)
    ea.close()
    eb.close()
    return {"tree": "tiny", "exchange": exchange, "err": worst, "bit_exact": exact, "tol": 1e-6,
            "inner_is_theta": inner_ok, "replicas_identical": identical,
            "ok": bool(worst <= 1e-6 and identical and inner_ok)}


def parity_dropin_exchanges(dev, ws, rank):
    """The exchanges behind the reference's calls at N > 1: the outer model get_outer_model
    returns, with exchange="sharded" (opt-in here) and "a2a" against "replicated" (the
    headline's, the default placement's default), tiny tree
    in 4 MiB buckets, 2 outer steps: θ, .grad, the momentum buffers (the sharded ones
    gathered on read) and the inner params normwise <= 1e-6 per tensor (bit-exact at n <= 2), every
    replica identical."""
    from diloco_amd.utils import compute_pseudo_gradient, sync_inner_model

    spec = get_tree("tiny")
    runs = {}
    for ex in ("replicated", "sharded", "a2a"):
        inner, outer, opt, comm = _dropin_objects(spec, dev, rank, "f32", 1 << 20, ex)
        for s in (1, 2):
            if s > 1:
                synth.inner_tree_device([p.data.view(-1).to(dev) for p in outer.parameters()], s,
                                        rank, out=[p.data.view(-1) for p in inner.parameters()])
            compute_pseudo_gradient(inner, outer)
            comm.sync_gradients(outer)
            opt.step()
            sync_inner_model(outer, inner)
        flat = {k: torch.cat([t.detach().reshape(-1).to(dev) for t in ts]) for k, ts in (
            ("theta", list(outer.parameters())), ("grad", [p.grad for p in outer.parameters()]),
            ("mom", [opt.state[p]["momentum_buffer"] for p in outer.parameters()]),
            ("inner", list(inner.parameters())))}
        runs[ex] = (flat, [p.numel() for p in outer.parameters()])
        outer._diloco_mirror.close()
        del inner, outer, opt
    torch.cuda.synchronize()
    ref, numels = runs["replicated"]
    out = {"tree": "tiny", "tol": 1e-6}
    for ex in ("sharded", "a2a"):
        got = runs[ex][0]
        worst, exact = 0.0, True
        for k in ("theta", "grad", "mom", "inner"):
            exact &= bool(torch.equal(got[k], ref[k]))
            for a, b in zip(got[k].split(numels), ref[k].split(numels)):
                worst = max(worst, float((a - b).abs().max())
                            / float(b.abs().max().clamp_min(1e-30)))
        out[ex] = {"err": worst, "bit_exact": exact,
                   "identical": _identical(got["theta"], ws)}
    out["err"] = max(out["sharded"]["err"], out["a2a"]["err"])
    out["ok"] = bool(out["err"] <= 1e-6 and out["sharded"]["identical"]
                     and out["a2a"]["identical"] and (ws > 2 or out["sharded"]["bit_exact"]))
    return out


# ---- N > 1 side legs ------------------------------------------------------------------------
def rccl_reference(dev, ws, rank, elems, reps=5):
    """What RCCL itself reaches on this node for the given bytes: one fp32 all_reduce (SUM) of
    `elems` elements, and a reduce_scatter + all_gather pair of the same size, back to back,
    max over ranks. busBW = 2(n-1)/n · bytes / t (the nccl-tests convention)."""
    out = {}
    group = dp_group(dev)
    if dist.get_backend(group) == "gloo":
        # a gloo rehearsal on one GPU stages whole tensors through host memory in every rank:
        # 8 ranks x a 5 GB tree exceed the box's host-memory cap, and the rate is gloo's anyway
        cap = (256 << 20) // 4 // (64 * ws) * (64 * ws)
        if elems > cap:
            out["capped_for_gloo_elems"] = elems
            elems = cap
    x = torch.ones(elems, device=dev)
    sh = torch.empty(elems // ws, device=dev)
    for name in ("all_reduce", "reduce_scatter+all_gather"):
        for it in range(reps + 1):
            if it == 1:  # the first call warms the communicator's buffers
                _sync(ws)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
            if name == "all_reduce":
                dist.all_reduce(x, group=group)
            else:
                dist.reduce_scatter_tensor(sh, x, group=group)
                dist.all_gather_into_tensor(x, sh, group=group)
        e1.record()
        e1.synchronize()
        ms = _max_over_ranks(e0.elapsed_time(e1) / reps, dev, ws)
        bus = 2.0 * (ws - 1) / ws * 4 * elems
        out[name] = {"ms": round(ms, 4), "busbw_GBs": round(bus / (ms * 1e-3) / 1e9, 1)}
    out["bytes"] = 4 * elems
    del x, sh
    torch.cuda.empty_cache()
    return out


def exchange_efficiency(step_res, ref, ws):
    """The whole outer step as bus bytes / step time against RCCL's own all_reduce of the same
    bytes (same node, same run): the north star's ">= 80 % of algorithmic xGMI all-reduce
    bandwidth" at N = 8 on the 1.3B bucket set."""
    if not (isinstance(step_res, dict) and "ms_per_step" in step_res and isinstance(ref, dict)
            and "all_reduce" in ref):
        return None
    bus = 2.0 * (ws - 1) / ws * 4 * step_res["params"]
    bw = bus / (step_res["ms_per_step"] * 1e-3) / 1e9
    ar = ref["all_reduce"]["busbw_GBs"]
    return {"step_busbw_GBs": round(bw, 1), "rccl_allreduce_busbw_GBs": ar,
            "frac_of_rccl_allreduce": round(bw / ar, 4),
            "frac_of_link_peak": round(bw / ((ws - 1) * XGMI_LINK_GBS), 4)}


def gradsync_rate(spec, dev, ws, rank, steps, exchange="rccl"):
    """Per-step DP gradient average of device grads (src/train.py:249-251,
    src/comm.py:117-123): dl_gather -> RCCL all_reduce -> dl_unpack_avg, pipelined buckets."""
    from diloco_amd.gradsync import GradSync

    shapes = [s for _, s in spec.params()]
    params = [torch.nn.Parameter(t.view(s))
              for t, s in zip(synth.outer_tree_device(spec, dev), shapes)]
    for i, p in enumerate(params):
        p.grad = torch.empty_like(p)
        synth.fill_device(p.grad.view(-1), synth.noise_seed(9, rank), i, 0.0, 1e-3)
    gs = GradSync(params, dp_group(dev), ws, exchange=exchange)
    gs.sync()
    _sync(ws)
    t0 = time.perf_counter()
    for _ in range(steps):
        gs.sync()
    _sync(ws)
    dt = _max_over_ranks((time.perf_counter() - t0) / steps, dev, ws)
    P = spec.total()
    gs.close()
    return {"tree": spec.name, "params": P, "value": 4.0 * P / dt / 1e9,
            "value_aggregate": ws * 4.0 * P / dt / 1e9, "ms_per_step": dt * 1e3,
            "exchange": exchange}


def run_two_stages(spec, dev, ws, rank, steps, warmup, cap):
    """The reference's two-stage layout (src/world.py:96-97, stage = rank % 2): two disjoint DP
    groups of ws/2 ranks run the sharded outer step at the same time, each over its own RCCL
    communicator. value = 2 · 4P / t_step (two trees reduced per step)."""
    from diloco_amd import comm

    groups = [dist.new_group([r for r in range(ws) if r % 2 == s], backend=comm.dp_backend())
              for s in range(2)]
    eng = build(spec, dev, rank, torch.float32, cap, group=groups[rank % 2])
    for _ in range(max(warmup, 1)):
        eng.step()
    _sync(ws)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.step()
    _sync(ws)
    dt = _max_over_ranks(time.perf_counter() - t0, dev, ws) / steps
    eng.close()
    del eng
    torch.cuda.empty_cache()
    return {"tree": spec.name, "params": spec.total(), "stages": 2, "dp_per_stage": ws // 2,
            "ms_per_step": dt * 1e3, "value": 2 * 4.0 * spec.total() / dt / 1e9,
            "value_aggregate": ws * 4.0 * spec.total() / dt / 1e9}


def dropin_pcie(spec, dev, ws, rank, steps):
    """The reference's host-resident outer model (placement="host", src/utils.py:216) through
    the four calls, PCIe transfers included, a device synchronize ending every step: the
    PCIe-inclusive rate DESIGN.md §7 records (not the headline)."""
    from types import SimpleNamespace

    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)

    shapes = [s for _, s in spec.params()]
    inner = torch.nn.Module()
    inner.ps = torch.nn.ParameterList(
        [torch.nn.Parameter(t.view(s)) for t, s in zip(synth.outer_tree_device(spec, dev), shapes)])
    outer = get_outer_model(inner, "host", write_back="sync")  # host tensors authoritative
    opt = get_optimizer(outer, SimpleNamespace(type="SGD", lr=0.7, momentum=0.9, nesterov=True))
    comm = training_comm(spec.n_embd)
    synth.inner_tree_device([p.data.view(-1) for p in inner.parameters()], 1, rank,
                            out=[p.data.view(-1) for p in inner.parameters()])
    phases = [0.0] * 4

    def one(record):
        t = [time.perf_counter()]
        compute_pseudo_gradient(inner, outer)
        t.append(time.perf_counter())
        comm.sync_gradients(outer)
        t.append(time.perf_counter())
        opt.step()
        t.append(time.perf_counter())
        sync_inner_model(outer, inner)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        if record:
            for i in range(4):
                phases[i] += t[i + 1] - t[i]

    one(False)
    if ws > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        one(True)
    dt = _max_over_ranks((time.perf_counter() - t0) / steps, dev, ws)
    P = spec.total()
    outer._diloco_mirror.close()
    return {"tree": spec.name, "params": P, "value": 4.0 * P / dt / 1e9,
            "value_aggregate": ws * 4.0 * P / dt / 1e9, "ms_per_step": dt * 1e3,
            "phase_ms": dict(zip(("compute_pseudo_gradient", "sync_gradients", "outer_step",
                                  "sync_inner_model"),
                                 (round(v / steps * 1e3, 3) for v in phases))),
            "d2h_bytes_per_step": (16 if ws > 1 else 12) * P}


def xgmi_link_probe(dev, ws, rank, reps=5, mib=256):
    """Peer read rates through IPC-mapped buffers (what the 153 GB/s per link
    means): every rank at once reads `mib` MiB from its ring neighbour (one direction of one
    link each), then from every peer at once, then from its own HBM; max time over ranks."""
    import ctypes

    from diloco_amd.xgmi import PeerMap

    n = (mib << 20) // 4
    buf = torch.empty(n, device=dev)
    synth.fill_device(buf, 3, rank, 0.0, 1.0)
    dst = torch.empty(max(1, ws - 1) * n, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _lib.call("dl_sys_fence", stream)  # the filled bytes leave this GPU's L2 before peers read
    pm = PeerMap({"buf": buf}, None, dev)
    if not pm.ok:
        return {"ok": False, "error": pm.reason}
    _lib.call("dl_sys_fence", stream)
    tab = pm.table("buf")
    p64 = ctypes.POINTER(ctypes.c_uint64)

    def timed(srcs):
        arr = np.asarray(srcs, dtype=np.uint64)
        _sync(ws)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            _lib.call("dl_peer_gather", arr.ctypes.data_as(p64), len(srcs), n * 4,
                      dst.data_ptr(), stream)
        e1.record()
        e1.synchronize()
        ms = _max_over_ranks(e0.elapsed_time(e1) / reps, dev, ws)
        return round(len(srcs) * n * 4 / (ms * 1e-3) / 1e9, 1)

    one = timed([int(tab[(rank + 1) % ws])])
    want = torch.empty(n, device=dev)  # the neighbour's buffer, regenerated here
    synth.fill_device(want, 3, (rank + 1) % ws, 0.0, 1.0)
    ok = bool(torch.equal(dst[:n], want))
    allp = timed([int(tab[q]) for q in range(ws) if q != rank])
    local = timed([int(tab[rank])])
    _sync(ws)
    pm.close()
    _sync(ws)
    return {"bytes_per_source": n * 4, "one_peer_read_GBs": one, "all_peers_read_GBs": allp,
            "local_hbm_read_GBs": local, "peers": ws - 1, "value": one, "ok": ok}


def parity_xgmi(dev, ws, rank):
    """The direct exchange without a wire (exchange="xgmi_inner") against the RCCL sharded step
    on the tiny tree, 2 outer steps: θ and momentum normwise <= 1e-6 per tensor, inner == θ,
    replicas identical."""
    spec = get_tree("tiny")
    ea = build(spec, dev, rank, torch.float32, 1 << 20, exchange="xgmi_inner")
    eb = build(spec, dev, rank, torch.float32, 1 << 20)
    for s in (1, 2):
        for e in (ea, eb):
            if s > 1:
                th = [t.reshape(-1) for t in e.unpacked(e.theta)]
                synth.inner_tree_device(th, s, rank, out=[p.view(-1) for p in e.params])
            e.step()
    torch.cuda.synchronize()
    worst = 0.0
    for x, y in ((ea.theta, eb.theta), (ea.momentum_full(), eb.momentum_full())):
        for a, b in zip(ea.unpacked(x), eb.unpacked(y)):
            worst = max(worst, float((a - b).abs().max()) / float(b.abs().max().clamp_min(1e-30)))
    inner_ok = all(torch.equal(p, t) for p, t in zip(ea.params, ea.unpacked(ea.theta)))
    identical = _identical(ea.theta, ws)
    ea.close()
    eb.close()
    return {"tree": "tiny", "err": worst, "tol": 1e-6, "inner_is_theta": inner_ok,
            "replicas_identical": identical, "ok": bool(worst <= 1e-6 and identical and inner_ok)}


def peer_access_legs(spec13, dev, ws, rank, steps, cap, parity_too, dump):
    """In isolated child processes (a fault while peers' memory is mapped ends the children,
    not the run): the direct peer-access exchange without a wire on the 1.3B set, its parity
    check and the link probe. dump(result) after every leg."""
    res = {"legs": {}, "parity": {}}
    if parity_too:
        res["parity"]["xgmi"] = _guard(parity_xgmi, dev, ws, rank)
        dump(res)
    res["legs"]["xgmi_link_probe"] = _guard(xgmi_link_probe, dev, ws, rank)
    dump(res)
    r = _guard(run_engine, spec13, dev, ws, rank, max(3, steps // 4), 1, torch.float32, cap,
               False, None, "xgmi_inner")
    roof = r.get("roofline") if isinstance(r, dict) else None
    if isinstance(roof, dict) and torch.cuda.device_count() < ws:
        # a rehearsal with every rank on one GPU: the "peer" reads are local HBM reads
        roof["frac_vs_link"], roof["frac"] = roof.get("frac"), None
        roof["note"] = "ranks share one GPU: peer reads are local, the link peak does not apply"
    res["legs"][f"{spec13.name}_xgmi_inner"] = r
    dump(res)
    return res


# ---- the CPU baseline (the reference's path on the host's cores) -------------------------------
def _host_info():
    model = ""
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        model = next((ln.split(":", 1)[1].strip() for ln in out.splitlines()
                      if ln.startswith("Model name")), "")
    except Exception:
        pass
    return {"cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "model": model, "torch": torch.__version__}


def cpu_baseline(spec, seconds_budget=12.0):
    """The reference's per-tensor CPU sequence (oracle/torch_restatement.py), 1 thread."""
    sys.path.insert(0, HERE)
    from oracle.torch_restatement import time_steps

    t, n = time_steps(spec.numels(), steps=2, threads=1, budget_s=seconds_budget)
    return {"value": round(4.0 * spec.total() / t / 1e9, 4), "unit": "GB/s", "cores": 1,
            "kind": "port",
            "sample": (f"{spec.name} full tree ({spec.total()} params), {n} outer steps after 1 "
                       f"warm, per-tensor torch CPU restatement of src/utils.py:218-226 + torch "
                       f"SGD-Nesterov (n=1: no all_reduce), 1 thread; {t:.3f} s/step"),
            "host": _host_info()}


def cpu_baseline_dist(spec, ws, rank, seconds_budget=12.0, group=None):
    """§8d CPU baseline at N > 1: this process is one of N CPU processes (GPUs hidden) in a
    gloo group, each running the reference's per-tensor sequence on the full tree with one
    thread -- delta, per-tensor gloo all_reduce(SUM) + /= n, torch SGD-Nesterov, copy-back
    (oracle/torch_restatement.TorchOuterStep) -- N cores in all; value = 4P / t_step, max time
    over ranks. group: a gloo group over the N ranks when the bench's own rank processes run
    it (rehearsals with every rank on one GPU); default the child's world."""
    sys.path.insert(0, HERE)
    from oracle.torch_restatement import TorchOuterStep

    group = group or dist.group.WORLD
    torch.set_num_threads(1)
    g = torch.Generator().manual_seed(rank)
    inner = [torch.empty(n).uniform_(-0.03, 0.03, generator=g) for n in spec.numels()]
    st = TorchOuterStep(inner, group=group)
    for t in inner:
        t.add_(torch.empty_like(t).uniform_(-1e-3, 1e-3, generator=g))
    st.step()  # creates the momentum buffers (not timed)
    dist.barrier(group=group)
    t0 = time.perf_counter()
    st.step()
    one = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(one, op=dist.ReduceOp.MAX, group=group)
    k = max(2, int(seconds_budget / max(float(one.item()), 1e-3)))
    dist.barrier(group=group)
    t0 = time.perf_counter()
    for _ in range(k):
        st.step()
    dt = torch.tensor([(time.perf_counter() - t0) / k], dtype=torch.float64)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX, group=group)
    t = float(dt.item())
    return {"value": round(4.0 * spec.total() / t / 1e9, 4), "unit": "GB/s", "cores": ws,
            "kind": "port",
            "sample": (f"{spec.name} full tree ({spec.total()} params) per process, {ws} CPU "
                       f"processes (gloo, 1 thread each), {k} outer steps after 2: per-tensor "
                       f"torch restatement of src/utils.py:218-226 + per-tensor all_reduce/n "
                       f"(src/comm.py:120-123) + torch SGD-Nesterov; {t:.3f} s/step"),
            "host": _host_info()}


# CPU-baseline children see no GPU: they are host processes like the reference's --device cpu
HIDE_GPUS = {"CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""}


def _guard(fn, *a, **k):
    try:
        return fn(*a, **k)
    except Exception as e:  # reported in the record, never hidden
        log(f"{fn.__name__} failed: {e!r}")
        return {"ok": False, "error": repr(e)[:300]}


def isolated_legs(a, dev, ws, rank, timeout_s, which, extra_env=None):
    """Run a set of legs in a child process per rank (their own process group on a fresh
    rendezvous port): which="peer" -> peer_access_legs; which="cpu_baseline" -> the N-core CPU
    baseline. The parents wait (bounded), then carry on. Returns rank 0's child result, or an
    error record."""
    port = [0]
    if rank == 0:
        import socket

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port[0] = sk.getsockname()[1]
    dist.broadcast_object_list(port, src=0)
    out = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"dl_bench_child_{port[0]}_{rank}.json")
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port[0]), **(extra_env or {}))
    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", str(ws), "--steps", str(a.steps),
           "--warmup", str(a.warmup), "--tree", a.tree, "--extra-tree", a.extra_tree,
           "--bucket-mb", str(a.bucket_mb), "--deadline", str(max(30.0, timeout_s - 10)),
           "--child-legs", which, "--child-out", out] + (["--no-parity"] if a.no_parity else [])
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    try:
        rc = subprocess.run(cmd, env=env, timeout=timeout_s, stdout=sys.stderr).returncode
    except subprocess.TimeoutExpired:
        rc = "timeout"
    res = {"ok": False, "error": f"child exit {rc}"}
    if rank == 0 and os.path.exists(out):
        try:
            with open(out) as f:
                res = json.load(f)  # what the children finished, even if they were stopped
            res["child_exit"] = rc
        except ValueError as e:
            res = {"ok": False, "error": f"child exit {rc}; unreadable result: {e!r}"}
    if os.path.exists(out):
        os.remove(out)
    _sync(ws)  # every parent is past its child before anyone moves on
    return res


# ---- the one line --------------------------------------------------------------------------------
def _r(x, nd=4):
    return None if x is None else round(float(x), nd)


def leg_summary(r):
    """A side leg as one small record: GB/s (value), the roofline fraction, ms per step, and
    the HBM bytes per parameter where the leg states them; an error record passes its error."""
    if not isinstance(r, dict):
        return None
    if "value" not in r:
        return {"ok": False, "error": str(r.get("error", "no value"))[:120]}
    s = {"GBs": _r(r["value"], 1)}
    roof = r.get("roofline")
    if isinstance(roof, dict):
        s["frac"] = _r(roof.get("frac"))
    if "ms_per_step" in r:
        s["ms"] = _r(r["ms_per_step"], 4)
    if "mean_ms_per_step" in r:  # a median-timed leg: its mean beside it
        s["mean_ms"] = _r(r["mean_ms_per_step"], 4)
    if "hbm_bytes_per_param" in r:
        s["Bpp"] = r["hbm_bytes_per_param"]
    return s


def parity_summary(r):
    if not isinstance(r, dict):
        return None
    return {"ok": bool(r.get("ok", False)), "err": _r(r.get("err"), 9)}


def assemble_line(meta, head, cpu, legs, parity, exch=None, extra=None):
    """The one stdout line (<= LINE_MAX_BYTES) from the run's records: meta (n_gpus, steps,
    warmup, tree spec fields), the headline record, the CPU baseline, side legs and parity
    checks (name -> full record; only their one-number summaries go into the line) and the
    exchange efficiencies at N > 1. Strings that could grow are capped; if the line is still
    too long, side legs are dropped from the end (their records stay in the detail file)."""
    ws = meta["n_gpus"]
    roof = dict(head["roofline"])
    keep = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "bytes_per_launch",
            "avg_ms")
    roof = {k: roof.get(k) for k in keep}
    cold = head.get("cold")
    cb = None
    if isinstance(cpu, dict) and "value" in cpu:
        cb = {k: cpu.get(k) for k in ("value", "unit", "cores", "kind")}
        cb["sample"] = str(cpu.get("sample", ""))[:320]
    elif isinstance(cpu, dict):
        cb = {"value": None, "error": str(cpu.get("error", ""))[:120]}
    line = {
        "metric": METRIC,
        "value": _r(head["value"], 3),
        "value_aggregate": _r(head["value_aggregate"], 3),
        "value_cold": _r(cold["value"], 3) if isinstance(cold, dict) else None,
        "unit": "GB/s",
        "n_gpus": ws,
        "steps": meta["steps"],
        "warmup": meta["warmup"],
        "ms_per_step": _r(head["ms_per_step"], 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (counter-based GPT-2-shaped tree, SURVEY.md §8d)",
        "config": {"workload": meta["workload"][:300], "tree": head["tree"],
                   "placement": head.get("placement"),
                   "params": head["params"], "tensors": head["tensors"], "wire": head["wire"],
                   "buckets": head["buckets"], "exchange": head["exchange"],
                   "hbm_bytes_per_param": head["hbm_bytes_per_param"],
                   "parallelism": f"dp{ws}"},
        "roofline": roof,
        "cpu_baseline": cb,
        "legs": {k: leg_summary(v) for k, v in legs.items()},
        "parity": {k: parity_summary(v) for k, v in parity.items()},
    }
    if exch:
        line["exchange_efficiency"] = exch
    if extra:
        line.update(extra)
    while len(json.dumps(line)) > LINE_MAX_BYTES - 64 and line["legs"]:
        line["legs"].pop(next(reversed(line["legs"])))
        line.setdefault("legs_dropped_from_line", 0)
        line["legs_dropped_from_line"] += 1
    return line


class _Emitter:
    """The one JSON line, printed exactly once by rank 0, and the detail file beside it.

    A watchdog (every rank, same deadline) bounds the whole run: if a side leg hangs, the line
    with the headline and every leg finished so far is printed, naming the leg that was
    running, and every rank leaves with os._exit -- the driver still gets its measurement. A
    heartbeat thread names the running leg on stderr every 20 s (a silent minute would read as
    a hang). Legs that would start after the soft budget are skipped and listed."""

    def __init__(self, rank, deadline_s, detail_path=None, heartbeat_s=20.0):
        self.rank, self.t0, self.deadline = rank, time.perf_counter(), deadline_s
        self.build = None  # () -> the line, from what has finished so far
        self.detail, self.detail_path = {}, detail_path
        self.running, self.skipped = "headline", []
        self.lock = threading.Lock()
        self.done = False
        # the JSON line goes to the process's original stdout; everything else written to fd 1
        # during the run (gloo's "[Gloo] Rank ..." notices, library chatter) goes to stderr
        sys.stdout.flush()
        self.out_fd = os.dup(1)
        os.dup2(2, 1)
        self.timer = threading.Timer(deadline_s, self._fire)
        self.timer.daemon = True
        self.timer.start()
        self._beat = threading.Event()
        if heartbeat_s:
            t = threading.Thread(target=self._heartbeat, args=(heartbeat_s,), daemon=True)
            t.start()

    def _heartbeat(self, every):
        while not self._beat.wait(every):
            log(f"{self.elapsed():.0f} s: running {self.running}")

    def elapsed(self):
        return time.perf_counter() - self.t0

    def emit(self, incomplete=None):
        with self.lock:
            if self.done:
                return
            self.done = True
            self._beat.set()
            if self.rank != 0:
                return
            line = self.build() if self.build is not None else None
            if line is None:
                return
            if self.skipped:
                line["skipped_legs"] = self.skipped[:12]
            if incomplete:
                line["incomplete"] = incomplete
            line["wall_s"] = round(self.elapsed(), 1)
            if self.detail_path:
                try:
                    os.makedirs(os.path.dirname(self.detail_path) or ".", exist_ok=True)
                    with open(self.detail_path, "w") as f:
                        json.dump(dict(self.detail, line=line), f, indent=1, default=str)
                    line["detail"] = os.path.relpath(self.detail_path, HERE)
                except OSError as e:
                    log(f"detail file not written: {e!r}")
            buf = (json.dumps(line) + "\n").encode()
            while buf:
                buf = buf[os.write(self.out_fd, buf):]

    def _fire(self):
        log(f"watchdog: {self.deadline:.0f} s reached while running {self.running!r}")
        has_line = self.build is not None
        try:
            self.emit({"leg": self.running, "deadline_s": self.deadline})
        except Exception as e:  # the exit below must happen whatever the line does
            log(f"emit failed: {e!r}")
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0 if has_line else 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50,
                    help="timed steps K (the first timed step also carries the host's issue of "
                         "its calls after the barrier: 1/K of the per-step figure)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--tree", default="t125")
    ap.add_argument("--bucket-mb", type=int, default=256)
    ap.add_argument("--extra-tree", default="t1.3b", help="second tree measured beside (or 'none')")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-xgmi", action="store_true",
                    help="skip the isolated peer-access legs at N > 1")
    ap.add_argument("--only-headline", action="store_true",
                    help="headline only, no cold pass (rocprofv3 runs of the same kernel)")
    ap.add_argument("--no-b2b", action="store_true", help=argparse.SUPPRESS)  # kept: old scripts
    ap.add_argument("--detail", default=None,
                    help="side file of full records (default gpurun_out/bench_detail_n<N>.json)")
    ap.add_argument("--deadline", type=float,
                    default=float(os.environ.get("DILOCO_BENCH_DEADLINE_S", "420")),
                    help="hard wall-clock bound of the whole run (s); side legs stop starting "
                         "at 70 %% of it")
    ap.add_argument("--child-legs", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--child-out", default=None, help=argparse.SUPPRESS)
    a = ap.parse_args()

    if a.child_legs == "cpu_baseline":  # one CPU process of the N > 1 CPU baseline
        ws, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
        timer = _Emitter(rank, a.deadline, heartbeat_s=0)
        dist.init_process_group("gloo", timeout=timedelta(minutes=3))
        r = cpu_baseline_dist(get_tree(a.tree), ws, rank)
        if rank == 0:
            with open(a.child_out + ".tmp", "w") as f:
                json.dump(r, f)
            os.replace(a.child_out + ".tmp", a.child_out)
        timer.done = True
        dist.barrier()
        dist.destroy_process_group()
        timer.timer.cancel()
        return
    if a.child_legs:  # one isolated child of isolated_legs
        ws, rank, dev = setup_dist(a.gpus)
        timer = _Emitter(rank, a.deadline, heartbeat_s=0)
        _lib.load()

        def dump(r):
            if rank == 0:
                with open(a.child_out + ".tmp", "w") as f:
                    json.dump(r, f)
                os.replace(a.child_out + ".tmp", a.child_out)

        peer_access_legs(get_tree(a.extra_tree), dev, ws, rank, a.steps,
                         (a.bucket_mb << 20) // 4, not a.no_parity, dump)
        timer.done = True
        if dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()
        timer.timer.cancel()
        return

    ws0 = int(os.environ.get("WORLD_SIZE", "1"))
    detail = a.detail or os.path.join(HERE, "gpurun_out", f"bench_detail_n{ws0}.json")
    em = _Emitter(int(os.environ.get("RANK", "0")), a.deadline, detail)
    soft = 0.7 * a.deadline
    ws, rank, dev = setup_dist(a.gpus)
    # child legs put a second process per rank on the GPU: with every rank on one GPU (a gloo
    # rehearsal) 2N + 1 processes (the launcher too) must stay within the box's 16 per GPU
    shared_gpu = ws > max(1, torch.cuda.device_count())
    children_fit = not shared_gpu or 2 * ws + 1 <= 16
    cap = (a.bucket_mb << 20) // 4
    _lib.load()
    spec = get_tree(a.tree)
    es = get_tree(a.extra_tree) if a.extra_tree not in ("none", a.tree) else None
    log(f"rank {rank}/{ws} tree {spec.name} ({spec.total()} params)")

    # the headline: the reference's four calls on the fused device outer model
    head = run_dropin(spec, dev, ws, rank, a.steps, a.warmup, cold=ws == 1 and not a.only_headline)
    workload = (f"DiLoCo outer step, {spec.name} tree per rank, through the reference's calls "
                "(src/train.py:263-269) on get_outer_model's default (CPU) outer model, stepped "
                "on its HBM twin: "
                + ("per bucket dl_delta_pack -> RCCL all_reduce (the default placement's "
                   "replicated exchange: .grad and the momentum local on every rank) -> "
                   "dl_unpack_sgd (/n, Nesterov SGD, copy to inner)" if ws > 1 else
                   "one dl_delta_pack_sgd per step (delta + outer.grad + Nesterov SGD + copy "
                   "to inner; no exchange at one replica, src/comm.py:118-119)"))
    meta = {"n_gpus": ws, "steps": a.steps, "warmup": a.warmup, "workload": workload}
    legs, parity, exch = {}, {}, {}
    cpu = None
    em.detail.update(headline=head, legs=legs, parity=parity, host=platform.node())
    em.build = lambda: assemble_line(meta, head, cpu, legs, parity, exch or None)
    log(f"headline done at {em.elapsed():.1f} s: {head['value']:.1f} GB/s")

    def leg(name, fn, *args, into=legs, always=False):
        """One side leg, in the same order on every rank; skipped (on every rank alike: the
        decision uses the max over ranks of the elapsed time) past the soft budget, unless
        `always` (the parity checks the line must carry)."""
        t = _max_over_ranks(em.elapsed(), dev, ws)
        if t > soft and not always:
            em.skipped.append(name)
            log(f"skipping {name}: {t:.0f} s elapsed > soft budget {soft:.0f} s")
            return None
        em.running = name
        r = _guard(fn, *args)
        if ws > 1 and dist.get_backend(dp_group(dev)) == "gloo":
            # gloo's pinned staging blocks of the leg just run (a private torch call: skipped
            # on a build without it)
            empty_host_cache = getattr(torch._C, "_host_emptyCache", None)
            if empty_host_cache is not None:
                empty_host_cache()
        into[name] = r
        log(f"{name} done at {em.elapsed():.1f} s")
        return r

    # the CPU baseline first after the headline (the line needs it; the side legs do not)
    if not a.no_cpu_baseline and not a.only_headline:
        em.running = "cpu_baseline"
        if ws == 1:
            cpu = _guard(cpu_baseline, spec)
        elif not children_fit:
            # every rank on one GPU (a gloo rehearsal): the rank processes run the N-core
            # baseline themselves (a child per rank would put 2N + 1 processes on the card)
            nthreads = torch.get_num_threads()
            cpu = _guard(cpu_baseline_dist, spec, ws, rank, 12.0, dist.new_group(backend="gloo"))
            torch.set_num_threads(nthreads)
        else:  # N CPU processes under gloo (one per rank, GPUs hidden), N cores
            cpu = isolated_legs(a, dev, ws, rank, 150.0, "cpu_baseline", HIDE_GPUS)
        em.detail["cpu_baseline"] = cpu
        log(f"cpu_baseline done at {em.elapsed():.1f} s")

    # then the parity the line must carry at any N, ahead of every side leg (a slow side leg
    # can no longer cost the line its parity): the f32 average against torch, and at N > 1
    # the headline path's exchanges behind the reference's calls against each other
    if not a.no_parity and not a.only_headline:
        leg("f32", parity_f32, dev, ws, rank, into=parity, always=True)
        if ws > 1:
            leg("dropin_exchanges", parity_dropin_exchanges, dev, ws, rank, into=parity,
                always=True)

    if not a.only_headline:
        if ws == 1:
            leg(f"{spec.name}_engine", run_engine, spec, dev, ws, rank, a.steps, a.warmup,
                torch.float32, cap, True, None, "rccl", True)
            if es is not None:
                ks = max(3, a.steps // 4)
                leg(f"{es.name}_dropin", run_dropin, es, dev, ws, rank, ks, 1)
                leg(f"{es.name}_bf16", run_engine, es, dev, ws, rank, ks, 1, torch.bfloat16, cap,
                    False)
                leg(f"{es.name}_int8", run_q8, es, dev, ws, rank, ks, 1, cap)
            leg(f"{spec.name}_dropin_device", run_dropin, spec, dev, ws, rank, a.steps,
                a.warmup, "f32", None, None, False, False, "device")
            leg(f"{spec.name}_dropin_synced", run_dropin, spec, dev, ws, rank, 30, 1, "f32",
                None, None, False, True)
            leg("dropin_pcie", dropin_pcie, spec, dev, ws, rank, 5)
        else:
            if es is not None:
                # first: the north star's N > 1 figure -- the 1.3B bucket set through the calls
                # against RCCL's own all_reduce of the same bytes, this node, this run
                ks = max(3, a.steps // 4)
                # get_outer_model's default placement, as the headline: the CPU outer model
                # holds 4 B/param resident per rank (its θ; the pageable .grad / momentum
                # arenas fill only when read), 5.3 GB at 1.3B. A gloo rehearsal with
                # every rank on one GPU keeps these outer models in HBM instead: gloo stages
                # each rank's whole 1.3B wire and θ through pinned host memory as well (cached
                # in power-of-two blocks), which eight ranks on one box cannot also hold
                # (with the default placement's exchange, replicated: RCCL's all_reduce itself)
                p13 = "device" if shared_gpu else None
                x13 = "replicated" if shared_gpu else None
                r13 = leg(f"{es.name}_dropin", run_dropin, es, dev, ws, rank, ks, 1, "f32", None,
                          x13, False, False, p13)
                ref13 = leg(f"rccl_ref_{es.name}", rccl_reference, dev, ws, rank,
                            es.total() // (64 * ws) * (64 * ws), 3, into=em.detail)
                e = exchange_efficiency(r13, ref13, ws)
                if e:
                    exch[es.name] = e
            ref = leg(f"rccl_ref_{spec.name}", rccl_reference, dev, ws, rank,
                      head["padded"] // (64 * ws) * (64 * ws), into=em.detail)
            e = exchange_efficiency(head, ref, ws)
            if e:
                exch[spec.name] = e
            for ex in ("sharded", "a2a"):  # the opt-in exchanges (the headline is replicated)
                leg(f"{spec.name}_dropin_{ex}", run_dropin, spec, dev, ws, rank, a.steps,
                    a.warmup, "f32", None, ex)
            leg(f"{spec.name}_engine", run_engine, spec, dev, ws, rank, a.steps, a.warmup,
                torch.float32, cap)
            if es is not None:
                leg(f"{es.name}_dropin_bf16", run_dropin, es, dev, ws, rank, ks, 1, "bf16", None,
                    x13, False, False, p13)
                leg(f"{es.name}_dropin_int8", run_dropin, es, dev, ws, rank, ks, 1, "int8", None,
                    x13, False, False, p13)
            leg(f"{spec.name}_grad_sync", gradsync_rate, spec, dev, ws, rank, max(3, a.steps // 2))
            if ws >= 4 and ws % 2 == 0:
                leg(f"{spec.name}_two_stages", run_two_stages, spec, dev, ws, rank, a.steps,
                    a.warmup, cap)
        if not a.no_parity:
            leg("bf16", codec_parity, get_tree("tiny"), dev, ws, rank, 1 << 20, into=parity)
            leg("int8", parity_q8, dev, ws, rank, into=parity)
            leg("sharded", parity_sharded, dev, ws, rank, into=parity)
            leg("a2a", parity_sharded, dev, ws, rank, "a2a", into=parity)
            if ws > 1:
                if es is not None:
                    nt = len(es.params())
                    leg(f"bf16_{es.name}", codec_parity, es, dev, ws, rank, cap,
                        [0] + list(range(1, 10)) + [nt - 1], into=parity)
        if ws > 1 and not a.no_xgmi and es is not None:
            if not children_fit:
                em.skipped.append("peer_access_legs (one GPU shared by all ranks)")
            else:
                left = a.deadline - _max_over_ranks(em.elapsed(), dev, ws) - 15
                if left < 60:
                    em.skipped.append("peer_access_legs")
                else:
                    em.running = "peer_access_legs (child processes)"
                    r = isolated_legs(a, dev, ws, rank, min(240.0, left), "peer")
                    if "legs" in r:
                        legs.update(r["legs"])
                        parity.update(r["parity"])
                    else:
                        legs["peer_access_legs"] = r
                    log(f"peer_access_legs done at {em.elapsed():.1f} s")
    em.running = "teardown"
    em.emit()
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    em.timer.cancel()


if __name__ == "__main__":
    main()
