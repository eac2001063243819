#!/usr/bin/env python3
"""Benchmark: DiLoCo outer step, device-resident, GB/s of parameters reduced.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--tree t125] [--wire f32|bf16]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

One step = one full outer step of src/train.py:261-269 over the whole synthetic tree on every
rank, device-resident (θ_outer, momentum and the wire buffer live in HBM), made through the
reference's own calls -- compute_pseudo_gradient -> TrainingComm.sync_gradients ->
outer_optimizer.step() -> sync_inner_model (diloco_amd's drop-in modules, src/train.py
untouched) on the fused device outer model (get_outer_model(..., placement="device")):
    N = 1  one dl_delta_pack_sgd (wire = outer.grad = θ_outer - inner, Nesterov SGD, inner = θ)
           (BASELINE config #2's delta + pack, plus the SGD and copy-back the step needs)
    N > 1  per bucket dl_delta_pack -> RCCL all_reduce, then dl_unpack_sgd (/n, SGD, inner = θ)
The engine behind the fast path (OuterSync.step: N = 1 the same one-pass kernel; N > 1
dl_delta_pack -> RCCL reduce_scatter -> dl_shard_sgd -> all_gather(θ) -> dl_scatter) is timed
beside it ("extra.<tree>_engine", with its per-kernel, cold and back-to-back figures).
Same tree per rank at every N (weak scaling). value = 4 * params / t_step (SURVEY.md §8d:
"GB/s params reduced" = the bytes of ONE parameter tree reduced per DP step; max time over
ranks); the weak-scaling aggregate N * 4 * params / t_step is reported beside it as
"value_aggregate". At N = 1 the step is also timed cold (the 256 MiB Infinity Cache scrubbed
between steps, outside the timed events: in training H inner steps run in between) next to
the back-to-back (warm) rate, and a flat copy kernel of the same access shape gives the
same-run copy ceiling the roofline fractions are also read against.
Rank 0 prints ONE JSON line: the headline with its roofline kernel (HIP events, PMC traffic
from profiles/) and the CPU baseline (N = 1), then side legs (other trees and wires, the
one-pass kernel, parity self-checks, drop-in rates, and at N > 1 the replicated variant,
RCCL's own all_reduce rate, the two-stage layout; last, in isolated child processes, the
direct peer-access exchange, the link probe, the device p2p transport and RCCL setting
variants). A watchdog bounds the run (--deadline): the line is printed whatever a side leg
does.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import platform
import subprocess
import sys
import time
from datetime import timedelta

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


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


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
    # (RCCL refuses two ranks per device); the driver's multi-GPU runs use RCCL.
    backend = os.environ.get("DILOCO_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local %= max(1, torch.cuda.device_count())
        # the drop-in legs' DP group (TrainingComm.dp_group) too
        os.environ.setdefault("DILOCO_DP_BACKEND", "gloo")
        if "diloco_amd.comm" in sys.modules:
            sys.modules["diloco_amd.comm"].DP_BACKEND = os.environ["DILOCO_DP_BACKEND"]
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if ws > 1:
        # a hung collective becomes an error after 5 minutes instead of the 10-minute default
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, timeout=timedelta(minutes=5), **kw)
    return ws, rank, dev


def build(spec, dev, rank, wire, cap, fuse=False, shard=None, exchange="rccl", tile=None,
          group=None, keep_wire=False):
    shapes = [s for _, s in spec.params()]
    theta0 = synth.outer_tree_device(spec, dev)
    params = [t.view(s) for t, s in zip(theta0, shapes)]
    eng = OuterSync(params, lr=0.7, momentum=0.9, nesterov=True, wire_dtype=wire,
                    bucket_cap_elems=cap, fuse_single=fuse, shard=shard, exchange=exchange,
                    group=group, keep_wire=keep_wire,
                    **({} if tile is None else {"tile_chunks": tile}))
    # inner = θ_0 + this rank's noise (stands in for H inner steps)
    synth.inner_tree_device([p.view(-1) for p in params], 1, rank, out=[p.view(-1) for p in params])
    return eng


def _max_over_ranks(x, dev, ws):
    if ws == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _sync(ws):
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()


def kernel_entry(bytes_per_launch, ms, traffic=None, bound="hbm", peak=HBM_PEAK_GBS, rw=None):
    """rw = (read bytes, read streams, write bytes, write streams) per launch: the kernel's
    byte mix, read against the same-run read and write ceilings by with_copy_ceiling."""
    ach = bytes_per_launch / (ms * 1e-3) / 1e9
    e = {"bound": bound, "achieved": round(ach, 1), "peak": peak, "unit": "GB/s",
         "frac": round(ach / peak, 4), "traffic": round(traffic) if traffic else None,
         "bytes_per_launch": bytes_per_launch, "avg_ms": round(ms, 5)}
    if rw is not None:  # (read bytes, read streams, write bytes, write streams)
        e["read_bytes"], e["read_streams"] = int(rw[0]), int(rw[1])
        e["write_bytes"], e["write_streams"] = int(rw[2]), int(rw[3])
    return e


SCRUB_MIB = 512  # >= 2 x the 256 MiB Infinity Cache moved per scrub (read 512 + write 512)


class Scrubber:
    """Evicts the step's bytes from the Infinity Cache (and every L2) between cold steps:
    a default-policy dl_copy of SCRUB_MIB MiB (1 GiB of traffic), enqueued outside the timed
    events. In training H inner steps (forward/backward over far more than 256 MiB) run
    between two outer steps, so the cold figure is the one a DiLoCo run sees."""

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


def copy_ceiling(dev, mib=1024, reps=15):
    """What the memory system gives streaming kernels on this box in this run, `reps` launches
    back to back over `mib` MiB (far beyond the Infinity Cache), each in the walker's access
    shape (dl_copy): a two-stream copy -- default and non-temporal policy, 4 (the walker's
    shape) and 8 float4 loads in flight per lane; the fastest is the copy ceiling the roofline
    fractions are read against beside the 8 TB/s spec peak (boxes differ by ~15 %) -- and the
    pure read and pure write rates over 1-4 streams (DL_COPY_READ / DL_COPY_WRITE), which
    bound a kernel of R bytes read from s_r buffers and W written to s_w at
    t >= R / read_GBs[s_r] + W / write_GBs[s_w]: the mix ceiling (tools/rw_mix.hip, DESIGN.md
    §3 -- HBM writes are the slower half). Rates use the median launch."""
    n = (mib << 20) // 4
    a = torch.ones(n, device=dev)
    b = torch.empty(n, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    out = {"bytes_per_copy": 2 * 4 * n}
    nt, wide = _lib.TUNE_NT_LOADS, _lib.COPY_WIDE

    def rate(flags, moved, nbytes=4 * n):
        """moved bytes / the median duration of `reps` back-to-back launches (events on the
        launching stream around each)"""
        _lib.call("dl_copy", a.data_ptr(), b.data_ptr(), nbytes, flags, st)  # warm the launch
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        ev[0].record()
        for i in range(reps):
            src, dst = (a, b) if i % 2 == 0 else (b, a)
            _lib.call("dl_copy", src.data_ptr(), dst.data_ptr(), nbytes, flags, st)
            ev[i + 1].record()
        ev[-1].synchronize()
        ms = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(reps))[reps // 2]
        return round(moved / (ms * 1e-3) / 1e9, 1)

    for name, flags in (("plain", 0), ("nt", nt), ("plain_x8", wide), ("nt_x8", nt | wide)):
        out[f"{name}_GBs"] = rate(flags, 2 * 4 * n)
    out["GBs"] = max(v for k, v in out.items() if k.endswith("_GBs"))
    # pure read / pure write over 1-4 streams (the walker kernels read 1-3 and write 1-4
    # buffers; default and non-temporal policy, the faster of the two)
    for kind, flag in (("read", _lib.COPY_READ), ("write", _lib.COPY_WRITE)):
        out[f"{kind}_GBs"] = {}
        for k in (1, 2, 3, 4):
            nb = 4 * n // (16 * k) * (16 * k)  # k equal streams of whole float4s
            out[f"{kind}_GBs"][k] = max(rate(f | flag | _lib.COPY_STREAMS(k), nb, nb)
                                        for f in (0, nt))
    del a, b
    torch.cuda.empty_cache()
    return out


def with_copy_ceiling(entry, ceiling):
    """A kernel_entry with its achieved rate also read against the same-run copy ceiling and,
    for an entry that carries its byte mix, the same-run mix ceiling
    (R + W) / (R / read_GBs + W / write_GBs)."""
    if entry is None or not isinstance(ceiling, dict) or not ceiling.get("GBs"):
        return entry
    e = dict(entry)
    e["copy_ceiling"] = ceiling["GBs"]
    e["frac_vs_copy"] = round(e["achieved"] / ceiling["GBs"], 4)
    r, w = e.get("read_bytes"), e.get("write_bytes")
    rg, wg = ceiling.get("read_GBs"), ceiling.get("write_GBs")
    if r is not None and rg and wg:
        sr, sw = e["read_streams"], e["write_streams"]
        t = (r / rg[sr] if r else 0.0) + (w / wg[sw] if w else 0.0)
        e["mix_ceiling"] = round((r + w) / t, 1)
        e["frac_vs_mix"] = round(e["achieved"] * t / (r + w), 4)
    if max(e["frac_vs_copy"], e.get("frac_vs_mix", 0.0)) > 1.0:
        # the probes are reference rates of simpler access shapes, not bounds for this one
        e["ceiling_exceeded"] = True
        e["ceiling_note"] = ("fraction above 1: the same-run probes (a 2-stream 1 GiB dl_copy; "
                             "1-4-stream pure reads / writes) are reference rates of simpler "
                             "access shapes, not bounds: a kernel with more streams can run "
                             "above them, warm (Infinity-Cache reuse between back-to-back "
                             "launches) and cold with its own write-back charged "
                             "(cold.flushed_step_ms) alike. The roofline is `peak`")
    return e


def run_tree(spec, dev, ws, rank, steps, warmup, wire, cap, fuse=False, b2b_loops=True,
             shard=None, exchange="rccl", tile=None, cold=False, keep_wire=False):
    """Timed region (K outer steps, nothing else on the stream), then an instrumented pass of
    K more steps with HIP events between the kernels on the stream they run on (events in the
    timed region would cost the step ~35 us each), then the same kernels back to back."""
    eng = build(spec, dev, rank, wire, cap, fuse, shard, exchange, tile, keep_wire=keep_wire)
    P = spec.total()
    for _ in range(max(warmup, 1)):  # >= 1: the timed steps run the steady-state SGD mode
        eng.step()
    _sync(ws)
    # two events on the step's stream bracket the timed loop (inside the wall-clock brackets,
    # none between steps): the loop's GPU span, <= the wall time by construction
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
    single = ws == 1
    # instrumented pass (the kernels in their in-step context)
    # the kernels are timed on the stream they run on: eng._step launches on the current
    # stream (eng.step would hop to the engine's side stream and back, ~20-30 us of
    # cross-stream latency inside the events)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for e in ev:
        e[0].record()
        if single and fuse:
            eng._step(None)
            e[1].record()
        elif single:
            eng.pseudo_gradient()
            e[1].record()
            eng.apply()
            eng.steps_done += 1
        else:
            eng.step()
            e[1].record()
        e[2].record()
    torch.cuda.synchronize()
    first = sum(e[0].elapsed_time(e[1]) for e in ev) / steps
    second = sum(e[1].elapsed_time(e[2]) for e in ev) / steps
    warm_span = sum(e[0].elapsed_time(e[2]) for e in ev) / steps
    pmc = load_pmc(spec.name) if wire == torch.float32 else {}
    res = {"tree": spec.name, "params": P, "tensors": len(spec.params()),
           "padded": eng.tree.total, "buckets": eng.tree.n_buckets, "chunks": eng.tree.n_chunks,
           "ms_per_step": dt / steps * 1e3, "value": 4.0 * P / (dt / steps) / 1e9,
           "loop_gpu_ms_per_step": round(loop_ms, 5),
           "value_aggregate": ws * 4.0 * P / (dt / steps) / 1e9,
           "wire": "bf16" if wire == torch.bfloat16 else "f32",
           "tile_chunks": eng.tile_chunks if single and not fuse else None,
           "variant": ("one replica: dl_delta_pack_sgd (one pass, pseudo-gradient kept in the "
                       "packed wire)" if single and fuse and keep_wire
                       else "one replica: dl_delta_sgd (one pass, no wire)" if single and fuse
                       else "direct exchange from the peers' inner arenas (dl_xgmi_delta_sgd)"
                       if eng.xgmi_inner
                       else ("one replica: dl_delta_pack -> dl_unpack_sgd"
                             + (f", tiles of {eng.tile_chunks} chunks" if eng.tile_chunks
                                else ", whole-range launches")) if single
                       else "direct peer-access exchange (IPC, dl_xgmi_reduce_sgd)" if eng.xgmi
                       else "all_to_all -> rank-order reduce + shard SGD (dl_shard_reduce_sgd) "
                            "-> all_gather" if eng.a2a
                       else "reduce_scatter -> shard SGD -> all_gather" if eng.sharded
                       else "all_reduce -> replicated SGD")}
    fused_name = "delta_pack_sgd" if keep_wire else "delta_sgd"
    # read θ, inner, buf; write θ, buf, inner (+ the wire)
    fused_bytes = (24 + (wb if keep_wire else 0)) * P
    fused_rw = (12 * P, 3, fused_bytes - 12 * P, 4 if keep_wire else 3)
    pack_rw, unpack_rw = (8 * P, 2, wb * P, 1), ((wb + 8) * P, 3, 12 * P, 3)
    if single and fuse:
        res["kernels"] = {fused_name: kernel_entry(fused_bytes, first, pmc.get(fused_name),
                                                   rw=fused_rw)}
    elif single:
        res["kernels"] = {
            "delta_pack": kernel_entry((8 + wb) * P, first, pmc.get("delta_pack"), rw=pack_rw),
            "unpack_sgd": kernel_entry((wb + 20) * P, second, pmc.get("unpack_sgd"),
                                       rw=unpack_rw),
        }
    else:
        res["step_ms_instrumented"] = round(first, 4)
    if single and cold:
        # cold: the same kernels with the Infinity Cache scrubbed before every step (outside
        # the events), as after H inner steps in training
        scr = Scrubber(dev)
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
        tiled = not fuse and eng.tile_chunks
        for e in ev:
            scr()
            e[0].record()
            if fuse or tiled:  # the step as the engine runs it, on this stream
                eng._step(None)
                e[1].record()
            else:
                eng.pseudo_gradient()
                e[1].record()
                eng.apply()
                eng.steps_done += 1
            e[2].record()
        torch.cuda.synchronize()
        # The end event of a cold step fires when its kernels end, with written lines possibly
        # still dirty in the Infinity Cache (their HBM write-back lands during the next
        # scrub). "flushed": K (scrub, step) cycles plus a closing scrub, as one span, minus
        # K + 1 scrubs alone -- the step charged with its own write-back.
        def cycles(with_step):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            scr()
            e0.record()
            for _ in range(steps):
                scr()
                if with_step:
                    if fuse or tiled:
                        eng._step(None)
                    else:
                        eng.pseudo_gradient()
                        eng.apply()
                        eng.steps_done += 1
            scr()
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1)

        scrub_only = min(cycles(False) for _ in range(2))
        flushed_ms = max(cycles(True) - scrub_only, 1e-6) / steps
        scr.close()
        c_first = sum(e[0].elapsed_time(e[1]) for e in ev) / steps
        c_second = sum(e[1].elapsed_time(e[2]) for e in ev) / steps
        c_step = sum(e[0].elapsed_time(e[2]) for e in ev) / steps
        res["cold"] = {"step_ms": round(c_step, 5), "value": 4.0 * P / (c_step * 1e-3) / 1e9,
                       # the same event span in the warm instrumented pass: the like-for-like
                       # comparison (the headline value is wall-clock, gaps between steps in)
                       "warm_step_ms": round(warm_span, 5),
                       "warm_value": 4.0 * P / (warm_span * 1e-3) / 1e9,
                       "flushed_step_ms": round(flushed_ms, 5),
                       "flushed_value": 4.0 * P / (flushed_ms * 1e-3) / 1e9,
                       "note": "Infinity Cache scrubbed before each step (512 MiB copy, "
                               "outside the events); step = the kernels' event span, no "
                               "inter-step gap (compare warm_step_ms, not the headline); "
                               "flushed = (scrub + step) cycles minus scrubs alone, the "
                               "step's deferred HBM write-back included"}
        if fuse:
            res["cold"]["kernels"] = {fused_name: kernel_entry(fused_bytes, c_first, rw=fused_rw),
                                      fused_name + "_flushed": kernel_entry(
                                          fused_bytes, flushed_ms, rw=fused_rw)}
        elif tiled:
            res["cold"]["kernels"] = {}  # tile-interleaved launches: the step only
        else:
            res["cold"]["kernels"] = {
                "delta_pack": kernel_entry((8 + wb) * P, c_first, rw=pack_rw),
                "unpack_sgd": kernel_entry((wb + 20) * P, c_second, rw=unpack_rw)}
    # the same kernels back to back (cold inputs: no Infinity-Cache reuse across kernels)
    reps = max(steps, 10)

    def b2b(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / reps

    if b2b_loops and single and fuse:
        res["kernels_b2b"] = {fused_name: kernel_entry(fused_bytes,
                                                        b2b(lambda: eng._step(None)),
                                                        rw=fused_rw)}
    elif b2b_loops and not (eng.sharded or eng.xgmi):
        res["kernels_b2b"] = {"delta_pack": kernel_entry((8 + wb) * P, b2b(eng.pseudo_gradient),
                                                         rw=pack_rw),
                              "unpack_sgd": kernel_entry((wb + 20) * P, b2b(eng.apply),
                                                         rw=unpack_rw)}
    if single and fuse:
        # one kernel per step: its average launch duration is the timed loop's own GPU span
        # / K (the rocprofv3 average of the same command agrees, profiles/), never above
        # ms_per_step; the instrumented pass's figure stays under "kernels"
        res["roofline"] = dict(kernel_entry(fused_bytes, loop_ms, pmc.get(fused_name),
                                            rw=fused_rw),
                               kernel=fused_name, timing="timed loop GPU span / K")
    elif single:
        ks = res["kernels"]
        dom = max(ks, key=lambda k: ks[k]["avg_ms"])
        res["roofline"] = dict(ks[dom], kernel=dom, timing="instrumented pass (events between "
                                                          "the step's kernels)")
    elif eng.xgmi:
        # the exchange kernel moves (n-1)/n·4P in (peer wires) and (n-1)/n·4P out (θ stores);
        # over the whole step time this is a lower bound on its xGMI rate
        bus = 2.0 * (ws - 1) / ws * 4 * eng.tree.total
        res["roofline"] = dict(kernel_entry(bus, dt / steps * 1e3, bound="xgmi",
                                            peak=(ws - 1) * XGMI_LINK_GBS),
                               kernel="dl_xgmi_reduce_sgd (whole step, lower bound)",
                               bus_bytes_per_step=bus)
    else:
        def collectives_all():
            for b in range(eng.tree.n_buckets):
                if eng.sharded:
                    eng.reduce_scatter(b, async_op=False)
                    eng.all_gather(b, async_op=False)
                else:
                    eng.all_reduce(b, async_op=False)

        reps_ar = max(3, steps // 2)
        _sync(ws)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps_ar):
            collectives_all()
        e1.record()
        e1.synchronize()
        ar_ms = _max_over_ranks(e0.elapsed_time(e1) / reps_ar, dev, ws)
        # all-reduce: 2(n-1)/n · wire bytes; sharded: (n-1)/n · wire (RS) + (n-1)/n · 4 B (AG of θ)
        frac = (ws - 1) / ws * eng.tree.total
        bus = frac * (wb + 4) if eng.sharded else 2.0 * frac * wb
        name = ("rccl all_to_all + all_gather (all buckets, back to back)" if eng.a2a
                else "rccl reduce_scatter + all_gather (all buckets, back to back)" if eng.sharded
                else "rccl all_reduce (all buckets, back to back)")
        res["roofline"] = dict(kernel_entry(bus, ar_ms, bound="xgmi",
                                            peak=(ws - 1) * XGMI_LINK_GBS),
                               kernel=name, bus_bytes_per_step=bus)
    eng.close()
    del eng
    torch.cuda.empty_cache()
    return res


def parity_check(dev, ws, rank, wire):
    """The HIP (+ RCCL at N > 1) path against a plain torch fp32 statement of the same step
    on the tiny tree with 3 buckets. fp32 wire: averaged deltas normwise <= 1e-6 (north-star
    tolerance). bf16 wire: the codec error vs the exact fp32 average, bound n*2^-8. Both: every
    replica bit-identical after the full step."""
    spec = get_tree("tiny")
    eng = build(spec, dev, rank, wire, 1 << 20, shard=False)
    nb = eng.tree.n_buckets
    for b in range(nb):
        eng.pseudo_gradient(b)
        if ws > 1:
            eng.all_reduce(b, async_op=False)
    got = [t.float().reshape(-1) / ws for t in eng.unpacked(eng.wire)]
    theta0 = synth.outer_tree_device(spec, dev)
    acc = [torch.zeros_like(t) for t in theta0]
    for r in range(ws):  # every rank's inner, regenerated locally (counter-based)
        inner_r = synth.inner_tree_device(theta0, 1, r)
        acc = [a + (t - i) for a, t, i in zip(acc, theta0, inner_r)]
    worst = 0.0
    for g, a in zip(got, acc):
        ref = a / ws
        scale = float(ref.abs().max().clamp_min(1e-30))
        worst = max(worst, float((g - ref).abs().max()) / scale)
    for b in range(nb):
        eng.apply(b)
    eng.steps_done += 1
    torch.cuda.synchronize()
    bits = eng.theta.view(torch.int32).to(torch.int64).sum()
    ck = torch.stack([bits, -bits])
    if ws > 1:
        dist.all_reduce(ck, op=dist.ReduceOp.MAX)
    identical = bool(ck[0].item() == -ck[1].item())
    # bf16: unit roundoff 2^-8 for the cast, plus one rounding per partial sum of the
    # collective's bf16 reduction (at most ws - 1 of them)
    tol = 1e-6 if wire == torch.float32 else ws * 2.0 ** -8
    eng.close()
    return {"tree": "tiny", "buckets": nb, "wire": "f32" if wire == torch.float32 else "bf16",
            "avg_delta_normwise_err": worst, "tolerance": tol,
            "replicas_identical": identical, "ok": bool(worst <= tol and identical)}


def run_two_stages(spec, dev, ws, rank, steps, warmup, cap):
    """The reference's two-stage SWARM layout (src/world.py:96-97, stage = rank % 2): two
    disjoint DP groups of ws/2 ranks run their sharded outer steps at the same time, each over
    its own RCCL communicator. value = ws · 4P / t_step (every rank steps a full
    tree), max over all ranks."""
    groups = [dist.new_group([r for r in range(ws) if r % 2 == s]) for s in range(2)]
    g = groups[rank % 2]
    eng = build(spec, dev, rank, torch.float32, cap, group=g)
    for _ in range(max(warmup, 1)):
        eng.step()
    _sync(ws)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.step()
    _sync(ws)
    dt = _max_over_ranks(time.perf_counter() - t0, dev, ws)
    res = {"tree": spec.name, "stages": 2, "dp_per_stage": ws // 2,
           "ms_per_step": dt / steps * 1e3,
           # two trees (one per stage group) reduced per step
           "value": 2 * 4.0 * spec.total() / (dt / steps) / 1e9,
           "value_aggregate": ws * 4.0 * spec.total() / (dt / steps) / 1e9,
           "variant": "reduce_scatter -> shard SGD -> all_gather" if eng.sharded
           else "all_reduce -> replicated SGD"}
    eng.close()
    del eng
    torch.cuda.empty_cache()
    return res


def rccl_reference(dev, ws, rank, elems, reps=5):
    """What RCCL itself reaches on this node for the headline's bytes: one fp32 all_reduce
    (SUM) of `elems` elements, and a reduce_scatter + all_gather pair of the same size,
    back to back, max over ranks. busBW = 2(n-1)/n · bytes / t (the nccl-tests convention,
    SURVEY §8d): the measured 'algorithmic all-reduce bandwidth' the exchange is held to."""
    out = {}
    if dist.get_backend() == "gloo":
        # a gloo rehearsal on one GPU (DILOCO_BENCH_BACKEND=gloo) stages whole tensors through
        # host memory in every rank: 8 ranks x several copies of a 5 GB tree exceed the box's
        # host-memory cap, and the rate would be gloo's anyway
        cap = (256 << 20) // 4 // (64 * ws) * (64 * ws)
        if elems > cap:
            out["capped_for_gloo_elems"] = elems
            elems = cap
    x = torch.ones(elems, device=dev)
    sh = torch.empty(elems // ws, device=dev)
    for name in ("all_reduce", "reduce_scatter+all_gather"):
        for it in range(reps + 1):
            if it == 1:  # first call warms the communicator's buffers
                _sync(ws)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
            if name == "all_reduce":
                dist.all_reduce(x)
            else:
                dist.reduce_scatter_tensor(sh, x)
                dist.all_gather_into_tensor(x, sh)
        e1.record()
        e1.synchronize()
        ms = _max_over_ranks(e0.elapsed_time(e1) / reps, dev, ws)
        bus = 2.0 * (ws - 1) / ws * 4 * elems
        out[name] = {"ms": round(ms, 4), "busbw_GBs": round(bus / (ms * 1e-3) / 1e9, 1)}
    out["bytes"] = 4 * elems
    return out


def xgmi_link_probe(dev, ws, rank, reps=5, mib=256):
    """Peer read rates through IPC-mapped buffers (what the 153 GB/s per link
    means): every rank at once reads `mib` MiB from its ring neighbour (one direction of one
    link each), then `mib` MiB from every peer at once (all links incoming), then the same
    amount from its own HBM; max time over ranks."""
    import ctypes

    import numpy as np

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
    _lib.call("dl_sys_fence", stream)  # no stale copies of peers' lines in this GPU's L2
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
    ok = bool(torch.equal(dst[:n], want))  # the peer's bytes arrived intact
    del want
    peers = [int(tab[q]) for q in range(ws) if q != rank]
    allp = timed(peers)
    local = timed([int(tab[rank])])
    _sync(ws)
    pm.close()
    _sync(ws)
    return {"bytes_per_source": n * 4, "one_peer_read_GBs": one,
            "all_peers_read_GBs": allp, "local_hbm_read_GBs": local, "peers": ws - 1,
            "note": "read rate per rank (GB/s of source bytes), all ranks concurrently; "
                    "one_peer = ring neighbour = one direction of one link", "ok": ok}


def parity_xgmi(dev, ws, rank, exchange="xgmi"):
    """The direct exchange (exchange='xgmi') against the RCCL sharded step on the tiny tree,
    2 outer steps: θ and momentum normwise <= 1e-6 per tensor (bit-exact at n <= 2; the direct
    exchange sums in rank order, RCCL in its own order), inner == θ, replicas identical."""
    spec = get_tree("tiny")
    ea = build(spec, dev, rank, torch.float32, 1 << 20, exchange=exchange)
    eb = build(spec, dev, rank, torch.float32, 1 << 20)
    for s in (1, 2):
        for e in (ea, eb):
            if s > 1:
                th = [t.reshape(-1) for t in e.unpacked(e.theta)]
                synth.inner_tree_device(th, s, rank, out=[p.view(-1) for p in e.params])
            e.step()
    torch.cuda.synchronize()
    worst, exact = 0.0, True
    ma, mb = ea.momentum_full(), eb.momentum_full()
    for x, y in ((ea.theta, eb.theta), (ma, mb)):
        for a, b in zip(ea.unpacked(x), eb.unpacked(y)):
            exact &= bool(torch.equal(a, b))
            scale = float(b.abs().max().clamp_min(1e-30))
            worst = max(worst, float((a - b).abs().max()) / scale)
    inner_ok = all(torch.equal(p, t) for p, t in zip(ea.params, ea.unpacked(ea.theta)))
    bits = ea.theta.view(torch.int32).to(torch.int64).sum()
    ck = torch.stack([bits, -bits])
    if ws > 1:
        dist.all_reduce(ck, op=dist.ReduceOp.MAX)
    identical = bool(ck[0].item() == -ck[1].item())
    ea.close()
    eb.close()
    return {"tree": "tiny", "steps": 2, "xgmi_vs_rccl_normwise_err": worst, "bit_exact": exact,
            "tolerance": 1e-6, "inner_is_theta": inner_ok, "replicas_identical": identical,
            "ok": bool(worst <= 1e-6 and identical and inner_ok)}


def parity_sharded(dev, ws, rank, exchange="rccl", wire=torch.float32):
    """The sharded step (reduce-scatter -> dl_shard_sgd -> all-gather -> dl_scatter; with
    exchange="a2a" all_to_all -> dl_shard_reduce_sgd -> all-gather) against the replicated one
    (all-reduce -> dl_unpack_sgd, fp32 wire) on the tiny tree, 2 outer steps: θ, momentum and
    inner normwise <= 1e-6 per tensor (bit-exact where the two sum in the same order; a bf16
    wire within 2^-8 of the fp32 step, the codec's one rounding -- the a2a reduce never
    re-rounds the sum), every replica bit-identical."""
    spec = get_tree("tiny")
    ea = build(spec, dev, rank, wire, 1 << 20, shard=True, exchange=exchange)
    eb = build(spec, dev, rank, torch.float32, 1 << 20, shard=False)
    for s in (1, 2):
        for e in (ea, eb):
            if s > 1:
                th = [t.reshape(-1) for t in e.unpacked(e.theta)]
                synth.inner_tree_device(th, s, rank, out=[p.view(-1) for p in e.params])
            e.step()  # N = 1: local shard copies vs the two-kernel step
    torch.cuda.synchronize()
    worst, exact = 0.0, True
    ma, mb = ea.momentum_full(), eb.momentum_full()
    for x, y in ((ea.theta, eb.theta), (ma, mb)):
        exact &= bool(torch.equal(x, y))
        for a, b in zip(ea.unpacked(x), eb.unpacked(y)):
            scale = float(b.abs().max().clamp_min(1e-30))
            worst = max(worst, float((a - b).abs().max()) / scale)
    inner_ok = all(torch.equal(p, t) for p, t in zip(ea.params, ea.unpacked(ea.theta)))
    bits = ea.theta.view(torch.int32).to(torch.int64).sum()
    ck = torch.stack([bits, -bits])
    if ws > 1:
        dist.all_reduce(ck, op=dist.ReduceOp.MAX)
    identical = bool(ck[0].item() == -ck[1].item())
    buckets = ea.tree.n_buckets
    ea.close()
    eb.close()
    tol = 1e-6 if wire == torch.float32 else 2.0 ** -8
    return {"tree": "tiny", "buckets": buckets, "steps": 2, "exchange": exchange,
            "wire": "bf16" if wire == torch.bfloat16 else "f32",
            "sharded_vs_replicated_normwise_err": worst, "bit_exact": exact,
            "tolerance": tol, "inner_is_theta": inner_ok, "replicas_identical": identical,
            "ok": bool(worst <= tol and identical and inner_ok)}


def codec_error(spec, dev, ws, rank, cap):
    """The bf16 wire's error at this N on the named 1.3B tree: one outer
    step (the first: buf = g) through the real exchange -- the replicated RCCL bf16 all-reduce
    (the bf16 default) and the ordered exchange (exchange="a2a": bf16 slices summed in fp32 in
    rank order) -- against the fp32 statement of the same step in torch on sampled tensors
    (wte whole, block 0's tensors, the last tensor). Reported: the normwise error of the
    applied update, max|u_bf16 - u_fp32| / max|u_fp32|, and its worst ratio to the per-element
    a-priori bound (diloco_amd.outer.bf16_codec_bound, <= 1 required)."""
    from diloco_amd.outer import U_F32, bf16_codec_bound

    nt = len(spec.params())
    picks = [0] + list(range(1, 10)) + [nt - 1]
    out = {"tree": spec.name, "n": ws, "tensors": picks, "step": 1}
    for name, kw in (("rccl_bf16_allreduce", dict(shard=False)),
                     ("a2a_fp32_sum", dict(shard=None, exchange="a2a"))):
        eng = build(spec, dev, rank, torch.bfloat16, cap, **kw)
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
            bound = (0.7 * 1.9 * bf16_codec_bound(sabs, ws, "a2a" if "a2a" in name else "rccl")
                     + 4 * U_F32 * (x0.abs() + th1[t].reshape(-1).abs() + 2 * u32.abs()))
            worst_norm = max(worst_norm, float(err.max()) / max(float(u32.abs().max()), 1e-30))
            worst_ratio = max(worst_ratio, float((err / bound).max()))
            del sabs, g, u32, ubf, err, bound
        out[name] = {"normwise_update_err": worst_norm,
                     "max_err_over_bound": round(worst_ratio, 4),
                     "ok": bool(worst_ratio <= 1.0)}
        eng.close()
        del eng, th0, th1
        torch.cuda.empty_cache()
    out["ok"] = all(out[k]["ok"] for k in ("rccl_bf16_allreduce", "a2a_fp32_sum"))
    out["note"] = ("bf16 default at N > 1 = the replicated RCCL bf16 all-reduce (4(n-1)/n "
                   "B/param on the bus vs 6(n-1)/n for a2a); a2a's error does not grow with n")
    return out


def run_q8(spec, dev, ws, rank, steps, warmup, cap):
    """int8 wire: per-bucket dl_delta_q8 -> all_to_all -> dl_q8_reduce ->
    all_gather -> dl_unpack_sgd_q8. Bus bytes per peer: 2(n-1)/n * slot bytes (1.016 B/param)
    instead of 2(n-1)/n * 4 B/param. At one replica the exchange is skipped; the kernels run."""
    from diloco_amd.kernels import Q8_SLOT

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
    nb = eng.tree.n_buckets
    slot_bytes = eng.tree.n_chunks * Q8_SLOT
    res = {"tree": spec.name, "params": P, "buckets": nb, "chunks": eng.tree.n_chunks,
           "ms_per_step": dt / steps * 1e3, "value": 4.0 * P / (dt / steps) / 1e9,
           "value_aggregate": ws * 4.0 * P / (dt / steps) / 1e9,
           "wire": "int8", "wire_bytes_per_param": round(slot_bytes / P, 4),
           "bus_bytes_per_step": 2.0 * (ws - 1) / ws * slot_bytes}
    if ws == 1:  # the three kernels, each over the whole tree (as the one-replica step runs
        # them: no bucket is padded at n = 1), timed in place
        from diloco_amd.plan import SLOT_INNER

        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        tot = [0.0, 0.0, 0.0]
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
                tot[i] += ev[i].elapsed_time(ev[i + 1])
        ms = [t / steps for t in tot]
        pmc = load_pmc(spec.name)  # the same whole-tree launches (tools/kernel_driver.py)
        res["kernels"] = {
            "delta_q8": kernel_entry(8 * P + slot_bytes, ms[0], pmc.get("delta_q8"),
                                     rw=(8 * P, 2, slot_bytes, 1)),
            "q8_reduce": kernel_entry(2 * slot_bytes, ms[1], pmc.get("q8_reduce"),
                                      rw=(slot_bytes, 1, slot_bytes, 1)),
            "unpack_sgd_q8": kernel_entry(slot_bytes + 20 * P, ms[2], pmc.get("unpack_sgd_q8"),
                                          rw=(slot_bytes + 8 * P, 3, 12 * P, 3)),
        }
    eng.close()
    del eng
    torch.cuda.empty_cache()
    return res


def parity_q8(dev, ws, rank):
    """int8 codec on the tiny tree (3 buckets): the averaged g every replica applies against the
    exact fp32 average, element by element, within the quantiser's own bound
        |g - avg| <= (1/n) Σ_r s_r/2 + s'/2,   s_r = amax_chunk(delta_r)/127,
        s' = amax_chunk(avg')/127 <= (amax_chunk(avg) + (1/n) Σ_r s_r/2)/127
    (plus 1e-5 relative slack for the fp32 sums); and every replica bit-identical after it."""
    from diloco_amd.kernels import Q8_SLOT

    spec = get_tree("tiny")
    eng = build(spec, dev, rank, torch.int8, 1 << 20)
    nb = eng.tree.n_buckets
    deq = []
    for b in range(nb):
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
    for b in range(nb):
        eng.apply(b)
    eng.steps_done += 1
    torch.cuda.synchronize()
    bits = eng.theta.view(torch.int32).to(torch.int64).sum()
    ck = torch.stack([bits, -bits])
    if ws > 1:
        dist.all_reduce(ck, op=dist.ReduceOp.MAX)
    identical = bool(ck[0].item() == -ck[1].item())
    eng.close()
    return {"tree": "tiny", "buckets": nb, "wire": "int8",
            "max_err_over_bound": worst, "tolerance": 1.0,
            "replicas_identical": identical, "ok": bool(worst <= 1.0 and identical)}


# HBM bytes per parameter of the device drop-in sequence (placement="device"), by (fused, N>1):
# fused one peer: dl_delta_pack_sgd (read θ, inner, m; write wire, θ, m, inner); fused N > 1:
# dl_delta_pack (12) before each bucket's all_reduce + dl_unpack_sgd with the /n and the inner
# write (24); eager: dl_delta_pack 12 + (dl_unpack_avg 8) + dl_unpack_sgd 20 + dl_scatter 8
DROPIN_DEVICE_BPP = {(True, False): 28, (True, True): 36, (False, False): 40, (False, True): 48}


def dropin_rate(spec, dev, ws, rank, steps, placement="host", write_back="sync", inner_fn=None,
                fused=None):
    """The reference's call sequence (src/train.py:261-269) through the drop-in functions.
    placement "host": the reference's host-resident outer model, PCIe transfers included
    (DESIGN.md "Host-memory ends"); "device": the outer model in HBM,
    fused (default: DILOCO_OUTER_FUSED, on) or eager (fused=False; mirror.DeviceOuterMirror).
    write_back "deferred": the host placement's write-back DMAs issued by sync_inner_model
    and not waited for. inner_fn: GPU work standing in for the inner steps that follow an
    outer step in training, enqueued after it and inside the timed cycle (the reference
    synchronises the device after every inner step, src/train.py:243). Each cycle ends with a
    device synchronize, so the host work of the four calls is inside the time."""
    from types import SimpleNamespace

    from diloco_amd.comm import TrainingComm
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)
    from diloco_amd.world import World

    if not dist.is_initialized():
        import tempfile

        dist.init_process_group("gloo", init_method="file://" + tempfile.mktemp(prefix="dlpg"),
                                rank=0, world_size=1)
    shapes = [s for _, s in spec.params()]
    inner = torch.nn.Module()
    inner.ps = torch.nn.ParameterList(
        [torch.nn.Parameter(t.view(s)) for t, s in zip(synth.outer_tree_device(spec, dev), shapes)])
    outer = get_outer_model(inner, placement, write_back=write_back, fused=fused)
    is_fused = bool(getattr(outer, "_diloco_fused", False))
    opt = get_optimizer(outer, SimpleNamespace(type="SGD", lr=0.7, momentum=0.9, nesterov=True))
    comm = TrainingComm(World.from_default_group(1), (1, 1, spec.n_embd), None)
    synth.inner_tree_device([p.data.view(-1) for p in inner.parameters()], 1, rank,
                            out=[p.data.view(-1) for p in inner.parameters()])
    phases = {"compute_pseudo_gradient": 0.0, "sync_gradients": 0.0, "outer_step": 0.0,
              "sync_inner_model": 0.0}

    def one(record):
        t = [time.perf_counter()]
        compute_pseudo_gradient(inner, outer)
        t.append(time.perf_counter())
        comm.sync_gradients(outer)
        t.append(time.perf_counter())
        opt.step()
        t.append(time.perf_counter())
        sync_inner_model(outer, inner)
        if inner_fn is not None:
            inner_fn()
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        if record:
            for k, a, b in zip(phases, t, t[1:]):
                phases[k] += b - a

    one(False)
    if ws > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        one(True)
    dt = _max_over_ranks((time.perf_counter() - t0) / steps, dev, ws)
    P = spec.total()
    d2h = 0
    if placement == "host":
        d2h = (16 if ws > 1 and write_back == "sync" else 12) * P
    if inner_fn is not None:
        phases["inner_work_and_sync"] = phases.pop("sync_inner_model")
    res = {"tree": spec.name, "value": round(4.0 * P / dt / 1e9, 2), "unit": "GB/s",
           "value_aggregate": round(ws * 4.0 * P / dt / 1e9, 2),
           "ms_per_step": round(dt * 1e3, 3),
           "phase_ms": {k: round(v / steps * 1e3, 3) for k, v in phases.items()},
           "placement": placement, "write_back": write_back,
           "d2h_bytes_per_step": d2h,
           "note": ("host outer model (reference semantics); D2H of delta, (avg,) θ, momentum"
                    if placement == "host" else
                    "outer model in HBM (params/.grad/momentum are packed views); no PCIe")}
    if placement == "device" and inner_fn is None:
        # the GPU span of the four calls (events on the stream they launch on, around each
        # cycle; no synchronize inside): at one peer and fused, the one dl_delta_pack_sgd
        bpp = DROPIN_DEVICE_BPP[(is_fused, ws > 1)]
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(steps)]
        for e in ev:
            e[0].record()
            compute_pseudo_gradient(inner, outer)
            comm.sync_gradients(outer)
            opt.step()
            sync_inner_model(outer, inner)
            e[1].record()
        torch.cuda.synchronize()
        span = sum(e[0].elapsed_time(e[1]) for e in ev) / steps
        res.update(fused=is_fused, hbm_bytes_per_param=bpp, gpu_span_ms=round(span, 5),
                   kernels_launched=("dl_delta_pack_sgd" if is_fused and ws == 1 else
                                     "dl_delta_pack / all_reduce / dl_unpack_sgd(+inner)"
                                     if is_fused else
                                     "dl_delta_pack / (all_reduce + dl_unpack_avg) / "
                                     "dl_unpack_sgd / dl_scatter"))
        if ws == 1:
            name = "delta_pack_sgd" if is_fused else "dropin_eager_sequence"
            res["roofline"] = dict(kernel_entry(bpp * P, span), kernel=name)
        # the values the calls leave behind equal the engine's one-pass step (bit-exact):
        # checked by tests/test_dropin_gpu.py at T125 against the C oracle
    return res


def run_dropin(spec, dev, ws, rank, steps, warmup, wire="f32", bucket_elems=None):
    """The outer step through the reference's own call surface, src/train.py:263-269 --
    compute_pseudo_gradient -> TrainingComm.sync_gradients -> outer_optimizer.step() ->
    sync_inner_model -- on the device-resident fused outer model (get_outer_model(...,
    placement="device"), mirror.DeviceOuterMirror): K steps back to back between barrier +
    synchronize, as the engine legs are timed (the four Python calls of step k+1 are issued
    while step k's kernels run). N = 1: one dl_delta_pack_sgd per step; N > 1: per bucket
    dl_delta_pack -> RCCL all_reduce, then dl_unpack_sgd (/n, SGD, inner write). wire="bf16":
    BASELINE config #5 behind the same calls (the pack casts to bf16, RCCL sums bf16, the SGD
    pass reads the wire). bucket_elems: the DP exchange's bucket size (the
    DILOCO_OUTER_BUCKET_ELEMS knob; default 64 Mi elements)."""
    from types import SimpleNamespace

    from diloco_amd.comm import TrainingComm
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)
    from diloco_amd.world import World

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
        outer = get_outer_model(inner, "device", fused=True, wire=wire)
    finally:
        if bucket_elems is not None:
            if prev is None:
                os.environ.pop(knob, None)
            else:
                os.environ[knob] = prev
    opt = get_optimizer(outer, SimpleNamespace(type="SGD", lr=0.7, momentum=0.9, nesterov=True))
    comm = TrainingComm(World.from_default_group(1), (1, 1, spec.n_embd), None)
    # inner = θ_0 + this rank's noise (H inner steps' stand-in); later steps see inner = θ
    synth.inner_tree_device([p.data.view(-1) for p in inner.parameters()], 1, rank,
                            out=[p.data.view(-1) for p in inner.parameters()])

    def one():
        compute_pseudo_gradient(inner, outer)
        comm.sync_gradients(outer)
        opt.step()
        sync_inner_model(outer, inner)

    for _ in range(max(warmup, 1)):
        one()
    _sync(ws)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    ev[0].record()
    for _ in range(steps):
        one()
    ev[1].record()
    _sync(ws)
    dt = _max_over_ranks((time.perf_counter() - t0) / steps, dev, ws)
    loop_ms = ev[0].elapsed_time(ev[1]) / steps
    P = spec.total()
    m = outer._diloco_mirror
    res = {"tree": spec.name, "params": P, "tensors": len(shapes), "padded": m.tree.total,
           "buckets": m.tree.n_buckets, "chunks": getattr(m.tree, "n_chunks", None),
           "ms_per_step": dt * 1e3, "value": 4.0 * P / dt / 1e9,
           "value_aggregate": ws * 4.0 * P / dt / 1e9, "loop_gpu_ms_per_step": round(loop_ms, 5),
           "wire": wire, "fused": m.fused,
           "variant": ("the reference's four calls on the fused device outer model: "
                       + ("dl_delta_pack_sgd" if ws == 1 else
                          "dl_delta_pack -> RCCL all_reduce (per bucket) -> dl_unpack_sgd "
                          "(/n, inner write)"))}
    if ws == 1:
        res["roofline"] = dict(kernel_entry(28 * P, loop_ms, load_pmc(spec.name).get("delta_pack_sgd"),
                                            rw=(12 * P, 3, 16 * P, 4)),
                               kernel="delta_pack_sgd", timing="timed loop GPU span / K")
    else:
        # the exchange: the same all_reduce calls the step makes (every bucket of the packed
        # wire, on the DP group), back to back; bus bytes 2(n-1)/n of the wire
        group = comm.dp.dp_group(dev)
        w = m.d_wire16 if wire == "bf16" else m.d_wire
        reps_ar = max(3, steps // 2)
        _sync(ws)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps_ar):
            for lo, hi in m.tree.bucket_ranges:
                dist.all_reduce(w[lo:hi], group=group)
        e1.record()
        e1.synchronize()
        ar_ms = _max_over_ranks(e0.elapsed_time(e1) / reps_ar, dev, ws)
        bus = 2.0 * (ws - 1) / ws * w.element_size() * m.tree.total
        res["roofline"] = dict(kernel_entry(bus, ar_ms, bound="xgmi",
                                            peak=(ws - 1) * XGMI_LINK_GBS),
                               kernel="rccl all_reduce (all buckets, back to back)",
                               bus_bytes_per_step=bus)
    m.close()
    del outer, opt, inner, m
    torch.cuda.empty_cache()
    return res


def dropin_overlap(spec, dev, ws, rank, cycles, inner_ms=50.0):
    """The host outer model in a training cycle: outer step, then `inner_ms` of GPU work
    standing in for the inner steps that follow (bf16 GEMMs; a T125 inner step of the
    reference's batch 512 x 1024 tokens is several times longer), then a device synchronize
    as src/train.py:243 does. Exposed outer-step cost = cycle - inner work alone, for the
    sync write-back and the deferred one (whose PCIe DMAs run under the inner work)."""
    n = 8192
    a = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    b = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    c = torch.empty(n, n, device=dev, dtype=torch.bfloat16)

    def gemms(k):
        for _ in range(k):
            torch.mm(a, b, out=c)

    gemms(3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gemms(10)
    torch.cuda.synchronize()
    per = (time.perf_counter() - t0) / 10
    k = max(1, int(round(inner_ms * 1e-3 / per)))
    t0 = time.perf_counter()
    for _ in range(cycles):
        gemms(k)
        torch.cuda.synchronize()
    t_in = _max_over_ranks((time.perf_counter() - t0) / cycles, dev, ws)
    out = {"tree": spec.name, "inner_work_ms": round(t_in * 1e3, 3),
           "inner_work": f"{k} bf16 GEMMs {n}^3 per cycle"}
    P = spec.total()
    for wb in ("sync", "deferred"):
        r = dropin_rate(spec, dev, ws, rank, cycles, "host", wb, lambda: gemms(k))
        exposed = max(r["ms_per_step"] - t_in * 1e3, 1e-3)
        out[wb] = {"cycle_ms": r["ms_per_step"], "exposed_outer_ms": round(exposed, 3),
                   "value": round(4.0 * P / (exposed * 1e-3) / 1e9, 2),
                   "phase_ms": r["phase_ms"], "d2h_bytes_per_step": r["d2h_bytes_per_step"]}
    out["unit"] = "GB/s"
    out["note"] = ("value = 4P / exposed outer-step time (cycle - inner work alone), host "
                   "outer model (reference placement), PCIe included")
    return out


def gradsync_rate(spec, dev, ws, rank, steps, exchange="rccl"):
    """Per-step DP gradient average of device grads (src/train.py:249-251,
    src/comm.py:117-123): dl_gather -> RCCL all_reduce -> dl_unpack_avg, pipelined buckets
    (exchange="a2a": all_to_all -> rank-order average -> all_gather -> copy back)."""
    from diloco_amd.gradsync import GradSync

    shapes = [s for _, s in spec.params()]
    params = [torch.nn.Parameter(t.view(s))
              for t, s in zip(synth.outer_tree_device(spec, dev), shapes)]
    for i, p in enumerate(params):
        p.grad = torch.empty_like(p)
        synth.fill_device(p.grad.view(-1), synth.noise_seed(9, rank), i, 0.0, 1e-3)
    gs = GradSync(params, None, ws, exchange=exchange)
    gs.sync()
    _sync(ws)
    t0 = time.perf_counter()
    for _ in range(steps):
        gs.sync()
    _sync(ws)
    dt = _max_over_ranks((time.perf_counter() - t0) / steps, dev, ws)
    P = spec.total()
    gs.close()
    return {"tree": spec.name, "value": round(4.0 * P / dt / 1e9, 2), "unit": "GB/s",
            "value_aggregate": round(ws * 4.0 * P / dt / 1e9, 2),
            "ms_per_step": round(dt * 1e3, 4), "buckets": gs.tree.n_buckets,
            "exchange": exchange}


def p2p_rate(spec, dev, ws, rank, steps):
    """Device p2p transport (src/comm.py:16-69): two stages (rank % 2),
    stage-0 rank r sends a framed (2, mbs, seq, n_embd) activation to r+1 and gets it back;
    header over gloo, payload over RCCL data groups (isolated child legs, even N)."""
    from diloco_amd.p2p import DeviceRecvThread, DeviceSendThread, boundary_data_groups
    from diloco_amd.world import World

    if ws < 2 or ws % 2:
        return {"ok": False, "error": "needs an even number of ranks >= 2"}
    w = World.from_default_group(2)  # the reference's stage groups (gloo)
    dg = boundary_data_groups(w, backend=dist.get_backend())
    shape = (8, 1024, spec.n_embd)  # mbs 8, seq 1024 (SURVEY §8f row 3 activations)
    kw = dict(start=False, serialize=True)
    if w.stage == 0:
        tx = DeviceSendThread(shape, w.next_stage_group, dg[(0, 1, "fwd")], dev, **kw)
        rx = DeviceRecvThread(shape, w.next_stage_group, dg[(0, 1, "bwd")], dev, **kw)
    else:
        tx = DeviceSendThread(shape, w.prev_stage_group, dg[(0, 1, "bwd")], dev, **kw)
        rx = DeviceRecvThread(shape, w.prev_stage_group, dg[(0, 1, "fwd")], dev, **kw)
    act = torch.randn(shape, device=dev)
    ok = True

    def round_trip(i):
        nonlocal ok
        if w.stage == 0:
            tx.send_one(rank + 1, act, (rank, i))
            src, t, meta = rx.recv_one()
            ok &= src == rank + 1 and meta == (rank, i)
        else:
            src, t, meta = rx.recv_one()
            ok &= src == rank - 1 and meta == (src, i)
            tx.send_one(src, t.detach(), meta)

    round_trip(-1)
    _sync(ws)
    t0 = time.perf_counter()
    for i in range(steps):
        round_trip(i)
    _sync(ws)
    dt = _max_over_ranks((time.perf_counter() - t0) / steps, dev, ws)
    frame = 2 * act.numel() * 4
    return {"frame_bytes": frame, "ms_per_round_trip": round(dt * 1e3, 4),
            "value": round(2 * frame / dt / 1e9, 2), "unit": "GB/s per rank pair",
            "transport": f"header gloo, payload {dist.get_backend()}", "ok": bool(ok)}


def cpu_baseline(spec, seconds_budget=12.0):
    """The reference's per-tensor CPU sequence (oracle/torch_restatement.py), 1 thread."""
    sys.path.insert(0, HERE)
    from oracle.torch_restatement import time_steps

    t, n = time_steps(spec.numels(), steps=2, threads=1, budget_s=seconds_budget)
    return {
        "value": round(4.0 * spec.total() / t / 1e9, 4), "unit": "GB/s", "cores": 1,
        "kind": "port",
        "sample": (f"{spec.name} full tree ({spec.total()} params), {n} timed outer steps after 1 "
                   f"warm step, per-tensor torch CPU restatement of src/utils.py:218-226 + "
                   f"torch SGD-Nesterov (sync_gradients is a no-op at n=1), 1 thread; "
                   f"{t:.3f} s/step"),
        "host": _host_info(),
    }


def cpu_baseline_dist(spec, ws, rank, seconds_budget=12.0, group=None):
    """§8d CPU baseline at N > 1: this process is one of N fresh CPU processes (GPUs hidden)
    in a gloo group, each running the reference's per-tensor sequence on the full tree with
    one thread -- delta, per-tensor gloo all_reduce(SUM) + /= n, torch SGD-Nesterov, copy-back
    (oracle/torch_restatement.TorchOuterStep) -- N cores in all. Steps are counted so that the
    timed sample lasts about `seconds_budget`; value = 4P / t_step (the metric's definition),
    max time over ranks. group: a gloo group over the N ranks when the bench's own rank
    processes run it (rehearsals with every rank on one GPU); default the child's world."""
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
                       f"processes (gloo, 1 thread each), {k} timed outer steps after 2: "
                       f"per-tensor torch restatement of src/utils.py:218-226 + per-tensor "
                       f"all_reduce/n (src/comm.py:120-123) + torch SGD-Nesterov; "
                       f"{t:.3f} s/step"),
            "host": _host_info()}


def _host_info():
    model = ""
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        model = next((l.split(":", 1)[1].strip() for l in out.splitlines()
                      if l.startswith("Model name")), "")
    except Exception:
        pass
    return {"cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "model": model, "torch": torch.__version__}


# CPU-baseline children see no GPU: they are host processes like the reference's --device cpu
HIDE_GPUS = {"CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""}


def _guard(fn, *a, **k):
    try:
        return fn(*a, **k)
    except Exception as e:  # reported in the JSON line, never hidden
        log(f"{fn.__name__} failed: {e!r}")
        return {"ok": False, "error": repr(e)}


def _brief(r):
    keep = ("value", "value_aggregate", "ms_per_step", "roofline", "kernels", "kernels_b2b",
            "buckets", "params", "wire", "variant", "wire_bytes_per_param", "bus_bytes_per_step",
            "tile_chunks", "cold")
    return {k: r[k] for k in keep if k in r}


def peer_access_legs(spec, dev, ws, rank, steps, warmup, cap, parity_too, dump=None,
                     extra_spec=None):
    """The legs that map peers' memory or run point-to-point traffic between GPUs: the direct
    exchange, its parity check, the link probe and the device p2p transport (even N). Run by
    the isolated child processes below; `dump(result)` is called after every leg so that a
    child stopped by its watchdog still reports what it finished."""
    res = {"extra": {}, "parity": {}}
    dump = dump or (lambda r: None)
    for ex in ("xgmi", "xgmi_inner"):  # peers' wires / peers' inner arenas (no pack pass)
        r = _guard(run_tree, spec, dev, ws, rank, steps, warmup, torch.float32, cap, False,
                   False, None, ex)
        res["extra"][f"{spec.name}_{ex}_exchange"] = _brief(r) if "value" in r else r
        dump(res)
        if parity_too:
            res["parity"][ex] = _guard(parity_xgmi, dev, ws, rank, ex)
            dump(res)
    res["extra"]["xgmi_link_probe"] = _guard(xgmi_link_probe, dev, ws, rank)
    dump(res)
    if ws % 2 == 0:  # header over gloo, framed payload over RCCL
        res["extra"]["p2p_device_transport"] = _guard(p2p_rate, spec, dev, ws, rank, 10)
        dump(res)
    if extra_spec is not None:  # the north star's 1.3B fp32 bucket set through the direct
        # exchange (last: the largest peer mappings)
        torch.cuda.empty_cache()
        r = _guard(run_tree, extra_spec, dev, ws, rank, max(3, steps // 4), 1, torch.float32,
                   cap, False, False, None, "xgmi_inner")
        res["extra"][f"{extra_spec.name}_xgmi_inner_exchange"] = _brief(r) if "value" in r else r
        dump(res)
    return res


# RCCL settings tried beside the defaults at N > 1 (channel count and protocol are
# the knobs for the xGMI all-reduce target); each runs in its own child process group
RCCL_ENV_VARIANTS = {"min_channels_64": {"NCCL_MIN_NCHANNELS": "64"},
                     "proto_simple": {"NCCL_PROTO": "Simple"},
                     # collectives on high-priority streams: the bucket pipeline's kernels
                     # then yield the CUs to RCCL's
                     "high_priority_streams": {"TORCH_NCCL_HIGH_PRIORITY": "1"}}


def rccl_env_legs(spec, dev, ws, rank, steps, warmup, cap, dump=None):
    """Under the child's RCCL environment: RCCL's own all_reduce / reduce_scatter+all_gather
    rate on the headline's bytes and the headline's sharded outer step."""
    res = {"env": {k: os.environ[k] for k in ("NCCL_MIN_NCHANNELS", "NCCL_PROTO", "NCCL_ALGO",
                                              "TORCH_NCCL_HIGH_PRIORITY") if k in os.environ}}
    dump = dump or (lambda r: None)
    res["rccl_allreduce_ref"] = _guard(rccl_reference, dev, ws, rank,
                                       spec.total() // (64 * ws) * (64 * ws))
    dump(res)
    r = _guard(run_tree, spec, dev, ws, rank, steps, warmup, torch.float32, cap, False, False)
    res["sharded_step"] = _brief(r) if "value" in r else r
    dump(res)
    return res


def isolated_legs(a, dev, ws, rank, timeout_s, which="peer", extra_env=None):
    """Run a set of legs in a child process per rank (their own process group on a fresh
    rendezvous port): which="peer" -> peer_access_legs, so that a GPU fault or an abort while
    peers' memory is mapped ends the children, not this run; which="rccl_env" ->
    rccl_env_legs under `extra_env` (RCCL settings are read once per process). The parents
    wait (bounded), then carry on to print the line. Returns rank 0's child result, or an
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
           "--bucket-mb", str(a.bucket_mb),
           "--deadline", str(max(30.0, timeout_s - 10)), "--child-legs", which,
           "--child-out", out] + (["--no-parity"] if a.no_parity else [])
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


def _xgmi_efficiency(line, extra, tree, ws):
    """The direct exchange on the 1.3B set against RCCL's all_reduce of the same bytes (the
    parent's rccl_allreduce_ref_<tree> leg), as exchange_efficiency_<tree> does for the RCCL
    step."""
    r = extra.get(f"{tree}_xgmi_inner_exchange")
    ref = extra.get(f"rccl_allreduce_ref_{tree}")
    if not (isinstance(r, dict) and "ms_per_step" in r and isinstance(ref, dict)
            and "all_reduce" in ref):
        return
    P = get_tree(tree).total()
    bw = 2.0 * (ws - 1) / ws * 4 * P / (r["ms_per_step"] * 1e-3) / 1e9
    arbw = ref["all_reduce"]["busbw_GBs"]
    line[f"exchange_efficiency_{tree}_xgmi_inner"] = {
        "step_ms": round(r["ms_per_step"], 3), "step_busbw_GBs": round(bw, 1),
        "rccl_allreduce_busbw_GBs": arbw, "frac_of_rccl_allreduce": round(bw / arbw, 4),
        "frac_of_link_peak": round(bw / ((ws - 1) * XGMI_LINK_GBS), 4),
        "note": "direct peer-access exchange (exchange='xgmi_inner'), whole outer step"}


class _Emitter:
    """The one JSON line, assembled as the legs finish, printed exactly once by rank 0.

    A watchdog (every rank, same deadline) bounds the whole run: if a side leg hangs (an RCCL
    collective or a peer-access kernel at N > 1 that no test box can rehearse), the line with
    the headline and every leg finished so far is printed, naming the leg that was running,
    and every rank leaves with os._exit -- the driver still gets its measurement instead of a
    killed run. Legs that would start after the soft budget are skipped and listed."""

    def __init__(self, rank, deadline_s):
        import threading

        self.rank, self.t0, self.deadline = rank, time.perf_counter(), deadline_s
        self.line, self.running, self.skipped = None, "headline", []
        self.lock = threading.Lock()
        self.done = False
        # the JSON line goes to the process's original stdout; everything else written to
        # fd 1 during the run (gloo's C++ "[Gloo] Rank ..." notices, library chatter) has
        # been sent to stderr, so stdout carries exactly one line
        sys.stdout.flush()
        self.out_fd = os.dup(1)
        os.dup2(2, 1)
        self.timer = threading.Timer(deadline_s, self._fire)
        self.timer.daemon = True
        self.timer.start()

    def elapsed(self):
        return time.perf_counter() - self.t0

    def emit(self):
        with self.lock:
            if self.done:
                return
            self.done = True
            if self.rank == 0 and self.line is not None:
                if self.skipped:
                    self.line["skipped_legs"] = self.skipped
                buf = (json.dumps(self.line) + "\n").encode()
                while buf:
                    buf = buf[os.write(self.out_fd, buf):]

    def _fire(self):
        log(f"watchdog: {self.deadline:.0f} s reached while running {self.running!r}")
        if self.line is not None:
            self.line["incomplete"] = {"leg": self.running, "deadline_s": self.deadline}
        self.emit()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0 if self.line is not None else 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50,
                    help="timed steps K (the first timed step also carries the host's issue of "
                         "its calls after the barrier: 1/K of the per-step figure)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--tree", default="t125")
    ap.add_argument("--wire", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--bucket-mb", type=int, default=256)
    ap.add_argument("--extra-tree", default="t1.3b", help="second tree measured beside (or 'none')")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip the host-outer-model rate")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-xgmi", action="store_true",
                    help="skip the isolated legs at N > 1 (direct peer-access exchange, link "
                         "probe, device p2p transport)")
    ap.add_argument("--p2p", action="store_true",
                    help="(kept for compatibility: the device p2p transport is timed at every "
                         "even N > 1, in the isolated child legs)")
    ap.add_argument("--only-headline", action="store_true",
                    help="headline tree only (for rocprofv3 runs of the same kernels)")
    ap.add_argument("--no-b2b", action="store_true",
                    help="skip the back-to-back kernel loops (rocprofv3 averages = in-step launches)")
    ap.add_argument("--deadline", type=float,
                    default=float(os.environ.get("DILOCO_BENCH_DEADLINE_S", "420")),
                    help="hard wall-clock bound of the whole run (s); side legs stop starting "
                         "at 70 %% of it")
    ap.add_argument("--child-legs", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--child-out", default=None, help=argparse.SUPPRESS)
    a = ap.parse_args()

    if a.child_legs == "cpu_baseline":  # one CPU process of the N > 1 CPU baseline
        ws, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
        timer = _Emitter(rank, a.deadline)
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
        threading_timer = _Emitter(rank, a.deadline)  # bounds the child too
        _lib.load()

        def dump(r):
            if rank == 0:
                tmp = a.child_out + ".tmp"
                with open(tmp, "w") as f:
                    json.dump(r, f)
                os.replace(tmp, a.child_out)

        args = (get_tree(a.tree), dev, ws, rank, a.steps, a.warmup, (a.bucket_mb << 20) // 4)
        if a.child_legs == "peer":
            es = (get_tree(a.extra_tree) if a.extra_tree not in ("none", a.tree) else None)
            peer_access_legs(*args, not a.no_parity, dump, es)
        else:
            rccl_env_legs(*args, dump)
        threading_timer.done = True
        if dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()
        threading_timer.timer.cancel()
        return

    em = _Emitter(int(os.environ.get("RANK", "0")), a.deadline)
    soft = 0.7 * a.deadline
    ws, rank, dev = setup_dist(a.gpus)
    # child legs put a second process per rank on the GPU: with every rank on one GPU (a gloo
    # rehearsal) 2N + 1 processes (the launcher too) must stay within the box's 16 per GPU
    shared_gpu = ws > max(1, torch.cuda.device_count())
    children_fit = not shared_gpu or 2 * ws + 1 <= 16
    wire = torch.bfloat16 if a.wire == "bf16" else torch.float32
    cap = (a.bucket_mb << 20) // 4
    _lib.load()
    spec = get_tree(a.tree)
    log(f"rank {rank}/{ws} tree {spec.name} ({spec.total()} params) wire {a.wire}")
    # headline at N = 1: whole-range launches (tile 0), so the per-kernel figures and the
    # rocprofv3 averages describe the same launches; cache blocking is neutral on T125
    # (tools/tile_ab.py) and is what the T1.3B leg below runs (OuterSync's default tile)
    fallback = None
    # The engine (OuterSync.step, the device-resident fast path): at N = 1 the one-replica step
    # in one pass, pseudo-gradient kept (dl_delta_pack_sgd) -- with its per-kernel, cold and
    # back-to-back figures; at N > 1 the sharded step.
    try:
        eng_res = run_tree(spec, dev, ws, rank, a.steps, a.warmup, wire, cap, fuse=ws == 1,
                           b2b_loops=not a.no_b2b, tile=0, cold=not a.only_headline,
                           keep_wire=True)
    except Exception as e:  # N > 1: the replicated all-reduce step still gives the driver a line
        if ws == 1:
            raise
        fallback = repr(e)
        log(f"sharded engine step failed ({fallback}); measuring the all-reduce step instead")
        eng_res = run_tree(spec, dev, ws, rank, a.steps, a.warmup, wire, cap, False,
                           not a.no_b2b, False)
    # The headline: the same outer step through the reference's own call surface
    # (src/train.py:263-269 unchanged: compute_pseudo_gradient -> TrainingComm.sync_gradients
    # -> outer_optimizer.step() -> sync_inner_model) on the fused device outer model; the
    # engine's figure stays in extra. fp32 wire only (the drop-in surface has no wire knob).
    main_res, dropin_error = eng_res, None
    if wire == torch.float32:
        try:
            main_res = run_dropin(spec, dev, ws, rank, a.steps, a.warmup)
            main_res["kernels"] = eng_res.get("kernels")
            main_res["cold"] = eng_res.get("cold")
            main_res["kernels_b2b"] = eng_res.get("kernels_b2b")
        except Exception as e:
            if ws == 1:
                raise
            dropin_error = repr(e)
            log(f"drop-in headline failed ({dropin_error}); the engine's step is the headline")
    extra, parity = {}, {}
    ceiling = None
    if not a.only_headline:
        ceiling = _guard(copy_ceiling, dev)
        log(f"copy ceiling {ceiling}")
    roof = main_res["roofline"]
    if ws == 1:
        roof = with_copy_ceiling(roof, ceiling)
    cold = main_res.get("cold")
    roof_cold = None
    if cold:
        ks = cold["kernels"]
        dom = max(ks, key=lambda k: ks[k]["avg_ms"])
        roof_cold = dict(with_copy_ceiling(ks[dom], ceiling), kernel=dom)
        cold = dict(cold, value=round(cold["value"], 3), warm_value=round(cold["warm_value"], 3),
                    kernels={k: with_copy_ceiling(v, ceiling) for k, v in ks.items()})
    dropin = main_res is not eng_res
    if dropin:
        workload = (f"DiLoCo outer step, {spec.name} tree per rank, through the reference's "
                    "calls (src/train.py:263-269: compute_pseudo_gradient -> "
                    "TrainingComm.sync_gradients -> outer SGD step -> sync_inner_model) on the "
                    "fused device-resident outer model: "
                    + ("delta_pack -> RCCL all_reduce (per bucket) -> unpack_sgd (/n, Nesterov "
                       "SGD, inner write)" if ws > 1 else
                       "one dl_delta_pack_sgd per step (delta + outer.grad + Nesterov SGD + "
                       "copy to inner; no exchange at one replica, src/comm.py:118-119)"))
    else:
        workload = (f"DiLoCo outer step, {spec.name} tree per rank: "
                    + ("delta_pack -> RCCL reduce_scatter -> shard_sgd (1/n of θ, "
                       "momentum) -> RCCL all_gather(θ) -> scatter to inner (bucketed, "
                       "pipelined)" if ws > 1 else
                       "delta + pack (wire = outer.grad) + Nesterov SGD + copy to inner "
                       "in one pass (dl_delta_pack_sgd; no exchange at one replica, "
                       "src/comm.py:118-119)"))
    em.line = {
        "metric": METRIC,
        "value": round(main_res["value"], 3),
        "value_aggregate": round(main_res["value_aggregate"], 3),
        "value_cold": cold["value"] if cold else None,
        "unit": "GB/s",
        "n_gpus": ws,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(main_res["ms_per_step"], 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if a.wire == "f32" else "f32 (bf16 wire)",
        "data": "synthetic (counter-based GPT-2-shaped tree, SURVEY.md §8d)",
        "config": {
            "workload": workload,
            "tree": spec.name, "params": main_res["params"], "tensors": main_res["tensors"],
            "wire": a.wire, "buckets": main_res["buckets"], "chunks": main_res["chunks"],
            "parallelism": f"dp{ws}",
        },
        "roofline": roof,
        "roofline_cold": roof_cold,
        "copy_ceiling": ceiling,
        "cpu_baseline": None,
        "kernels": main_res.get("kernels"),
        "cold": cold,
        "kernels_b2b": main_res.get("kernels_b2b"),
        "parity": None if a.no_parity or a.only_headline else parity,
        "dropin_pcie": None,
        "extra": extra,
        "host": platform.node(),
    }
    extra[f"{spec.name}_engine"] = _brief(eng_res) if dropin else None
    if dropin_error:
        em.line["headline_fallback"] = {"dropin_error": dropin_error}
    if fallback:
        em.line["engine_fallback"] = {"variant": eng_res["variant"], "sharded_error": fallback}
        if not dropin:
            em.line["config"]["workload"] = (f"DiLoCo outer step, {spec.name} tree per rank: "
                                             "delta_pack -> RCCL all_reduce -> unpack_sgd "
                                             "(replicated; the sharded step failed)")
    log(f"headline done at {em.elapsed():.1f} s")

    def leg(name, fn, *args, into=extra, brief=True):
        """One side leg, in the same order on every rank; skipped (on every rank alike: the
        decision uses the max over ranks of the elapsed time) past the soft budget."""
        t = _max_over_ranks(em.elapsed(), dev, ws)
        if t > soft:
            em.skipped.append(name)
            log(f"skipping {name}: {t:.0f} s elapsed > soft budget {soft:.0f} s")
            return None
        em.running = name
        r = _guard(fn, *args)
        if brief and isinstance(r, dict) and "value" in r:
            r = _brief(r)
        into[name] = r
        log(f"{name} done at {em.elapsed():.1f} s")
        return r

    if not a.only_headline:
        if ws == 1:
            # BASELINE config #2's two kernels as separate launches (delta_pack -> unpack_sgd,
            # whole-range: per-kernel warm / cold / back-to-back figures) and the cache-blocked
            # two-kernel step (OuterSync's tiles), then the one pass without the wire
            leg(f"{spec.name}_two_kernel", run_tree, spec, dev, ws, rank, a.steps, a.warmup,
                wire, cap, False, True, None, "rccl", 0, True)
            leg(f"{spec.name}_two_kernel_tiled", run_tree, spec, dev, ws, rank, a.steps,
                a.warmup, wire, cap, False, False, None, "rccl", None, True)
            leg(f"{spec.name}_fused_single", run_tree, spec, dev, ws, rank, a.steps, a.warmup,
                wire, cap, True, True, None, "rccl", None, True)
        if a.extra_tree != "none" and a.extra_tree != a.tree:
            es = get_tree(a.extra_tree)
            ks = max(3, a.steps // 4)
            r13 = leg(es.name, run_tree, es, dev, ws, rank, ks, 1, wire, cap)
            if ws > 1 and isinstance(r13, dict) and "value" in r13:
                # the north star's DP = 8 target on the 1.3B fp32 bucket set: the whole step's
                # bus rate against RCCL's own all_reduce of the same bytes, this node, this run
                ref13 = leg(f"rccl_allreduce_ref_{es.name}", rccl_reference, dev, ws, rank,
                            es.total() // (64 * ws) * (64 * ws), 3, brief=False)
                if isinstance(ref13, dict) and "all_reduce" in ref13:
                    bus = 2.0 * (ws - 1) / ws * 4 * es.total()
                    bw = bus / (r13["ms_per_step"] * 1e-3) / 1e9
                    arbw = ref13["all_reduce"]["busbw_GBs"]
                    em.line[f"exchange_efficiency_{es.name}"] = {
                        "step_ms": round(r13["ms_per_step"], 3),
                        "step_busbw_GBs": round(bw, 1),
                        "rccl_allreduce_busbw_GBs": arbw,
                        "frac_of_rccl_allreduce": round(bw / arbw, 4),
                        "frac_of_link_peak": round(bw / ((ws - 1) * XGMI_LINK_GBS), 4),
                    }
            if ws == 1:  # the headline's one-pass step on the 1.3B tree
                leg(f"{es.name}_fused_keep_wire", run_tree, es, dev, ws, rank, ks, 1, wire, cap,
                    True, False, None, "rccl", None, False, True)
            if wire == torch.float32:  # BASELINE config #5: bf16 wire + SGD fused into unpack
                leg(f"{es.name}_bf16_wire", run_tree, es, dev, ws, rank, ks, 1, torch.bfloat16,
                    cap)
                leg(f"{es.name}_int8_wire", run_q8, es, dev, ws, rank, ks, 1, cap)  # §8f row 4
                if ws > 1:  # config #5 with the ordered exchange: bf16 slices summed in fp32
                    leg(f"{es.name}_bf16_a2a", run_tree, es, dev, ws, rank, ks, 1,
                        torch.bfloat16, cap, False, False, True, "a2a")
                    # config #5 behind the reference's calls: the fused device outer model
                    # with the bf16 wire (cast in the pack, SGD reading the wire)
                    leg(f"{es.name}_dropin_bf16", run_dropin, es, dev, ws, rank, ks, 1, "bf16",
                        brief=False)
                    if not a.no_parity:  # both bf16 forms' error on this tree at this N
                        leg(f"bf16_codec_{es.name}", codec_error, es, dev, ws, rank, cap,
                            into=parity, brief=False)
        if ws > 1:
            # RCCL's own all-reduce rate on the headline's bytes (the exchange's yardstick)
            ref = leg("rccl_allreduce_ref", rccl_reference, dev, ws, rank,
                      main_res["padded"] // (64 * ws) * (64 * ws), brief=False)
            if isinstance(ref, dict) and "all_reduce" in ref:
                bw = main_res["roofline"]["bus_bytes_per_step"] / (main_res["ms_per_step"] * 1e-3) / 1e9
                em.line["exchange_efficiency"] = {
                    "step_busbw_GBs": round(bw, 1),
                    "rccl_allreduce_busbw_GBs": ref["all_reduce"]["busbw_GBs"],
                    "frac_of_rccl_allreduce": round(bw / ref["all_reduce"]["busbw_GBs"], 4),
                    "note": "whole outer step (kernels + collectives) as bus bytes / step time, "
                            "over RCCL's all_reduce of the same bytes",
                }
            # the replicated variant (all-reduce -> SGD on every peer) beside the sharded headline
            leg(f"{spec.name}_allreduce_variant", run_tree, spec, dev, ws, rank, a.steps,
                a.warmup, wire, cap, False, False, False)
            # bucket size for the xGMI pipeline: 64 MiB buckets (more overlap, more calls)
            leg(f"{spec.name}_bucket64MiB", run_tree, spec, dev, ws, rank, a.steps, a.warmup,
                wire, 16 << 20, False, False)
            # the same for the headline (the reference's calls on the fused device outer model):
            # eight 64 MiB buckets instead of two 256 MiB ones, i.e. a shorter exposed pack of the
            # first bucket and SGD pass of the last against four times the RCCL calls
            if wire == torch.float32:
                leg(f"{spec.name}_dropin_bucket64MiB", run_dropin, spec, dev, ws, rank, a.steps,
                    a.warmup, "f32", 16 << 20, brief=False)
            # the ordered sharded step: all_to_all + rank-order reduce (deterministic, same bus)
            leg(f"{spec.name}_a2a", run_tree, spec, dev, ws, rank, a.steps, a.warmup, wire, cap,
                False, False, True, "a2a")
            leg(f"{spec.name}_dp_grad_sync", gradsync_rate, spec, dev, ws, rank,
                max(3, a.steps // 2), brief=False)
            leg(f"{spec.name}_dp_grad_sync_a2a", gradsync_rate, spec, dev, ws, rank,
                max(3, a.steps // 2), "a2a", brief=False)
            if ws >= 4 and ws % 2 == 0:  # two concurrent disjoint DP groups (S = 2)
                leg(f"{spec.name}_two_stages", run_two_stages, spec, dev, ws, rank, a.steps,
                    a.warmup, cap, brief=False)
        if not a.no_parity:
            leg("f32", parity_check, dev, ws, rank, torch.float32, into=parity, brief=False)
            leg("bf16", parity_check, dev, ws, rank, torch.bfloat16, into=parity, brief=False)
            leg("int8", parity_q8, dev, ws, rank, into=parity, brief=False)
            leg("sharded", parity_sharded, dev, ws, rank, into=parity, brief=False)
            leg("a2a", parity_sharded, dev, ws, rank, "a2a", into=parity, brief=False)
            leg("a2a_bf16", parity_sharded, dev, ws, rank, "a2a", torch.bfloat16, into=parity,
                brief=False)
        if not a.no_dropin:
            em.line["dropin_pcie"] = leg("dropin_pcie", dropin_rate, spec, dev, ws, rank, 5,
                                         into={}, brief=False)
            leg(f"{spec.name}_dropin_device", dropin_rate, spec, dev, ws, rank, 10, "device",
                brief=False)
            leg(f"{spec.name}_dropin_device_eager", dropin_rate, spec, dev, ws, rank, 10,
                "device", "sync", None, False, brief=False)
            leg(f"{spec.name}_dropin_overlap", dropin_overlap, spec, dev, ws, rank, 5,
                brief=False)
        if ws == 1 and not a.no_cpu_baseline:
            # rank 0 at N = 1 (the reference's CPU path on one of this host's cores)
            em.running = "cpu_baseline"
            log("timing the CPU baseline")
            em.line["cpu_baseline"] = cpu_baseline(spec)
        elif ws > 1 and not a.no_cpu_baseline and not children_fit:
            # every rank on one GPU (a gloo rehearsal): a child per rank would put 2N + 1
            # processes on the card; the rank processes themselves run the N-core baseline
            em.running = "cpu_baseline (in the rank processes)"
            if a.deadline - _max_over_ranks(em.elapsed(), dev, ws) - 15 < 40:
                em.skipped.append("cpu_baseline")
            nthreads = torch.get_num_threads()
            if "cpu_baseline" not in em.skipped:
                r = _guard(cpu_baseline_dist, spec, ws, rank, 12.0,
                           dist.new_group(backend="gloo"))
                torch.set_num_threads(nthreads)
                if isinstance(r, dict):
                    r["ran_in"] = "the bench's rank processes (one GPU shared by all ranks)"
                em.line["cpu_baseline"] = r
                log(f"cpu_baseline done at {em.elapsed():.1f} s")
        elif ws > 1 and not a.no_cpu_baseline:
            # N CPU processes under gloo (one per rank, GPUs hidden): the reference's sequence
            # with its per-tensor all_reduce, N cores
            left = a.deadline - _max_over_ranks(em.elapsed(), dev, ws) - 15
            if left < 60:
                em.skipped.append("cpu_baseline")
            else:
                em.running = "cpu_baseline (child processes)"
                log("timing the CPU baseline (N CPU processes)")
                em.line["cpu_baseline"] = isolated_legs(a, dev, ws, rank, min(150.0, left),
                                                        "cpu_baseline", HIDE_GPUS)
                log(f"cpu_baseline done at {em.elapsed():.1f} s")
        if ws > 1 and not a.no_xgmi and not children_fit:
            em.skipped += ["peer_access_legs (one GPU shared by all ranks: a child per rank "
                           f"would put {2 * ws + 1} processes on it, the box allows 16)"] + [
                f"rccl_env_{name}" for name in RCCL_ENV_VARIANTS]
        elif ws > 1 and not a.no_xgmi:
            # last, in child processes: the direct peer-access exchange (IPC-mapped wires / θ,
            # one fused kernel), its parity check and the link probe
            left = a.deadline - _max_over_ranks(em.elapsed(), dev, ws) - 15
            if left < 60:
                em.skipped.append("peer_access_legs")
            else:
                em.running = "peer_access_legs (child processes)"
                r = isolated_legs(a, dev, ws, rank, min(240.0, left))
                if "extra" in r:
                    extra.update(r["extra"])
                    parity.update(r["parity"])
                    _xgmi_efficiency(em.line, extra, a.extra_tree, ws)
                else:
                    extra["peer_access_legs"] = r
                log(f"peer_access_legs done at {em.elapsed():.1f} s")
            for name, env in RCCL_ENV_VARIANTS.items():
                left = a.deadline - _max_over_ranks(em.elapsed(), dev, ws) - 15
                if left < 60:
                    em.skipped.append(f"rccl_env_{name}")
                    continue
                em.running = f"rccl_env_{name} (child processes)"
                extra[f"rccl_env_{name}"] = isolated_legs(a, dev, ws, rank, min(120.0, left),
                                                          "rccl_env", env)
                log(f"rccl_env_{name} done at {em.elapsed():.1f} s")
    em.running = "teardown"
    # every side leg's kernels read against the same-run copy and mix ceilings too
    for v in extra.values():
        if isinstance(v, dict):
            for key in ("kernels", "kernels_b2b"):
                if isinstance(v.get(key), dict):
                    v[key] = {k: with_copy_ceiling(e, ceiling) for k, e in v[key].items()}
            if isinstance(v.get("cold"), dict) and isinstance(v["cold"].get("kernels"), dict):
                v["cold"]["kernels"] = {k: with_copy_ceiling(e, ceiling)
                                        for k, e in v["cold"]["kernels"].items()}
    em.line["wall_s"] = round(em.elapsed(), 1)
    em.emit()
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    em.timer.cancel()


if __name__ == "__main__":
    main()
