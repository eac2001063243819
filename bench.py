#!/usr/bin/env python3
"""Benchmark: DiLoCo outer step, device-resident, GB/s of parameters reduced.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--tree t125] [--wire f32|bf16]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

One step = one full outer step of src/train.py:261-269 over the whole synthetic tree on every
rank, device-resident (θ_outer, momentum and the wire buffer live in HBM):
    dl_delta_pack (wire = θ_outer - inner) -> [RCCL all_reduce(SUM) per bucket, pipelined]
    -> dl_unpack_sgd (g = wire/n, Nesterov SGD, inner = θ_outer)
Workload at N=1 is BASELINE config #2 (125M synthetic GPT-2 tree, 1 GPU, fp32); the same tree
per rank at every N (weak scaling; configs #3/#4 as N grows). value = N * 4 * params / t_step.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

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


def setup_dist(n_gpus):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={ws}; launch N>1 with torchrun")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if ws > 1:
        dist.init_process_group("nccl", device_id=dev)
    return ws, rank, dev


def build(spec, dev, rank, wire, cap):
    shapes = [s for _, s in spec.params()]
    theta0 = synth.outer_tree_device(spec, dev)
    params = [t.view(s) for t, s in zip(theta0, shapes)]
    eng = OuterSync(params, lr=0.7, momentum=0.9, nesterov=True, wire_dtype=wire,
                    bucket_cap_elems=cap)
    # inner = θ_0 + this rank's noise (stands in for H inner steps)
    synth.inner_tree_device([p.view(-1) for p in params], 1, rank, out=[p.view(-1) for p in params])
    return eng


def timed_launches(fn, reps):
    """Average ms per launch of `fn` over `reps` back-to-back launches, HIP events on the
    current stream (the stream every dl_* kernel is launched on)."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def run_tree(spec, dev, ws, rank, steps, warmup, wire, cap):
    eng = build(spec, dev, rank, wire, cap)
    P = spec.total()
    for _ in range(max(warmup, 1)):  # >= 1: the timed steps run the steady-state SGD mode
        eng.step()
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.step()
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    wbytes = 2 if wire == torch.bfloat16 else 4
    # per-kernel average durations: the same kernels on the same buffers, back to back
    reps = max(steps, 10)
    kern_ms = {
        "delta_pack": timed_launches(eng.pseudo_gradient, reps),
        "unpack_sgd": timed_launches(eng.apply, reps),
    }
    kern_bytes = {
        "delta_pack": (4 + 4 + wbytes) * P,             # read θ, inner; write wire
        "unpack_sgd": (wbytes + 4 + 4 + 4 + 4 + 4) * P,  # read wire, θ, buf; write θ, buf, inner
    }
    kernels = {}
    for k, b in kern_bytes.items():
        ms = kern_ms[k]
        ach = b / (ms * 1e-3) / 1e9
        kernels[k] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                      "bytes_per_launch": b, "avg_ms": round(ms, 5)}
    res = {
        "tree": spec.name, "params": P, "tensors": len(spec.params()),
        "padded": eng.tree.total, "buckets": eng.tree.n_buckets, "chunks": eng.tree.n_chunks,
        "ms_per_step": dt / steps * 1e3,
        "value": ws * 4.0 * P / (dt / steps) / 1e9,
        "kernels": kernels,
    }
    if ws == 1:
        dom = max(kernels, key=lambda k: kernels[k]["avg_ms"])
        res["roofline"] = dict(kernels[dom], kernel=dom)
    else:
        # the exchange: every bucket's all-reduce back to back (RCCL over xGMI)
        def allreduce_all():
            for b in range(eng.tree.n_buckets):
                eng.all_reduce(b, async_op=False)
        if ws > 1:
            dist.barrier()
        ar_ms = timed_launches(allreduce_all, max(3, steps // 2))
        t = torch.tensor([ar_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ar_ms = float(t.item())
        bus = 2.0 * (ws - 1) / ws * wbytes * eng.tree.total
        ach = bus / (ar_ms * 1e-3) / 1e9
        peak = (ws - 1) * XGMI_LINK_GBS
        res["roofline"] = {"bound": "xgmi", "achieved": round(ach, 1), "peak": peak,
                           "unit": "GB/s", "frac": round(ach / peak, 4), "traffic": None,
                           "kernel": "rccl all_reduce (all buckets)", "avg_ms": round(ar_ms, 4),
                           "bus_bytes_per_step": bus}
    eng.close()
    del eng
    torch.cuda.empty_cache()
    return res


def cpu_baseline(spec, seconds_budget=12.0):
    """The reference's per-tensor CPU sequence (oracle/torch_restatement.py), 1 thread."""
    sys.path.insert(0, HERE)
    from oracle.torch_restatement import time_steps

    numels = spec.numels()
    t, n = time_steps(numels, steps=2, threads=1, budget_s=seconds_budget)
    model = ""
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        model = next((l.split(":", 1)[1].strip() for l in out.splitlines()
                      if l.startswith("Model name")), "")
    except Exception:
        pass
    return {
        "value": round(4.0 * spec.total() / t / 1e9, 4), "unit": "GB/s", "cores": 1,
        "kind": "port",
        "sample": (f"{spec.name} full tree ({spec.total()} params), {n} timed outer steps after 1 "
                   f"warm step, per-tensor torch CPU restatement of src/utils.py:218-226 + "
                   f"torch SGD-Nesterov (sync_gradients is a no-op at n=1), 1 thread; "
                   f"{t:.3f} s/step"),
        "host": {"cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
                 "model": model, "torch": torch.__version__},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--tree", default="t125")
    ap.add_argument("--wire", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--bucket-mb", type=int, default=256)
    ap.add_argument("--extra-tree", default="t1.3b", help="second tree measured beside (or 'none')")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()

    ws, rank, dev = setup_dist(a.gpus)
    wire = torch.bfloat16 if a.wire == "bf16" else torch.float32
    cap = (a.bucket_mb << 20) // 4
    _lib.load()
    spec = get_tree(a.tree)
    log(f"rank {rank}/{ws} tree {spec.name} ({spec.total()} params) wire {a.wire}")
    main_res = run_tree(spec, dev, ws, rank, a.steps, a.warmup, wire, cap)
    extra = {}
    if a.extra_tree != "none" and a.extra_tree != a.tree:
        es = get_tree(a.extra_tree)
        r = run_tree(es, dev, ws, rank, max(3, a.steps // 4), 1, wire, cap)
        extra[es.name] = {k: r[k] for k in ("value", "ms_per_step", "roofline", "buckets", "params")}
    cpu = None
    if rank == 0 and ws == 1 and not a.no_cpu_baseline:
        log("timing the CPU baseline")
        cpu = cpu_baseline(spec)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(main_res["value"], 3),
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
                "workload": (f"DiLoCo outer step, {spec.name} tree per rank: delta_pack -> "
                             + ("RCCL all_reduce (bucketed, pipelined) -> " if ws > 1 else "")
                             + "unpack_sgd (+copy to inner)"),
                "tree": spec.name, "params": main_res["params"], "tensors": main_res["tensors"],
                "wire": a.wire, "buckets": main_res["buckets"], "chunks": main_res["chunks"],
                "parallelism": f"dp{ws}",
            },
            "roofline": main_res["roofline"],
            "cpu_baseline": cpu,
            "kernels": main_res["kernels"],
            "extra": extra or None,
            "host": platform.node(),
        }
        print(json.dumps(line), flush=True)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
