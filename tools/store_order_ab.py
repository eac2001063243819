#!/usr/bin/env python3
"""Write-path A/B of the headline kernel dl_delta_pack_sgd.

The kernel reads 3 streams (θ, inner, momentum: 12 B/param) and writes 4 (wire, θ, momentum,
inner: 16 B/param); at T1.3B it runs at 0.707 of the 8 TB/s peak while dl_delta_sgd (one
written stream fewer) runs at 0.783 -- the write path is the limiter. This tool builds
variants of the library that differ only in how the kernel issues its stores, loads them all
into ONE process (ctypes, each its own copy of the library), and times the kernel of every
variant on the same buffers, interleaved round by round, with HIP events on the stream the
kernels are launched on:

  base        the product build (SGD arithmetic, then wire, θ, momentum, inner; NT stores;
              from round 6, XCD runs of 16 chunks below 2^28 elements)
  plain       the product build with plain stores (dl_tree_tune(NT loads only))
  wire_first  the wire's rows stored right after the subtraction, before the SGD arithmetic
  rows        row by row across the four streams (wire, θ, momentum, inner per float4 row)
  reverse     inner, momentum, θ, then the wire
  wire_plain  the wire stored plainly, θ / momentum / inner non-temporally
  xcd_contig  XCD x walks the x-th eighth of the chunk range in order (not interleaved)
  base_again  the product build once more, timed as a variant of its own: the spread between
              two identical kernels is the A/B's noise floor
  xcd_b<B>    XCD x walks runs of B consecutive chunks at every size (xcd_b1: the
              dispatcher's interleave, the product's mapping up to round 5)

    python tools/store_order_ab.py --build                  # here (hipcc, no GPU)
    python tools/store_order_ab.py --tree t1.3b --rounds 6  # on the GPU box
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "diloco-swarm_amd"))
OUT = os.path.join(REPO, "build_ab", "store_order")
CSRC = os.path.join(REPO, "diloco-swarm_amd", "csrc")
FLAGS = ("--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fvisibility=hidden -ffp-contract=off "
         "-fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero").split()
SRCS = ["dl_kernels.hip", "dl_q8.hip", "dl_xgmi.hip", "dl_comm.hip", "dl_abi.hip"]
VARIANTS = {"base": [], "wire_first": ["-DDL_DPS_ORDER=1"], "rows": ["-DDL_DPS_ORDER=2"],
            "reverse": ["-DDL_DPS_ORDER=3"], "wire_plain": ["-DDL_DPS_WIRE_PLAIN"],
            "xcd_b1": ["-DDL_XCD_XLOG=0"], "xcd_contig": ["-DDL_XCD_XLOG=-1"],
            "xcd_b4": ["-DDL_XCD_XLOG=2"], "xcd_b8": ["-DDL_XCD_XLOG=3"],
            "xcd_b16": ["-DDL_XCD_XLOG=4"], "xcd_b32": ["-DDL_XCD_XLOG=5"],
            "xcd_b64": ["-DDL_XCD_XLOG=6"], "xcd_b256": ["-DDL_XCD_XLOG=8"],
            "xcd_b2048": ["-DDL_XCD_XLOG=11"]}
DL_TUNE_NT_LOADS = 1


def build():
    os.makedirs(OUT, exist_ok=True)
    procs = []
    for name, defs in VARIANTS.items():
        cmd = ["/opt/rocm/bin/hipcc", *FLAGS, *defs, *SRCS, "-ldl", "-o",
               os.path.join(OUT, f"lib_{name}.so")]
        procs.append((name, subprocess.Popen(cmd, cwd=CSRC)))
    for name, p in procs:
        if p.wait() != 0:
            raise SystemExit(f"build of {name} failed")
    print("built", sorted(VARIANTS))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--tree", default="t1.3b")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None, help="comma-separated variants (plain: the base "
                    "library with plain stores)")
    a = ap.parse_args()
    if a.build:
        build()
        return
    import torch

    from diloco_amd import _lib, synth
    from diloco_amd.trees import get_tree

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    spec = get_tree(a.tree)
    numels = spec.numels()
    P = spec.total()
    inner = synth.outer_tree_device(spec, dev)
    libs, trees = {}, {}
    i64 = ctypes.c_int64
    arr = (i64 * len(numels))(*numels)
    for name in ([n for n in VARIANTS if n in set(a.only.split(",")) | {"base"}]
                 if a.only else VARIANTS):
        lib = ctypes.CDLL(os.path.join(OUT, f"lib_{name}.so"), mode=ctypes.RTLD_LOCAL)
        for fn, args in _lib.SIGNATURES.items():
            f = getattr(lib, fn)
            f.restype, f.argtypes = args
        t = ctypes.c_void_p()
        assert lib.dl_tree_create(arr, len(numels), 1 << 62, ctypes.byref(t)) == 0
        libs[name], trees[name] = lib, t
    total = ctypes.c_int64()
    ns, nb, nc = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    libs["base"].dl_tree_query(trees["base"], ctypes.byref(total), ctypes.byref(ns),
                               ctypes.byref(nb), ctypes.byref(nc))
    theta = torch.empty(total.value, device=dev)
    wire = torch.empty(total.value, device=dev)
    mom = torch.zeros(total.value, device=dev)
    theta.uniform_(-0.02, 0.02)
    stream = torch.cuda.current_stream(dev)
    s = stream.cuda_stream
    ptrs = (ctypes.c_uint64 * len(inner))(*[x.data_ptr() for x in inner])
    for name in libs:
        assert libs[name].dl_tree_bind(trees[name], 0, ptrs, len(inner), s) == 0
    runs = [(n, n, None) for n in VARIANTS] + [("plain", "base", DL_TUNE_NT_LOADS),
                                                ("base_again", "base", None)]
    if a.only:
        keep = set(a.only.split(",")) | {"base", "base_again"}
        runs = [r for r in runs if r[0] in keep]

    def launch(lib, tree):
        rc = lib.dl_delta_pack_sgd(tree, -1, 0, theta.data_ptr(), wire.data_ptr(), 0,
                                   mom.data_ptr(), 0.7, 0.9, 1, 0, s)
        assert rc == 0, lib.dl_last_error()

    res = {r[0]: [] for r in runs}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for rnd in range(a.rounds + 1):  # round 0: warm-up of every variant
        # the order rotates every round: a variant's position in the round (the first one runs
        # right after the previous round's synchronize) must not bias its time
        k = rnd % len(runs)
        for label, name, flags in runs[k:] + runs[:k]:
            lib, tree = libs[name], trees[name]
            lib.dl_tree_tune(tree, 0, -1 if flags is None else flags)
            launch(lib, tree)
            ev[0].record(stream)
            for _ in range(a.launches):
                launch(lib, tree)
            ev[1].record(stream)
            torch.cuda.synchronize()
            if rnd:
                res[label].append(ev[0].elapsed_time(ev[1]) / a.launches)
        print(f"round {rnd} " + " ".join(f"{k} {v[-1]:.4f}" for k, v in res.items() if v),
              flush=True)
    import statistics

    out = {"tree": a.tree, "params": P, "bytes_per_launch": 28 * P, "rounds": a.rounds,
           "launches_per_round": a.launches, "kernel": "dl_delta_pack_sgd (fp32 wire, MODE 2)",
           "variants": {}}
    for k, v in res.items():
        med = statistics.median(v)
        out["variants"][k] = {"ms_median": round(med, 5), "ms_min": round(min(v), 5),
                              "ms_max": round(max(v), 5),
                              "TBs": round(28 * P / med / 1e9, 4),
                              "frac_of_8TBs": round(28 * P / med / 1e9 / 8.0, 4)}
    base = out["variants"]["base"]["ms_median"]
    for k, v in out["variants"].items():
        v["vs_base"] = round(base / v["ms_median"], 4)
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
