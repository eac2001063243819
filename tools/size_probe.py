#!/usr/bin/env python3
"""Where the headline kernel's T125 shortfall comes from.

By rocprofv3 (`profiles/r06_kernel_table_{t125,t1.3b}.json`) dl_delta_pack_sgd runs at 0.740 of
8 TB/s over T125 and 0.793 over T1.3B; a straight line through the two gives ~43 µs per launch
that does not scale with the bytes, and the other NT-store SGD kernels show the same (~30-40 µs)
while the plain-store pack kernels do not. This probe times the kernel (OuterSync
fuse_single + keep_wire: one dl_delta_pack_sgd per step, 28 B/param) with HIP events on the
launch stream over trees that separate the candidate causes:

  t125         GPT-2 125M shapes, every inner tensor its own allocation (the bench's layout)
  t125_arena   the same shapes as views of one allocation
  flat125      one tensor of T125's element count
  t125x10      ten copies of the T125 shapes (1.24 B params, T125's tensor mix at T1.3B size)
  flat1.3b     one tensor of T1.3B's element count
  t1.3b        GPT-2 1.3B shapes, separate allocations

warm: 30 launches back to back between two events (the bench's regime); cold: each launch
after a 512 MiB default-policy copy (outside the events) that evicts the Infinity Cache.
Trees are interleaved round by round.

    python tools/size_probe.py --rounds 3 --out gpurun_out/size_probe.json
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diloco-swarm_amd"))

import torch  # noqa: E402

from diloco_amd.outer import OuterSync  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402

BPP = 28  # read θ, inner, momentum; write wire, θ, momentum, inner
PEAK = 8000.0


def shapes_of(name):
    if name in ("t125", "t125_arena"):
        return [s for _, s in get_tree("t125").params()]
    if name == "t125x10":
        return [s for _, s in get_tree("t125").params()] * 10
    if name == "flat125":
        return [(get_tree("t125").total(),)]
    if name == "flat1.3b":
        return [(get_tree("t1.3b").total(),)]
    return [s for _, s in get_tree("t1.3b").params()]


def make(name, dev):
    shapes = shapes_of(name)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    if name == "t125_arena":
        n = sum(torch.Size(s).numel() for s in shapes)
        arena = torch.empty(n, device=dev)
        params, o = [], 0
        for s in shapes:
            k = torch.Size(s).numel()
            params.append(arena[o:o + k].view(s))
            o += k
    else:
        params = [torch.empty(s, device=dev) for s in shapes]
    for p in params:
        p.uniform_(-0.05, 0.05, generator=g)
    eng = OuterSync(params, world_size=1, fuse_single=True, keep_wire=True)
    eng.step()  # the first (momentum-creating) step; later ones are the steady kernel
    eng.step()
    return params, eng, sum(p.numel() for p in params)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--warm", type=int, default=30)
    ap.add_argument("--cold", type=int, default=8)
    ap.add_argument("--trees", default="t125,t125_arena,flat125,t125x10,flat1.3b,t1.3b")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    names = a.trees.split(",")
    objs = {n: make(n, dev) for n in names}
    flush_src = torch.empty(128 << 20, device=dev)  # 512 MiB
    flush_dst = torch.empty_like(flush_src)
    res = {n: {"warm_us": [], "cold_us": []} for n in names}
    s = torch.cuda.current_stream(dev)
    for r in range(a.rounds):
        for n in names:
            _, eng, _ = objs[n]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            eng.step()
            e0.record(s)
            for _ in range(a.warm):
                eng.step()
            e1.record(s)
            e1.synchronize()
            res[n]["warm_us"].append(e0.elapsed_time(e1) * 1e3 / a.warm)
            cold = []
            for _ in range(a.cold):
                flush_dst.copy_(flush_src)
                c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                c0.record(s)
                eng.step()
                c1.record(s)
                c1.synchronize()
                cold.append(c0.elapsed_time(c1) * 1e3)
            res[n]["cold_us"].append(sorted(cold)[len(cold) // 2])
            print(f"round {r} {n}: warm {res[n]['warm_us'][-1]:.1f} us, cold median "
                  f"{res[n]['cold_us'][-1]:.1f} us", flush=True)
    out = {"bytes_per_param": BPP, "trees": {}}
    for n in names:
        P = objs[n][2]
        nbytes = BPP * P
        w = sorted(res[n]["warm_us"])[len(res[n]["warm_us"]) // 2]
        c = sorted(res[n]["cold_us"])[len(res[n]["cold_us"]) // 2]
        out["trees"][n] = {"params": P, "tensors": len(objs[n][0]), "bytes": nbytes,
                           "warm_us": round(w, 1), "cold_us": round(c, 1),
                           "warm_frac": round(nbytes / w / 1e3 / PEAK, 4),
                           "cold_frac": round(nbytes / c / 1e3 / PEAK, 4),
                           "rounds": res[n]}
        print(f"{n:11s} {len(objs[n][0]):5d} tensors {P:>13,d} params  warm {w:9.1f} us "
              f"({out['trees'][n]['warm_frac']:.3f})  cold {c:9.1f} us "
              f"({out['trees'][n]['cold_frac']:.3f})")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
