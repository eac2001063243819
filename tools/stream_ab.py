#!/usr/bin/env python3
"""Where the gap between the headline's ms/step and the fused kernel's own duration goes.

Warm, T125, the N = 1 headline engine (dl_delta_pack_sgd), variants interleaved round by round
in one process, K steps per timed window (events on the current stream):

  step_side      eng.step() with the engine's side stream (two stream joins per step; default)
  step_nojoin    same engine, the loop run under `with torch.cuda.stream(eng.stream)` (joins
                 become same-stream no-ops)
  step_cur       the same engine with its side stream switched off (the kernel on the caller's
                 stream, as side_stream=False builds it)
  kernel_b2b     the bare C-ABI launch back to back (lower bound: no Python, no bind)
  host_us        host time of one eng.step() call (no synchronisation), to see host-boundness

    python tools/stream_ab.py [--rounds 7] [--steps 20] [--out x.json]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diloco-swarm_amd"))

import torch  # noqa: E402

from diloco_amd import synth  # noqa: E402
from diloco_amd.outer import OuterSync  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402


def window(fn, k, stream=None):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(k):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tree", default="t125")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = get_tree(a.tree)
    P = spec.total()
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, dev), shapes)]
    synth.inner_tree_device([p.view(-1) for p in params], 1, 0, out=[p.view(-1) for p in params])
    side = OuterSync(params, world_size=1, fuse_single=True, keep_wire=True, side_stream=True)
    side.step()
    S = side.stream

    def nojoin():
        with torch.cuda.stream(S):
            side.step()

    def on_cur():
        side.stream = None
        try:
            side.step()
        finally:
            side.stream = S

    def b2b():
        side.k.delta_pack_sgd(side.tree, -1, 0, side.theta, side.wire, side.mom, side.lr,
                              side.momentum, side.nesterov, False)

    var = {"step_side": (side.step, None), "step_nojoin": (nojoin, S),
           "step_cur": (on_cur, None), "kernel_b2b": (b2b, None)}
    res = {k: [] for k in var}
    host = []
    for _ in range(a.rounds):
        for k, (fn, st) in var.items():
            res[k].append(window(fn, a.steps, st))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            side.step()
        host.append((time.perf_counter() - t0) / a.steps * 1e6)
        torch.cuda.synchronize()
    out = {"tree": a.tree, "params": P, "rounds": a.rounds, "steps": a.steps}
    for k, ms in res.items():
        ms = sorted(ms)
        med = ms[len(ms) // 2]
        out[k] = {"med_ms": round(med, 4), "min_ms": round(ms[0], 4),
                  "value_GBs": round(4 * P / med / 1e6, 1)}
        print(f"{k:12s} med {med:.4f} ms/step  {4 * P / med / 1e6:7.1f} GB/s (4P/t)", flush=True)
    host.sort()
    out["host_us_per_step"] = round(host[len(host) // 2], 1)
    print(f"host         {out['host_us_per_step']} us per eng.step() call", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
