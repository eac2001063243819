#!/usr/bin/env python3
"""Clock-slotted launches (dl_tree_slot) of the one-replica fused step vs the plain walker, on
the product kernel (dl_delta_pack_sgd, or --kernel delta_sgd), cold (the Infinity Cache
scrubbed before every launch, as after H inner steps) and warm (back to back), variants
interleaved round by round in one process. Slot period P in 10-ns ticks, read window 0.38 P.

    python tools/slot_sweep.py [--tree t125] [--rounds 11] [--periods 3000,3400,...] [--out x.json]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diloco-swarm_amd"))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

from diloco_amd import synth  # noqa: E402
from diloco_amd.outer import OuterSync  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tree", default="t125")
    ap.add_argument("--rounds", type=int, default=11)
    ap.add_argument("--kernel", default="delta_pack_sgd", choices=["delta_pack_sgd", "delta_sgd"])
    ap.add_argument("--periods", default="3000,3200,3400,3600,3800,4000,4200")
    ap.add_argument("--read-frac", type=float, default=0.38)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from bench import Scrubber

    dev = torch.device("cuda", 0)
    spec = get_tree(a.tree)
    P = spec.total()
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, dev), shapes)]
    synth.inner_tree_device([p.view(-1) for p in params], 1, 0, out=[p.view(-1) for p in params])
    keep = a.kernel == "delta_pack_sgd"
    eng = OuterSync(params, world_size=1, fuse_single=True, keep_wire=keep)
    eng.step()  # steady-state SGD mode from here on
    nbytes = (28 if keep else 24) * P
    variants = [("walker", 0, 0)] + [(f"slotted P={p}", p, int(p * a.read_frac))
                                     for p in map(int, a.periods.split(","))]
    scrub = Scrubber(dev)
    cold = {v[0]: [] for v in variants}
    warm = {v[0]: [] for v in variants}
    for _ in range(a.rounds):
        for name, per, rd in variants:
            eng.tree.slot(per, rd)
            for kind, store in (("cold", cold), ("warm", warm)):
                if kind == "cold":
                    scrub()
                e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                e[0].record()
                eng._step(None)
                e[1].record()
                if kind == "warm":  # two more back to back, the last one timed
                    eng._step(None)
                    e[2].record()
                    eng._step(None)
                    e[3].record()
                    e[3].synchronize()
                    store[name].append(e[2].elapsed_time(e[3]))
                else:
                    e[1].synchronize()
                    store[name].append(e[0].elapsed_time(e[1]))
    eng.tree.slot(0, 0)
    scrub.close()

    def summ(ms):
        ms = sorted(ms)
        med = ms[len(ms) // 2]
        return {"med_ms": round(med, 4), "min_ms": round(ms[0], 4),
                "med_GBs": round(nbytes / med / 1e6, 1)}

    out = {"tree": a.tree, "params": P, "kernel": a.kernel, "rounds": a.rounds,
           "bytes": nbytes, "read_frac": a.read_frac,
           "cold": {k: summ(v) for k, v in cold.items()},
           "warm": {k: summ(v) for k, v in warm.items()}}
    for kind in ("cold", "warm"):
        base = out[kind]["walker"]["med_ms"]
        for k, v in out[kind].items():
            v["vs_walker"] = round(v["med_ms"] / base, 4)
            print(f"{kind:4s} {k:18s} {v['med_ms']:8.4f} ms {v['med_GBs']:8.1f} GB/s "
                  f"x{v['vs_walker']:.3f}", flush=True)
    eng.close()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
