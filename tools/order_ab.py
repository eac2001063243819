#!/usr/bin/env python3
"""A/B of the two-kernel outer step's launch flags, interleaved in one process (guide §5.4
rule 24): dl_delta_pack then dl_unpack_sgd, each with its own dl_tree_tune flags, timed as a
pair with HIP events around both. Tests whether walking dl_unpack_sgd last chunk first
(DL_TUNE_REVERSE) reuses the wire/θ bytes dl_delta_pack just streamed through the Infinity
Cache.

    python tools/order_ab.py [--tree t125] [--rounds 20] [--out file.json]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diloco-swarm_amd"))

import torch  # noqa: E402

from diloco_amd import _lib, synth  # noqa: E402
from diloco_amd.outer import OuterSync  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402

L, S, R = _lib.TUNE_NT_LOADS, _lib.TUNE_NT_STORES, _lib.TUNE_REVERSE
VARIANTS = {  # name: (delta_pack flags, unpack_sgd flags)
    "auto (fwd/fwd)": (L, L | S),
    "unpack reversed": (L, L | S | R),
    "unpack reversed, plain stores": (L, L | R),
    "delta plain loads, unpack reversed": (0, L | S | R),
    "delta plain loads, unpack fwd": (0, L | S),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tree", default="t125")
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = get_tree(a.tree)
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, dev), shapes)]
    eng = OuterSync(params, world_size=1, fuse_single=False, side_stream=False,
                    bucket_cap_elems=0)
    synth.inner_tree_device([p.view(-1) for p in params], 1, 0, out=[p.view(-1) for p in params])
    eng.step()  # steady-state SGD mode from here on
    P = spec.total()
    res = {k: {"step": [], "delta": [], "unpack": []} for k in VARIANTS}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for _ in range(a.rounds):
        for k, (fd, fu) in VARIANTS.items():
            for _rep in range(2):  # second rep is the recorded one (same variant twice in a row)
                ev[0].record()
                eng.tree.tune(0, fd)
                eng.pseudo_gradient()
                ev[1].record()
                eng.tree.tune(0, fu)
                eng.apply()
                ev[2].record()
                ev[2].synchronize()
                eng.steps_done += 1
            res[k]["step"].append(ev[0].elapsed_time(ev[2]))
            res[k]["delta"].append(ev[0].elapsed_time(ev[1]))
            res[k]["unpack"].append(ev[1].elapsed_time(ev[2]))
    eng.tree.tune(0, _lib.TUNE_AUTO)
    out = {"tree": spec.name, "params": P, "rounds": a.rounds, "variants": {}}
    for k, d in res.items():
        row = {}
        for part, ms in d.items():
            ms = sorted(ms)
            row[part + "_med_ms"] = round(ms[len(ms) // 2], 4)
            row[part + "_min_ms"] = round(ms[0], 4)
        row["step_GBs_params"] = round(4 * P / row["step_med_ms"] / 1e6, 1)
        out["variants"][k] = row
        print(f"{k:40s} step {row['step_med_ms']:.4f} ms  delta {row['delta_med_ms']:.4f}  "
              f"unpack {row['unpack_med_ms']:.4f}  -> {row['step_GBs_params']} GB/s")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
