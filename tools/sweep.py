#!/usr/bin/env python3
"""A/B the walker launch shape (dl_tree_tune) on the real tree layout, interleaved in one
process (cdna_hip_programming.md §5.4 rule 24). Prints median / min ms and GB/s per variant.

    python tools/sweep.py [--tree t125] [--rounds 15]

Flags other than AUTO and NT loads [+ NT stores / DL_TUNE_PAIRS] exist only in the tuning
build: make -C diloco-swarm_amd/csrc TUNING=1 and DILOCO_HIP_LIB=<repo>/diloco-swarm_amd/lib/
libdiloco_hip_tuning.so (the product library rejects them).
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diloco-swarm_amd"))

import torch  # noqa: E402

from diloco_amd import synth  # noqa: E402
from diloco_amd.outer import OuterSync  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tree", default="t125")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = get_tree(a.tree)
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, dev), shapes)]
    eng = OuterSync(params, world_size=1)
    synth.inner_tree_device([p.view(-1) for p in params], 1, 0, out=[p.view(-1) for p in params])
    eng.step()  # momentum exists from here on: unpack_sgd in steady-state mode
    P = spec.total()
    variants = []
    for flags in (-1, 0, 1, 2, 3):
        for grid in (0, 2048, 8192):
            variants.append((flags, grid))
    res = {v: {"delta_pack": [], "unpack_sgd": []} for v in variants}
    for _ in range(a.rounds):
        for v in variants:
            eng.tree.tune(v[1], v[0])
            for name, fn in (("delta_pack", eng.pseudo_gradient), ("unpack_sgd", eng.apply)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                res[v][name].append(e0.elapsed_time(e1))
    bpp = {"delta_pack": 12, "unpack_sgd": 24}
    out = []
    for v in variants:
        row = {"flags": v[0], "grid": v[1]}
        for k, ms in res[v].items():
            ms = sorted(ms)
            med = ms[len(ms) // 2]
            row[k] = {"med_ms": round(med, 4), "min_ms": round(ms[0], 4),
                      "med_GBs": round(bpp[k] * P / med / 1e6, 1)}
        out.append(row)
        print(f"flags={v[0]} grid={v[1]:5d}  delta {row['delta_pack']['med_GBs']:7.1f} GB/s"
              f"  unpack_sgd {row['unpack_sgd']['med_GBs']:7.1f} GB/s")
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"tree": a.tree, "rounds": a.rounds, "variants": out}, f, indent=1)


if __name__ == "__main__":
    main()
