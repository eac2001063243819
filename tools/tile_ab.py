#!/usr/bin/env python3
"""A/B of the cache-blocked two-kernel outer step (dl_pack_sgd_tiled), interleaved in one
process (guide §5.4 rule 24): for every tile size and launch-flag set, K back-to-back outer
steps of the one-replica pipeline dl_delta_pack -> dl_unpack_sgd timed with HIP events, in
rotating order, median over rounds. Tile 0 = the whole-range launches (no blocking); the
one-pass dl_delta_sgd is timed beside them as the floor.

    python tools/tile_ab.py [--tree t125] [--rounds 12] [--steps 10] [--out file.json]

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

from diloco_amd import _lib, synth  # noqa: E402
from diloco_amd.outer import OuterSync  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402

L, S = _lib.TUNE_NT_LOADS, _lib.TUNE_NT_STORES
FLAGS = {"auto": _lib.TUNE_AUTO, "plain": 0, "nt-stores": S, "nt-loads": L}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tree", default="t125")
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--tiles", default="0,256,512,1024,2048,4096")
    ap.add_argument("--flags", default="auto,plain,nt-stores")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = get_tree(a.tree)
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, dev), shapes)]
    eng = OuterSync(params, world_size=1, fuse_single=False, side_stream=False, tile_chunks=0)
    synth.inner_tree_device([p.view(-1) for p in params], 1, 0, out=[p.view(-1) for p in params])
    eng.step()  # steady-state SGD mode from here on
    P = spec.total()
    variants = [(t, f) for f in a.flags.split(",") for t in map(int, a.tiles.split(","))]
    variants.append(("fused", "auto"))
    res = {v: [] for v in variants}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        order = variants[r % len(variants):] + variants[:r % len(variants)]
        for tile, fl in order:
            eng.tree.tune(0, FLAGS[fl])
            eng.fuse_single = tile == "fused"
            eng.tile_chunks = 0 if tile == "fused" else tile
            eng.step()  # one untimed step of this variant
            e0.record()
            for _ in range(a.steps):
                eng.step()
            e1.record()
            e1.synchronize()
            res[(tile, fl)].append(e0.elapsed_time(e1) / a.steps)
    eng.tree.tune(0, _lib.TUNE_AUTO)
    out = {"tree": spec.name, "params": P, "rounds": a.rounds, "steps": a.steps,
           "chunks": eng.tree.n_chunks, "variants": []}
    for (tile, fl), ms in res.items():
        ms = sorted(ms)
        med = ms[len(ms) // 2]
        row = {"tile_chunks": tile, "flags": fl, "med_ms": round(med, 4),
               "min_ms": round(ms[0], 4), "GBs_params": round(4 * P / med / 1e6, 1)}
        out["variants"].append(row)
        print(f"tile {str(tile):>6s} flags {fl:10s} step {med:.4f} ms (min {ms[0]:.4f}) "
              f"-> {row['GBs_params']} GB/s", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    eng.close()


if __name__ == "__main__":
    main()
