#!/usr/bin/env python3
"""A/B-only measurements moved out of bench.py: one GPU, one JSON object
on stdout, nothing the driver reads.

    python tools/bench_ab.py [--tree t125] [--steps 20] [--legs ceiling,two_kernel,...]

legs:
  ceiling      the same-run copy ceiling (dl_copy over 1 GiB, default / non-temporal policy,
               4 and 8 float4 loads in flight) and the pure read / write rates over 1-4
               streams (tools/rw_mix.hip's mix ceiling t >= R/read[s_r] + W/write[s_w]);
               reference rates of simpler access shapes, NOT bounds
  two_kernel   OuterSync's two-kernel step dl_delta_pack -> dl_unpack_sgd, whole-range and
               tiled (Infinity-Cache blocking), warm and cold, each kernel read against the
               ceilings
  fused        the one-pass step without the wire (dl_delta_sgd) and with it
               (dl_delta_pack_sgd), warm and cold (Infinity Cache scrubbed before each step)
"""
from __future__ import annotations

import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "diloco-swarm_amd"))


def copy_ceiling(dev, mib=1024, reps=15):
    """What the memory system gives streaming kernels on this box in this run (median launch):
    a two-stream dl_copy (4 / 8 loads in flight, default / nt policy; the fastest is "GBs")
    and pure reads / writes over 1-4 streams."""
    import torch

    from diloco_amd import _lib

    n = (mib << 20) // 4
    a = torch.ones(n, device=dev)
    b = torch.empty(n, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    out = {"bytes_per_copy": 2 * 4 * n}
    nt, wide = _lib.TUNE_NT_LOADS, _lib.COPY_WIDE

    def rate(flags, moved, nbytes=4 * n):
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
    """A roofline entry (bench.kernel_entry) also read against the same-run copy ceiling and,
    when it carries its byte mix (read_bytes / read_streams / write_bytes / write_streams),
    the mix ceiling (R + W) / (R / read_GBs[s_r] + W / write_GBs[s_w])."""
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
    return e


def step_legs(spec, dev, steps, ceiling, legs):
    """OuterSync's one-replica step forms, warm (events around each kernel, in the step) and
    cold (the Infinity Cache scrubbed before each step, outside the events)."""
    import torch

    import bench
    from diloco_amd.outer import ALL

    P = spec.total()
    out = {}
    forms = []
    if "two_kernel" in legs:
        forms += [("two_kernel", dict(fuse=False), 0), ("two_kernel_tiled", dict(fuse=False), None)]
    if "fused" in legs:
        forms += [("delta_sgd", dict(fuse=True), None),
                  ("delta_pack_sgd", dict(fuse=True, keep_wire=True), None)]
    for name, kw, tile in forms:
        eng = bench.build(spec, dev, 0, torch.float32, 64 << 20, **kw)
        if tile is not None:
            eng.tile_chunks = tile
        for _ in range(2):
            eng.step()
        rec = {}
        for mode in ("warm", "cold"):
            scr = bench.Scrubber(dev) if mode == "cold" else None
            ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
            for e in ev:
                if scr is not None:
                    scr()
                e[0].record()
                if name == "two_kernel":
                    eng.pseudo_gradient(ALL)
                    e[1].record()
                    eng.apply(ALL)
                    eng.steps_done += 1
                else:
                    eng._step(None)
                    e[1].record()
                e[2].record()
            torch.cuda.synchronize()
            if scr is not None:
                scr.close()
            step = sum(e[0].elapsed_time(e[2]) for e in ev) / steps
            r = {"step_ms": round(step, 5), "value": round(4.0 * P / (step * 1e-3) / 1e9, 1)}
            if name == "two_kernel":
                k1 = sum(e[0].elapsed_time(e[1]) for e in ev) / steps
                k2 = sum(e[1].elapsed_time(e[2]) for e in ev) / steps
                r["kernels"] = {
                    "delta_pack": with_copy_ceiling(bench.kernel_entry(
                        12 * P, k1, read_bytes=8 * P, read_streams=2, write_bytes=4 * P,
                        write_streams=1), ceiling),
                    "unpack_sgd": with_copy_ceiling(bench.kernel_entry(
                        24 * P, k2, read_bytes=12 * P, read_streams=3, write_bytes=12 * P,
                        write_streams=3), ceiling)}
            elif name in ("delta_sgd", "delta_pack_sgd"):
                nb = (28 if name == "delta_pack_sgd" else 24) * P
                r["kernel"] = with_copy_ceiling(bench.kernel_entry(
                    nb, step, read_bytes=12 * P, read_streams=3, write_bytes=nb - 12 * P,
                    write_streams=4 if name == "delta_pack_sgd" else 3), ceiling)
            rec[mode] = r
        out[name] = rec
        eng.close()
        del eng
        torch.cuda.empty_cache()
    return out


def main():
    import torch

    from diloco_amd import _lib
    from diloco_amd.trees import get_tree

    ap = argparse.ArgumentParser()
    ap.add_argument("--tree", default="t125")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--legs", default="ceiling,two_kernel,fused")
    a = ap.parse_args()
    legs = set(a.legs.split(","))
    _lib.load()
    dev = torch.device("cuda", 0)
    out = {"tree": a.tree}
    ceiling = copy_ceiling(dev) if "ceiling" in legs else None
    out["ceiling"] = ceiling
    out.update(step_legs(get_tree(a.tree), dev, a.steps, ceiling, legs))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
