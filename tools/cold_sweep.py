#!/usr/bin/env python3
"""Cold A/B of the product kernels (the state a DiLoCo outer step runs in: H inner steps have
evicted the Infinity Cache): the 256 MiB Infinity Cache is scrubbed (a 512 MiB dl_copy) before
every timed launch, variants interleaved round by round in one process (cdna_hip_programming.md
§5.4 rule 24); median / min ms and GB/s of algorithmic bytes.

    python tools/cold_sweep.py [--tree t125] [--rounds 11] [--out x.json] [--what flags,tiles]

flags : dl_tree_tune launch policy (NT loads / NT or write-through stores) of dl_delta_pack, dl_unpack_sgd,
        dl_delta_sgd one launch over the whole tree each. Plain loads and write-through stores
        exist only in the tuning build: make -C diloco-swarm_amd/csrc TUNING=1, then run with
        DILOCO_HIP_LIB=diloco-swarm_amd/lib/libdiloco_hip_tuning.so
tiles : the one-replica two-kernel step (dl_pack_sgd_tiled) at tile sizes 0 (whole-range
        launches), 1024 ... 16384 chunks, against the one-pass dl_delta_sgd
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diloco-swarm_amd"))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

from diloco_amd import _lib, synth  # noqa: E402
from diloco_amd.outer import OuterSync  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402


def timed_cold(fn, scrub):
    scrub()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1)


FLUSH_K = 3


def _span(body):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    body()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1)


def timed_flushed(fn, scrub, scrub_only_ms):
    """--flushed: FLUSH_K (scrub, fn) cycles and a closing scrub as one span, minus
    the same number of scrubs alone: fn charged with the HBM write-back of the lines it left
    dirty in the Infinity Cache (which the plain cold timing's end event does not wait for)."""
    scrub()

    def body():
        for _ in range(FLUSH_K):
            scrub()
            fn()
        scrub()

    return (_span(body) - scrub_only_ms) / FLUSH_K


def scrub_only_span(scrub, reps=5):
    def body():
        for _ in range(FLUSH_K + 1):
            scrub()

    scrub()
    return sorted(_span(body) for _ in range(reps))[reps // 2]


def summarize(ms, nbytes):
    ms = sorted(ms)
    med = ms[len(ms) // 2]
    return {"med_ms": round(med, 4), "min_ms": round(ms[0], 4),
            "med_GBs": round(nbytes / med / 1e6, 1), "best_GBs": round(nbytes / ms[0] / 1e6, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tree", default="t125")
    ap.add_argument("--rounds", type=int, default=11)
    ap.add_argument("--what", default="flags,tiles")
    ap.add_argument("--out", default=None)
    ap.add_argument("--wire", default="f32", help="flags: the wire of the two-kernel and "
                    "kept-wire engines (f32 | bf16)")
    ap.add_argument("--flushed", action="store_true",
                    help="time each launch with its own dirty-line write-back (timed_flushed)")
    a = ap.parse_args()
    from bench import Scrubber

    global timed_cold
    if a.flushed:
        plain = timed_cold  # noqa: F841 (kept for reference)

    dev = torch.device("cuda", 0)
    spec = get_tree(a.tree)
    P = spec.total()
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, dev), shapes)]
    synth.inner_tree_device([p.view(-1) for p in params], 1, 0, out=[p.view(-1) for p in params])
    scrub = Scrubber(dev)
    out = {"tree": a.tree, "params": P, "rounds": a.rounds}
    if a.flushed:
        base = scrub_only_span(scrub)
        out["flushed"] = {"cycles": FLUSH_K, "scrub_only_ms": round(base, 4)}
        timed_cold = lambda fn, scr: timed_flushed(fn, scr, base)  # noqa: E731
    what = a.what.split(",")
    if "flags" in what:
        wd = torch.bfloat16 if a.wire == "bf16" else torch.float32
        wb = 2 if a.wire == "bf16" else 4
        out["wire"] = a.wire
        two = OuterSync(params, world_size=1, fuse_single=False, tile_chunks=0, wire_dtype=wd)
        one = OuterSync(params, world_size=1, fuse_single=True)
        kept = OuterSync(params, world_size=1, fuse_single=True, keep_wire=True, wire_dtype=wd)
        for e in (two, one, kept):
            e.step()  # steady-state SGD mode from here on
        scratch = torch.empty_like(two.theta)
        kern = {"delta_pack": (two, two.pseudo_gradient, 8 + wb),
                "unpack_sgd": (two, two.apply, 20 + wb),
                "delta_sgd": (one, lambda: one._step(None), 24),
                "delta_pack_sgd": (kept, lambda: kept._step(None), 24 + wb),
                # the sharded step's write-back of θ into the inner params, and the per-step DP
                # grad sync's pack / average-back (GradSync) on the same tree
                # (timing only: scratch holds the gathered copy, the average is by 1)
                "scatter": (two, lambda: two.k.scatter(two.tree, -1, two.theta, 0), 8),
                "gather": (two, lambda: two.k.gather(two.tree, -1, 0, scratch), 8),
                "unpack_avg": (two, lambda: two.k.unpack_avg(two.tree, -1, scratch, 1, 0), 8)}
        half = (two.tree.n_chunks + 1) // 2
        # (flags, grid): grid half = two chunks per workgroup (grid-stride walk)
        pr = _lib.TUNE_PAIRS
        flag_names = {(1, 0): "nt_loads", (3, 0): "nt_loads+stores",
                      (1, half): "nt_loads,2chunks/wg", (3, half): "nt_loads+stores,2chunks/wg",
                      (_lib.TUNE_AUTO, 0): "auto"}
        if _lib.load().dl_tuning_build():  # policies only the tuning build instantiates
            flag_names.update({(0, 0): "plain", (2, 0): "nt_stores",
                               (1 | _lib.TUNE_WT_STORES, 0): "nt_loads+wt_stores",
                               (1 | pr, 0): "nt_loads,pairs", (3 | pr, 0): "nt_loads+stores,pairs"})
        res = {(k, f): [] for k in kern for f in flag_names}
        for _ in range(a.rounds):
            for (k, f) in res:
                eng, fn, _ = kern[k]
                eng.tree.tune(f[1], f[0])
                res[(k, f)].append(timed_cold(fn, scrub))
        for e in (two, one, kept):
            e.tree.tune(0, _lib.TUNE_AUTO)
        out["flags"] = {}
        for (k, f), ms in res.items():
            s = summarize(ms, kern[k][2] * P)
            out["flags"].setdefault(k, {})[flag_names[f]] = s
            print(f"{k:14s} {flag_names[f]:26s} med {s['med_ms']:.4f} ms {s['med_GBs']:7.1f} GB/s"
                  f"  best {s['best_GBs']:7.1f}", flush=True)
        for e in (two, one, kept):
            e.close()
    if "grids" in what:
        # resident-grid caps (dl_tree_tune max_blocks, grid-stride walk): k workgroups per CU
        # instead of one workgroup per chunk (tools/occupancy.hip: the memory system saturates
        # with very few waves), AUTO policy, the one-pass kept-wire step and the SGD unpack
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        kept = OuterSync(params, world_size=1, fuse_single=True, keep_wire=True)
        two = OuterSync(params, world_size=1, fuse_single=False, tile_chunks=0)
        for e in (kept, two):
            e.step()
        kern = {"delta_pack_sgd": (kept, lambda: kept._step(None), 28),
                "unpack_sgd": (two, two.apply, 24), "delta_pack": (two, two.pseudo_gradient, 12)}
        grids = {0: "one WG per chunk"}
        grids.update({k * cus: f"{k} WG/CU resident" for k in (1, 2, 3, 4, 6)})
        res = {(k, g): [] for k in kern for g in grids}
        for _ in range(a.rounds):
            for (k, g) in res:
                eng, fn, _ = kern[k]
                eng.tree.tune(g, _lib.TUNE_AUTO)
                res[(k, g)].append(timed_cold(fn, scrub))
        for e in (kept, two):
            e.tree.tune(0, _lib.TUNE_AUTO)
        out["grids"] = {}
        for (k, g), ms in res.items():
            s = summarize(ms, kern[k][2] * P)
            out["grids"].setdefault(k, {})[grids[g]] = s
            print(f"{k:14s} {grids[g]:26s} med {s['med_ms']:.4f} ms {s['med_GBs']:7.1f} GB/s"
                  f"  best {s['best_GBs']:7.1f}", flush=True)
        for e in (kept, two):
            e.close()
    if "q8" in what:  # the int8 wire's kernels, one bucket (every launch covers the tree)
        from diloco_amd.kernels import Q8_SLOT

        e = OuterSync(params, world_size=1, wire_dtype=torch.int8, bucket_cap_elems=0)
        e.step()
        nch, m, _ = e.q8_plan[0]
        region = e.q8_region(0)
        slot_bytes = nch * Q8_SLOT
        half = (e.tree.n_chunks + 1) // 2

        def red():
            e.k.q8_reduce(region, 1, m, 1, region)

        def unpack():
            e.apply(0)

        kern = {"delta_q8": (lambda: e.pseudo_gradient(0), 8 * P + slot_bytes),
                "q8_reduce": (red, 2 * slot_bytes),
                "unpack_sgd_q8": (unpack, slot_bytes + 20 * P)}
        shapes = {(1, 0): "nt_loads", (3, 0): "nt_loads+stores", (1, half): "nt_loads,2chunks/wg",
                  (3, half): "nt_loads+stores,2chunks/wg", (_lib.TUNE_AUTO, 0): "auto"}
        if _lib.load().dl_tuning_build():  # AUTO already is write-through for the unpack
            shapes[(1 | _lib.TUNE_WT_STORES, 0)] = "nt_loads+wt_stores"
        res = {(k, f): [] for k in kern for f in shapes}
        for _ in range(a.rounds):
            for (k, f) in res:
                e.tree.tune(f[1], f[0])
                res[(k, f)].append(timed_cold(kern[k][0], scrub))
        e.tree.tune(0, _lib.TUNE_AUTO)
        out["q8"] = {}
        for (k, f), ms in res.items():
            s = summarize(ms, kern[k][1])
            out["q8"].setdefault(k, {})[shapes[f]] = s
            print(f"{k:14s} {shapes[f]:26s} med {s['med_ms']:.4f} ms {s['med_GBs']:7.1f} GB/s"
                  f"  best {s['best_GBs']:7.1f}", flush=True)
        e.close()
    if "pipe" in what:
        # a producer and its consumer (VERDICT/ADVICE r02: are plain stores worth it when the
        # next kernel re-reads the output?): the two-kernel step, whole range -- dl_delta_pack
        # then dl_unpack_sgd -- under AUTO (plain wire stores below 2^28 elements) against every
        # kernel's stores NT; and the DP grad sync's pack + average-back (dl_gather ->
        # dl_unpack_avg, the all-reduce of one replica being the identity)
        two = OuterSync(params, world_size=1, fuse_single=False, tile_chunks=0)
        two.step()
        scratch = torch.empty_like(two.theta)

        def step2():
            two.pseudo_gradient()
            two.apply()

        def sync2():
            two.k.gather(two.tree, -1, 0, scratch)
            two.k.unpack_avg(two.tree, -1, scratch, 1, 0)

        kern = {"delta_pack+unpack_sgd": (step2, 36), "gather+unpack_avg": (sync2, 16)}
        pol = {_lib.TUNE_AUTO: "auto", 3: "nt_loads+stores", 1: "nt_loads"}
        res = {(k, f): [] for k in kern for f in pol}
        for _ in range(a.rounds):
            for (k, f) in res:
                two.tree.tune(0, f)
                res[(k, f)].append(timed_cold(kern[k][0], scrub))
        two.tree.tune(0, _lib.TUNE_AUTO)
        out["pipe"] = {}
        for (k, f), ms in res.items():
            st = summarize(ms, kern[k][1] * P)
            out["pipe"].setdefault(k, {})[pol[f]] = st
            print(f"{k:22s} {pol[f]:18s} med {st['med_ms']:.4f} ms {st['med_GBs']:7.1f} GB/s"
                  f"  best {st['best_GBs']:7.1f}", flush=True)
        two.close()
    if "tiles" in what:
        engs = {}
        for tile in (0, 1024, 2048, 4096, 8192, 16384):
            engs[f"tile{tile}"] = OuterSync(params, world_size=1, fuse_single=False,
                                            tile_chunks=tile)
        engs["delta_sgd"] = OuterSync(params, world_size=1, fuse_single=True)
        for e in engs.values():
            e.step()
        res = {k: [] for k in engs}
        for _ in range(a.rounds):
            for k, e in engs.items():
                res[k].append(timed_cold(e.step, scrub))
        out["tiles"] = {}
        for k, ms in res.items():
            s = summarize(ms, 4 * P)  # GB/s params reduced (the metric)
            out["tiles"][k] = s
            print(f"step {k:10s} med {s['med_ms']:.4f} ms {s['med_GBs']:7.1f} GB/s params reduced"
                  f"  best {s['best_GBs']:7.1f}", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
