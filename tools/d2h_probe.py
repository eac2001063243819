#!/usr/bin/env python3
"""Is a device->host copy into pinned memory fully visible to a host thread when
`stream.synchronize()` returns? (the gloo bf16 wrong-sum records.)

ProcessGroupGloo stages a CUDA tensor like this (AsyncAllreduceCUDAWork): an event recorded on
the caller's stream, a pool stream made to wait on it, `pinnedLike(t).copy_(t, non_blocking)`
on that stream, and later, on a gloo worker thread, `stream.synchronize()` followed at once by
the host-side ring reading the pinned buffer. This probe does exactly that with no gloo: per
iteration every bucket of a T1.3B-sized bf16 wire is written with a value of its own on the
current stream (after a spin kernel, so the copy's dependency is still pending when it is
queued: variant "dep"; or after a host synchronize: variant "nodep"), then staged the gloo
way; two host threads (gloo's default) synchronize each bucket's stream in order and scan the
pinned buffer right away. Any element that is not the bucket's value is stale; the report
gives the count, the 256-element blocks that hold them (mod 8: the XCD a round-robin
workgroup-to-XCD copy kernel would have written them from) and the first offsets.

    python tools/d2h_probe.py [--procs P] [--iters K] [--variants dep,nodep] [--nb NB]
"""
import argparse
import json
import os
import queue
import sys
import threading
import time

import numpy as np
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "diloco-swarm_amd"))


def bucket_sizes(nb):
    from diloco_amd.plan import plan_tables
    from diloco_amd.trees import get_tree

    num = get_tree("t1.3b").numels()
    seg, bnd = plan_tables(num)
    sizes = [int(seg[bnd[b + 1]] - seg[bnd[b]]) for b in range(len(bnd) - 1)]
    return sizes[:nb]


def scan(host, want_bits, m):
    a = host.view(torch.int16).numpy()[:m]
    bad = np.flatnonzero(a != want_bits)
    if bad.size == 0:
        return None
    blocks = np.unique(bad // 256)
    zero = int(np.count_nonzero(a[bad] == 0))
    return {"bad": int(bad.size), "zero": zero, "blocks": int(blocks.size),
            "xcd_hist": np.bincount(blocks % 8, minlength=8).tolist(),
            "first": bad[:4].tolist(), "first_blocks": blocks[:6].tolist()}


def worker(proc, nprocs, args, out_q):
    from diloco_amd import _lib

    torch.cuda.set_device(0)
    sizes = bucket_sizes(args.nb)
    dev = [torch.empty(m, dtype=torch.bfloat16, device="cuda") for m in sizes]
    torch.cuda.synchronize()
    res = {"proc": proc, "variants": {}}
    for variant in args.variants.split(","):
        stats = {"buckets": 0, "stale_buckets": 0, "records": [], "host_new_allocs": []}
        for it in range(args.iters):
            del_hosts = []
            torch._C._host_emptyCache()
            h0 = torch.cuda.host_memory_stats().get("num_host_alloc", 0)
            cur = torch.cuda.current_stream()
            q: "queue.Queue" = queue.Queue()
            found = []

            def check():
                while True:
                    item = q.get()
                    if item is None:
                        return
                    b, side, host, bits, m = item
                    side.synchronize()  # gloo: streams[i].synchronize() in run()
                    r = scan(host, bits, m)
                    if r is not None:
                        r.update(bucket=b, iter=it)
                        found.append(r)

            ths = [threading.Thread(target=check) for _ in range(2)]
            for t in ths:
                t.start()
            for b, d in enumerate(dev):
                # a distinct bf16 value per (proc, variant iteration, bucket): exact in bf16
                val = float(1 + ((proc * 131 + it * 17 + b) % 120) / 8.0)
                bits = int(torch.tensor([val], dtype=torch.bfloat16).view(torch.int16).item())
                if variant == "dep":
                    _lib.call("dl_spin", args.spin_us * 1000, cur.cuda_stream)
                d.fill_(val)
                if variant == "nodep":
                    cur.synchronize()
                ev = torch.cuda.Event()
                ev.record(cur)
                side = torch.cuda.Stream(priority=-1)  # from torch's stream pool, as gloo's
                side.wait_event(ev)
                with torch.cuda.stream(side):
                    host = torch.empty(d.numel(), dtype=torch.bfloat16, pin_memory=True)
                    host.copy_(d, non_blocking=True)
                del_hosts.append(host)
                q.put((b, side, host, bits, d.numel()))
            for _ in ths:
                q.put(None)
            for t in ths:
                t.join()
            torch.cuda.synchronize()
            stats["buckets"] += len(dev)
            stats["stale_buckets"] += len(found)
            stats["records"] += found[:4]
            stats["host_new_allocs"].append(
                torch.cuda.host_memory_stats().get("num_host_alloc", 0) - h0)
            del del_hosts
        res["variants"][variant] = stats
    out_q.put(res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=1)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--nb", type=int, default=25)
    ap.add_argument("--spin-us", type=int, default=10_000)
    ap.add_argument("--variants", default="dep,nodep")
    args = ap.parse_args()
    t0 = time.time()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(i, args.procs, args, q)) for i in range(args.procs)]
    for p in ps:
        p.start()
    res = [q.get() for _ in ps]
    for p in ps:
        p.join()
    summary = {}
    for v in args.variants.split(","):
        summary[v] = {"buckets": sum(r["variants"][v]["buckets"] for r in res),
                      "stale_buckets": sum(r["variants"][v]["stale_buckets"] for r in res),
                      "host_new_allocs": [r["variants"][v]["host_new_allocs"] for r in res][:2],
                      "records": [x for r in res for x in r["variants"][v]["records"]][:6]}
    print(json.dumps({"procs": args.procs, "iters": args.iters, "nb": args.nb,
                      "summary": summary, "s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
