#!/usr/bin/env python3
"""Do kernels lose workgroups when several processes share one GPU?

tools/stripe_diag.py caught it in the config #5 test: on one of eight ranks, dl_fill_synth's
stores into the wte tensor were missing for every 256-element block whose index is p mod 8 --
the blocks of the workgroups with id = p mod 8, i.e. of one XCD -- and still missing after a
host synchronize: the stores never happened, although the kernel completed and the stream went
on. This stress isolates that from the outer step. P processes on the one GPU, each for S
seconds: fill a T1.3B-wte-sized fp32 buffer with dl_fill_synth (4096 workgroups x 256 threads,
grid-stride) alternating two seeds, copy a reference into a second buffer with torch (one
element block per workgroup, no grid stride), stage 64 MiB to pinned host memory (the DMA
traffic gloo adds), synchronize, and compare both buffers with their references. A lost
workgroup shows as wrong 256-element blocks; per failure the report gives the blocks by phase
(block index mod 8) and, per phase, the first and last bad block (where in the grid-stride
loop the workgroups stopped).

    python tools/wave_loss_stress.py [--procs P] [--seconds S] [--ballast-gb G] [--add]
        [--pin-churn-mb M] [--dev-churn-mb M]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "diloco-swarm_amd"))

N = 103_022_592  # T1.3B wte


def blocks_report(bad):
    """bad: bool tensor over N elements -> phases of the wrong 256-element blocks."""
    nb = N // 256
    blk = bad[:nb * 256].view(nb, 256).any(1)
    idx = torch.nonzero(blk).flatten().cpu()
    if idx.numel() == 0:
        return None
    ph = idx % 8
    out = {"blocks": int(idx.numel()), "elems": int(bad.sum()),
           "phase": torch.bincount(ph, minlength=8).tolist(), "span": {}}
    for p in range(8):
        sel = idx[ph == p]
        if sel.numel():
            out["span"][p] = [int(sel[0]), int(sel[-1]), int(sel.numel())]
    return out


def worker(proc, args, q):
    from diloco_amd import synth

    torch.cuda.set_device(0)
    ballast = (torch.empty(int(args.ballast_gb * (1 << 30)) // 4, device="cuda")
               if args.ballast_gb > 0 else None)
    refs = []
    for seed in (11, 12):
        r = torch.empty(N, device="cuda")
        synth.fill_device(r, seed, 0, 0.0, 0.02)
        torch.cuda.synchronize()
        again = torch.empty(N, device="cuda")
        synth.fill_device(again, seed, 0, 0.0, 0.02)
        torch.cuda.synchronize()
        assert torch.equal(r, again), "reference fills disagree"
        del again
        refs.append(r)
    x = torch.empty(N, device="cuda")
    y = torch.empty(N, device="cuda")
    host = torch.empty(16 << 20, pin_memory=True)
    zero = torch.zeros(N, device="cuda") if args.add else None
    churn = None
    it, fails = 0, []
    t_end = time.time() + args.seconds
    while time.time() < t_end:
        k = it & 1
        synth.fill_device(x, (11, 12)[k], 0, 0.0, 0.02, add=zero)
        y.copy_(refs[k])
        if args.pin_churn_mb:
            # while the fill runs: a fresh pinned block mapped into the GPU's address space and
            # the previous one unmapped (what gloo's staging allocator does on a cache miss)
            churn = None
            torch._C._host_emptyCache()
            churn = torch.empty((args.pin_churn_mb << 20) // 4, pin_memory=True)
            churn[:16 << 20].copy_(refs[k][:16 << 20], non_blocking=True)
        if args.dev_churn_mb:  # a device allocation returned to the driver and made again
            tmp = torch.empty((args.dev_churn_mb << 20) // 4, device="cuda")
            del tmp
            torch.cuda.empty_cache()
        host.copy_(refs[k][:16 << 20], non_blocking=True)
        torch.cuda.synchronize()
        for name, buf in (("fill_synth", x), ("torch_copy", y)):
            bad = buf != refs[k]
            if bool(bad.any()):
                r = blocks_report(bad)
                r.update(kernel=name, iter=it)
                fails.append(r)
        it += 1
    if ballast is not None:
        del ballast
    q.put({"proc": proc, "iters": it, "fails": fails[:8], "n_fails": len(fails)})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--ballast-gb", type=float, default=16)
    ap.add_argument("--add", action="store_true", help="the fill reads an operand (add=)")
    ap.add_argument("--pin-churn-mb", type=int, default=0)
    ap.add_argument("--dev-churn-mb", type=int, default=0)
    args = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(i, args, q)) for i in range(args.procs)]
    t0 = time.time()
    for p in ps:
        p.start()
    res = []
    while len(res) < len(ps):  # a line every 20 s: a long run is never silent
        try:
            res.append(q.get(timeout=20))
        except Exception:
            print(f"... {time.time() - t0:.0f} s, {len(res)} of {len(ps)} done", flush=True)
    for p in ps:
        p.join()
    res.sort(key=lambda r: r["proc"])
    print(json.dumps({"procs": args.procs, "seconds": args.seconds, "add": args.add,
                      "pin_churn_mb": args.pin_churn_mb, "dev_churn_mb": args.dev_churn_mb,
                      "iters": sum(r["iters"] for r in res),
                      "n_fails": sum(r["n_fails"] for r in res),
                      "per_proc": res, "wall_s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
