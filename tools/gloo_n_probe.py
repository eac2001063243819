#!/usr/bin/env python3
"""Is the slow N = 4 gloo rehearsal gloo's own behaviour on device tensors, or something the
outer model's exchange does? N processes on the one GPU, plain torch only (no library kernel):
T125's two buckets (2 x 64 Mi floats), exchanged per step in several ways, each timed over a
few steps after one warm-up (max over ranks, ms per step):

  ar_sync        all_reduce of two separate tensors, one after the other (WORLD)
  ar_async       the same issued async_op=True back to back, then waited
  ar_async_view  async, the two buckets as views of one arena
  ar_async_sub   async on a subgroup of every rank made with use_local_synchronization=True
  rs_ag_async    the sharded exchange's pattern on views of one arena (WORLD): every bucket's
                 reduce_scatter into this rank's slice issued async; then per bucket wait, an
                 all_gather of the slice issued async; then wait all
  rs_ag_sub      rs_ag_async on the use_local_synchronization subgroup
  rs_only        the two buckets' reduce_scatters alone (async, then waited)
  ag_only        the two buckets' all_gathers alone (async, then waited)
  rs_sync        the two reduce_scatters synchronously

    python tools/gloo_n_probe.py N [STEPS]
"""
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

B = 64 << 20  # floats per bucket


def worker(rank, n, port, steps, q):
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n)
    sub = dist.new_group(list(range(n)), backend="gloo", use_local_synchronization=True)
    sep = [torch.full((B,), float(rank + 1), device="cuda") for _ in range(2)]
    arena = torch.full((2 * B,), float(rank + 1), device="cuda")
    views = [arena[:B], arena[B:]]
    s = B // n

    def ar(bufs, g, async_op):
        if not async_op:
            for b in bufs:
                dist.all_reduce(b, group=g)
            return
        ws = [dist.all_reduce(b, group=g, async_op=True) for b in bufs]
        for w in ws:
            w.wait()

    def rs_ag(g):
        rs = [dist.reduce_scatter_tensor(v[rank * s:(rank + 1) * s], v, group=g, async_op=True)
              for v in views]
        ag = []
        for v, w in zip(views, rs):
            w.wait()
            ag.append(dist.all_gather_into_tensor(v, v[rank * s:(rank + 1) * s], group=g,
                                                  async_op=True))
        for w in ag:
            w.wait()

    def rs_only(sync=False):
        ws = [dist.reduce_scatter_tensor(v[rank * s:(rank + 1) * s], v, async_op=not sync)
              for v in views]
        for w in ws:
            if w is not None:
                w.wait()

    def ag_only():
        ws = [dist.all_gather_into_tensor(v, v[rank * s:(rank + 1) * s], async_op=True)
              for v in views]
        for w in ws:
            w.wait()

    modes = {"ar_sync": lambda: ar(sep, None, False), "ar_async": lambda: ar(sep, None, True),
             "ar_async_view": lambda: ar(views, None, True),
             "ar_async_sub": lambda: ar(sep, sub, True),
             "rs_ag_async": lambda: rs_ag(None), "rs_ag_sub": lambda: rs_ag(sub),
             "rs_only": rs_only, "ag_only": ag_only, "rs_sync": lambda: rs_only(True)}
    only = os.environ.get("PROBE_MODES")
    if only:
        modes = {k: v for k, v in modes.items() if k in only.split(",")}
    out = {}
    for name, f in modes.items():
        times = []
        for i in range(steps + 1):
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            f()
            torch.cuda.synchronize()
            if i:
                times.append(time.perf_counter() - t0)
        t = torch.tensor([sum(times) / len(times)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out[name] = round(t.item() * 1e3, 1)
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    n = int(sys.argv[1])
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, n, port, steps, q)) for r in range(n)]
    for p in ps:
        p.start()
    res = q.get()
    for p in ps:
        p.join()
    print(json.dumps({"n": n, "ms_per_step": res, "torch": torch.__version__}), flush=True)
