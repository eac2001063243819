#!/usr/bin/env python3
"""How asynchronous is a gloo collective on device tensors in this torch build? Two processes
on the one GPU; each queues a 300 ms dl_spin on its current stream, then issues
dist.all_reduce / reduce_scatter_tensor / all_gather_into_tensor on a 64 MiB CUDA tensor with
async_op=True. Reported per collective: the host time the issuing call took, whether the Work
says it is completed when the call returns, and the time of work.wait(). An issue time of
about the spin means the call waited for the device before returning (the staging copy
ordered behind all earlier device work, and the host held): such a collective cannot race
its producer or its consumer, so the gloo tests cannot exercise asynchronous ordering.

    python tools/gloo_sync_probe.py
"""
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "diloco-swarm_amd"))


def worker(rank, port, q):
    from diloco_amd import _lib

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=2)
    n = 16 << 20
    x = torch.ones(n, device="cuda")
    sh = torch.empty(n // 2, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    out = {}
    for name in ("all_reduce", "reduce_scatter", "all_gather", "all_reduce_nospin"):
        torch.cuda.synchronize()
        dist.barrier()
        if name != "all_reduce_nospin":
            _lib.call("dl_spin", 300_000_000, s)
        t0 = time.perf_counter()
        if name.startswith("all_reduce"):
            w = dist.all_reduce(x, async_op=True)
        elif name == "reduce_scatter":
            w = dist.reduce_scatter_tensor(sh, x, async_op=True)
        else:
            w = dist.all_gather_into_tensor(x, sh, async_op=True)
        t1 = time.perf_counter()
        done = w.is_completed()
        w.wait()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        out[name] = {"issue_ms": round((t1 - t0) * 1e3, 1), "completed_at_return": done,
                     "wait_ms": round((t2 - t1) * 1e3, 1), "device_drain_ms": round((t3 - t2) * 1e3, 1)}
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get() for _ in ps)
    for p in ps:
        p.join()
    print(json.dumps({"torch": torch.__version__, "ranks": res}), flush=True)
