#!/usr/bin/env python3
"""Does a gloo all_reduce of a CUDA tensor (async, several in flight) ever read the buffer
before the kernel that wrote it on the current stream finished? World W ranks on one GPU;
per iteration every rank writes each bucket with a value of its own -- by a torch kernel
(fill_) or by the library's dl_copy (plain, or "_nt": non-temporal loads and stores) -- then issues the bucket's async SUM all_reduce right
away; after all waits every element must be the sum. Counts wrong elements per variant.

    python tools/gloo_race.py   (under torchrun: --nproc-per-node W)
"""
import os
import sys
from datetime import timedelta

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "diloco-swarm_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from diloco_amd import _lib  # noqa: E402


def main():
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", timeout=timedelta(minutes=5))
    _lib.load()
    nb, m = int(os.environ.get("RACE_NB", 6)), int(os.environ.get("RACE_M", 16 << 20))
    iters = int(os.environ.get("RACE_ITERS", 6))
    variants = os.environ.get("RACE_VARIANTS", "torch_fill_bf16,dl_copy_bf16,torch_fill_f32,"
                              "dl_copy_f32,dl_copy_bf16_sync").split(",")
    res = {}
    for variant in variants:
        dt = torch.bfloat16 if "bf16" in variant else torch.float32
        buf = torch.zeros(nb * m, dtype=dt, device="cuda")
        src = torch.empty_like(buf)
        slow = "slow" in variant
        if slow:  # a long kernel ahead of each write: a wide window for a copy that jumps it
            big_a = torch.zeros(512 << 20, dtype=torch.uint8, device="cuda")
            big_b = torch.empty_like(big_a)
        bad = 0
        for it in range(iters):
            val = float((rank + 1) * (it + 1))
            src.fill_(val)
            torch.cuda.synchronize()
            works = []
            for b in range(nb):
                view = buf[b * m:(b + 1) * m]
                if slow:
                    for _ in range(4):
                        _lib.call("dl_copy", big_a.data_ptr(), big_b.data_ptr(), big_a.numel(),
                                  0, torch.cuda.current_stream().cuda_stream)
                if variant.startswith("torch_fill"):
                    view.fill_(val)
                else:
                    _lib.call("dl_copy", src[b * m:].data_ptr(), view.data_ptr(),
                              m * buf.element_size(), 1 if "_nt" in variant else 0,
                              torch.cuda.current_stream().cuda_stream)
                if variant.endswith("_sync"):
                    torch.cuda.current_stream().synchronize()
                works.append(dist.all_reduce(view, async_op=True))
            for w in works:
                w.wait()
            want = float(sum((r + 1) * (it + 1) for r in range(ws)))
            bad += int((buf.float() != want).sum())
        res[variant] = bad
        del buf, src
        if slow:
            del big_a, big_b
        torch.cuda.empty_cache()
    if rank == 0:
        print({"world": ws, "bad_elements": res}, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
