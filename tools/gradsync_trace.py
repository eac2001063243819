#!/usr/bin/env python3
"""Per-step DP gradient sync (src/train.py:164,249-251) over a one-rank RCCL
group with torch reallocating every .grad before each step, as the reference's
`inner_optimizer.zero_grad()` (set_to_none=True) does. Prints the rate (GB/s of gradients
averaged) and, when run under `rocprofv3 --hip-trace`, lets the API trace show that the
steady-state steps issue no hipStreamSynchronize / hipDeviceSynchronize (dl_tree_bind is
asynchronous): the steps are bracketed by hipEventRecord markers on a marker stream.

    python tools/gradsync_trace.py [tree] [steps]
"""
import json
import os
import socket
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diloco-swarm_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from diloco_amd import synth  # noqa: E402
from diloco_amd.gradsync import GradSync  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402


def main():
    tree = sys.argv[1] if len(sys.argv) > 1 else "t125"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    spec = get_tree(tree)
    shapes = [s for _, s in spec.params()]
    params = [torch.nn.Parameter(t.view(s))
              for t, s in zip(synth.outer_tree_device(spec, dev), shapes)]

    held = []

    def fresh_grads(k):
        # zero_grad(set_to_none=True), then backward allocating new .grad tensors; the
        # previous step's grads stay referenced for a step (as a training loop's clipping /
        # logging may), so the allocator hands out new addresses and every sync rebinds
        held[:] = [p.grad for p in params if p.grad is not None]
        for p in params:
            p.grad = None
        for i, p in enumerate(params):
            p.grad = torch.empty_like(p)
            synth.fill_device(p.grad.view(-1), synth.noise_seed(9, k), i, 0.0, 1e-3)

    gs = GradSync(params, None, 1)  # the one-rank group: every bucket through RCCL
    fresh_grads(0)
    gs.sync()
    torch.cuda.synchronize()
    done = torch.cuda.Event()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    ptrs = set()
    # steady state: no host synchronisation inside a step except this loop's own
    # hipEventSynchronize at its end (the window's monotonic ns go to the JSON line so an API
    # trace can be cut to it)
    w0 = time.monotonic_ns()
    for k in range(steps):
        fresh_grads(k + 1)
        ptrs.add(params[0].grad.data_ptr())
        ev[k][0].record()
        gs.sync()
        ev[k][1].record()
        done.record()
        done.synchronize()
    w1 = time.monotonic_ns()
    gpu_ms = sum(a.elapsed_time(b) for a, b in ev) / steps
    P = spec.total()
    out = {"tree": tree, "steps": steps, "grad_bytes": 4 * P, "buckets": gs.tree.n_buckets,
           "distinct_grad_addresses": len(ptrs),
           "ms_per_step": round(gpu_ms, 4),
           "value": round(4.0 * P / (gpu_ms * 1e-3) / 1e9, 2), "unit": "GB/s",
           "window_monotonic_ns": [w0, w1],
           "note": "one-rank RCCL group (identity sum); .grad reallocated before every step "
                   "(set_to_none); value = gradient bytes / GPU time of GradSync.sync()"}
    print(json.dumps(out))
    gs.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
