#!/usr/bin/env python3
"""dl_shard_reduce_sgd timed cold (Infinity Cache scrubbed before each launch) for n = 1, 2, 4, 8
slices that together cover a tree's worth of elements (an n-peer rank's shard), fp32, steady-
state SGD; median ms and GB/s of algorithmic bytes. Run once per library build
(DILOCO_HIP_LIB) for interleaved A/Bs (tools/gpu_slices_ab.sh).
    python tools/slices_ab.py [tree] [rounds]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diloco-swarm_amd"))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

from diloco_amd.kernels import default_kernels  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402


def main():
    from bench import Scrubber

    tree = sys.argv[1] if len(sys.argv) > 1 else "t125"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 11
    dev = torch.device("cuda", 0)
    P = get_tree(tree).total()
    k = default_kernels()
    scrub = Scrubber(dev)
    cases = {}
    for n in (1, 2, 4, 8):
        L = P // n // 64 * 64
        cases[n] = (torch.randn(n * L, device=dev) * 1e-3, torch.randn(L, device=dev),
                    torch.zeros(L, device=dev), L)
        k.shard_reduce_sgd(cases[n][0], n, cases[n][1], cases[n][2], 0.7, 0.9, True, True)
    ms = {n: [] for n in cases}
    for _ in range(rounds):
        for n, (sl, th, m, L) in cases.items():
            scrub()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            k.shard_reduce_sgd(sl, n, th, m, 0.7, 0.9, True, False)
            e1.record()
            e1.synchronize()
            ms[n].append(e0.elapsed_time(e1))
    for n, v in ms.items():
        v.sort()
        L = cases[n][3]
        med = v[len(v) // 2]
        print(f"{tree} n={n} med {med:.4f} ms {(4 * n + 16) * L / med / 1e6:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
