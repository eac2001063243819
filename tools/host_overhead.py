#!/usr/bin/env python3
"""Host-side cost of one OuterSync.step() enqueue vs its GPU time (diagnostic)."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diloco-swarm_amd"))

import torch  # noqa: E402

from diloco_amd import synth  # noqa: E402
from diloco_amd.outer import OuterSync  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402


def main():
    tree = sys.argv[1] if len(sys.argv) > 1 else "t125"
    dev = torch.device("cuda", 0)
    spec = get_tree(tree)
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, dev), shapes)]
    eng = OuterSync(params, world_size=1)
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    K = 50
    # host enqueue time (GPU queue absorbs it)
    t0 = time.perf_counter()
    for _ in range(K):
        eng.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{tree}: host enqueue {1e3 * (t1 - t0) / K:.4f} ms/step, wall {1e3 * (t2 - t0) / K:.4f} ms/step")
    # kernel-only GPU time: events around 10 back-to-back launches of each kernel
    for name, fn in (("delta_pack", eng.pseudo_gradient), ("unpack_sgd", eng.apply)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        e1.synchronize()
        print(f"  {name}: {e0.elapsed_time(e1) / 10:.4f} ms per launch (10 back-to-back)")
    t0 = time.perf_counter()
    for _ in range(1000):
        eng._rebind(torch.cuda.current_stream().cuda_stream)
    print(f"  rebind check {1e3 * (time.perf_counter() - t0):.3f} us")


if __name__ == "__main__":
    main()
