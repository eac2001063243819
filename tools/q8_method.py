#!/usr/bin/env python3
"""The int8 step's dl_unpack_sgd_q8 at T1.3B timed the way bench.py's t1.3b_int8 leg times it
(run_q8: engine steps first, then event-timed launches) -- to set beside tools/q8_spread.py,
whose steady-state launches read ~5.0 ms where the bench leg reads ~4.3 ms.

    python tools/q8_method.py [tree] [steps]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "diloco-swarm_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402

if __name__ == "__main__":
    tree = sys.argv[1] if len(sys.argv) > 1 else "t1.3b"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    r = bench.run_q8(get_tree(tree), torch.device("cuda", 0), 1, 0, steps, 3, 64 << 20)
    print(json.dumps({k: {"avg_ms": v["avg_ms"], "rel_std": v["rel_std"], "frac": v["frac"]}
                      for k, v in r["kernels"].items()}))
