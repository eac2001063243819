#!/usr/bin/env python3
"""Per-allocation counters of the headline kernel: K fresh T125 outer models on the device
placement one after another (each freed before the next), 20 timed steps each; prints every
instance's event-timed ms per step. Run under `rocprofv3 --pmc ...` to pair each instance's
dispatches (3 warm-up + 20, in order) with its counters (tools/alloc_variance.py: the rate is
a property of the allocation -- 0.5-1.8 % spread on one, 6-7 % across fresh ones).

    python tools/alloc_pmc.py [K]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tools"))
sys.path.insert(0, os.path.join(HERE, "diloco-swarm_amd"))

import torch  # noqa: E402

from alloc_variance import batch, build, close  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402

if __name__ == "__main__":
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    spec = get_tree("t125")
    ms = []
    for _ in range(k):
        objs = build(dev, spec)
        ms.append(batch(objs, steps=20))
        close(objs)
        del objs
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    print(json.dumps({"per_instance_ms": ms, "dispatches_per_instance": 23}))
