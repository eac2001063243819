#!/usr/bin/env python3
"""Does a kernel's HBM rate depend on what the process allocated before? (The int8 step's
dl_unpack_sgd_q8 at T1.3B reads ~4.95 ms as the first thing a process does and ~4.3 ms as
bench.py's fourth leg.) One process, a fixed sequence of legs, each building and freeing its
own arenas; prints each leg's kernel time.

    python tools/alloc_history.py ORDER     ORDER: comma list of q8, f32, head, headdev
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
    dev = torch.device("cuda", 0)
    t13, t125 = get_tree("t1.3b"), get_tree("t125")
    out = []
    for leg in sys.argv[1].split(","):
        if leg == "q8":
            r = bench.run_q8(t13, dev, 1, 0, 10, 3, 64 << 20)
            out.append(("q8 unpack_sgd_q8", r["kernels"]["unpack_sgd_q8"]["avg_ms"],
                        r["kernels"]["delta_q8"]["avg_ms"]))
        elif leg == "f32":
            r = bench.run_engine(t13, dev, 1, 0, 10, 3, torch.float32, 64 << 20, keep_wire=True)
            out.append(("t1.3b delta_pack_sgd", r["roofline"]["avg_ms"], r["roofline"]["frac"]))
        elif leg in ("head", "headdev"):
            r = bench.run_dropin(t125, dev, 1, 0, 50, 3,
                                 placement="device" if leg == "headdev" else None)
            out.append((f"t125 {leg}", r["roofline"]["avg_ms"], r["roofline"]["frac"]))
        print(json.dumps(out[-1]), flush=True)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    print(json.dumps({"order": sys.argv[1], "legs": out}))
