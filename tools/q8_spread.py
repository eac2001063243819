#!/usr/bin/env python3
"""Per-launch durations of the int8-wire kernels over a whole tree (the
spread of dl_unpack_sgd_q8 at T1.3B, 4.82-5.73 ms over the 5 steady-state launches of
tools/kernel_driver.py).

    python tools/q8_spread.py [tree] [steps]

Runs `steps` one-replica int8 outer steps (dl_delta_q8 -> dl_q8_reduce -> dl_unpack_sgd_q8,
each one launch over the whole tree) back to back ("warm"), then `steps` more each after an
Infinity-Cache scrub ("cold"), with HIP events between the kernels, and prints every launch's
duration, so the first launches (first touch of the arenas, the momentum-free first step) can
be told from the steady state. Under `rocprofv3 --kernel-trace --stats` the same launches
appear in the kernel trace.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "diloco-swarm_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from diloco_amd.plan import SLOT_INNER  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402


def main():
    tree = sys.argv[1] if len(sys.argv) > 1 else "t1.3b"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    dev = torch.device("cuda", 0)
    spec = get_tree(tree)
    eng = bench.build(spec, dev, 0, torch.int8, 64 << 20)
    scr = bench.Scrubber(dev)
    out = {"tree": tree, "params": spec.total()}
    for mode in ("warm", "cold"):
        rows = []
        for s in range(steps):
            if mode == "cold":
                scr()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            ev[0].record()
            eng.k.delta_q8(eng.tree, -1, SLOT_INNER, eng.theta, eng.q_slots)
            ev[1].record()
            eng.k.q8_reduce(eng.q_slots, 1, eng.tree.n_chunks, 1, eng.q_slots)
            ev[2].record()
            eng.k.unpack_sgd_q8(eng.tree, -1, eng.q_slots, eng.theta, eng.mom, eng.lr,
                                eng.momentum, eng.nesterov, eng.steps_done == 0, SLOT_INNER)
            ev[3].record()
            eng.steps_done += 1
            torch.cuda.synchronize()
            rows.append([round(ev[i].elapsed_time(ev[i + 1]), 4) for i in range(3)])
        out[mode] = {"delta_q8_ms": [r[0] for r in rows], "q8_reduce_ms": [r[1] for r in rows],
                     "unpack_sgd_q8_ms": [r[2] for r in rows]}
        for k in ("delta_q8_ms", "q8_reduce_ms", "unpack_sgd_q8_ms"):
            t = torch.tensor(out[mode][k][1:], dtype=torch.float64)  # steady state: from step 2
            out[mode][k.replace("_ms", "_mean_ms")] = round(float(t.mean()), 4)
            out[mode][k.replace("_ms", "_rel_std")] = round(float(t.std() / t.mean()), 4)
    scr.close()
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
