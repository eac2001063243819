#!/usr/bin/env python3
"""Per-call time of the outer step behind the reference's calls at N ranks (torchrun; with
DILOCO_BENCH_BACKEND=gloo every rank may share one GPU): the four calls of src/train.py:263-269
each followed by a device synchronize and a barrier-free host clock, on bench.py's objects, for
the default placement and placement="device". Rank 0 prints one JSON line (medians, ms).

    DILOCO_BENCH_BACKEND=gloo torchrun --nproc-per-node N tools/step_breakdown.py [TREE] [STEPS]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402
from diloco_amd.utils import compute_pseudo_gradient, sync_inner_model  # noqa: E402


def main():
    tree = sys.argv[1] if len(sys.argv) > 1 else "t125"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    ws, rank, dev = bench.setup_dist(ws)
    spec = get_tree(tree)
    out = {"n": ws, "tree": tree}
    for placement in (None, "device"):
        inner, outer, opt, comm = bench._dropin_objects(spec, dev, rank, "f32", None, "sharded",
                                                        placement)
        calls = [("pseudo_gradient", lambda: compute_pseudo_gradient(inner, outer)),
                 ("sync_gradients", lambda: comm.sync_gradients(outer)),
                 ("opt_step", lambda: opt.step()),
                 ("sync_inner", lambda: sync_inner_model(outer, inner))]
        rec = {k: [] for k, _ in calls}
        rec["whole_unsynced"] = []
        for s in range(steps + 1):
            for k, f in calls:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                f()
                torch.cuda.synchronize()
                if s:
                    rec[k].append(time.perf_counter() - t0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _, f in calls:
                f()
            torch.cuda.synchronize()
            if s:
                rec["whole_unsynced"].append(time.perf_counter() - t0)
        out[placement or "default"] = {k: round(float(np.median(v)) * 1e3, 2) for k, v in rec.items()}
        mm = outer._diloco_mirror
        mm.close()
        del inner, outer, opt, mm
        torch.cuda.empty_cache()
    if rank == 0:
        print(json.dumps(out), flush=True)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
