#!/usr/bin/env python3
"""Is the headline kernel's rate a property of the allocation it runs on? T125 through the
reference's four calls on the device placement, dl_delta_pack_sgd timed by events over 50
back-to-back steps per batch:
  same  -- one outer model, 8 batches (100 ms apart)
  fresh -- 8 outer models one after another, each freed (and the cache emptied) before the next
  shift -- as fresh, with a kept random-size allocation (1-900 MiB) made before each model

    python tools/alloc_variance.py [same|fresh|shift] ...
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "diloco-swarm_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402
from diloco_amd.utils import compute_pseudo_gradient, sync_inner_model  # noqa: E402


def batch(objs, steps=50):
    inner, outer, opt, comm = objs

    def one():
        compute_pseudo_gradient(inner, outer)
        comm.sync_gradients(outer)
        opt.step()
        sync_inner_model(outer, inner)

    for _ in range(3):
        one()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(steps):
        one()
    e[1].record()
    e[1].synchronize()
    return round(e[0].elapsed_time(e[1]) / steps, 5)


def build(dev, spec):
    return bench._dropin_objects(spec, dev, 0, "f32", None, "sharded", "device")


def close(objs):
    objs[1]._diloco_mirror.close()


if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    spec = get_tree("t125")
    rng = np.random.default_rng(5)
    for mode in sys.argv[1:]:
        ms, keep = [], []
        if mode == "same":
            objs = build(dev, spec)
            for _ in range(8):
                ms.append(batch(objs))
                time.sleep(0.1)
            close(objs)
        else:
            for _ in range(8):
                if mode == "shift":
                    keep.append(torch.empty(int(rng.integers(1, 900)) << 18, device=dev))
                objs = build(dev, spec)
                ms.append(batch(objs))
                close(objs)
                del objs
                torch.cuda.synchronize()
                torch.cuda.empty_cache()
        del keep
        torch.cuda.empty_cache()
        a = np.array(ms)
        print(json.dumps({"mode": mode, "ms": ms, "min": a.min(), "max": a.max(),
                          "spread": round(float(a.max() / a.min() - 1), 4)}), flush=True)
