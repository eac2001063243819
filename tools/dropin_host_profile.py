#!/usr/bin/env python3
"""Host cost of the reference's four drop-in calls (T125, N = 1) for each placement: the
default (the reference's CPU outer model stepped on its HBM twin, write_back="lazy") and the
outer model in HBM (placement="device"): per-call wall time with the device idle at each
call's start (a synchronize between steps, as src/train.py:243-244 does before the outer
step), then a cProfile of the default's calls.
Diagnostic; usage: python tools/dropin_host_profile.py [steps]"""
import cProfile
import os
import pstats
import sys
import tempfile
import time
from types import SimpleNamespace

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diloco-swarm_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from diloco_amd import synth  # noqa: E402
from diloco_amd.comm import TrainingComm  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402
from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,  # noqa: E402
                              sync_inner_model)
from diloco_amd.world import World  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", init_method="file://" + tempfile.mktemp(prefix="dlpg"),
                            rank=0, world_size=1)
    spec = get_tree("t125")
    shapes = [s for _, s in spec.params()]
    inner = torch.nn.Module()
    inner.ps = torch.nn.ParameterList(
        [torch.nn.Parameter(t.view(s)) for t, s in zip(synth.outer_tree_device(spec, dev), shapes)])
    comm = TrainingComm(World.from_default_group(1), (1, 1, spec.n_embd), None)
    for placement in ("device", None):
        outer = get_outer_model(inner, placement)
        opt = get_optimizer(outer, SimpleNamespace(type="SGD", lr=0.7, momentum=0.9,
                                                   nesterov=True))
        calls = [("compute_pseudo_gradient", lambda: compute_pseudo_gradient(inner, outer)),
                 ("sync_gradients", lambda: comm.sync_gradients(outer)),
                 ("outer_step", opt.step),
                 ("sync_inner_model", lambda: sync_inner_model(outer, inner))]
        acc = {k: [] for k, _ in calls}
        for i in range(steps + 5):
            torch.cuda.synchronize()
            for k, fn in calls:
                t0 = time.perf_counter()
                fn()
                acc[k].append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        print(f"placement {placement or 'host (default, write_back lazy)'}")
        for k, v in acc.items():
            v = sorted(v[5:])
            print(f"  {k:24s} median {1e6 * v[len(v) // 2]:7.1f} us  min {1e6 * v[0]:7.1f} us")
    pr = cProfile.Profile()
    for _ in range(steps):
        torch.cuda.synchronize()
        pr.enable()
        for _, fn in calls:
            fn()
        pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
