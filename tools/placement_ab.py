#!/usr/bin/env python3
"""Interleaved A/B of the drop-in step's placements on T125, one GPU: the default (the
reference's CPU outer model stepped on its HBM twin, write_back="lazy", pinned host arenas),
and the outer model in HBM (placement="device"), built in the order given (round 4 also
compared pageable host arenas and theta / wire / momentum carved from one allocation:
profiles/r04_placement_ab_*.txt); rounds x K back-to-back steps each, the
loop's GPU span / K (events on the step's stream) and the wall time / K. Under rocprofv3
--kernel-trace the kernels' own durations tell GPU idle gaps from slower kernels.

    python tools/placement_ab.py [rounds] [steps] [order: comma list of lazy,device]
"""
import json
import os
import sys
import tempfile
import time
from types import SimpleNamespace

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "diloco-swarm_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from diloco_amd import synth  # noqa: E402
from diloco_amd.comm import TrainingComm  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402
from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,  # noqa: E402
                              sync_inner_model)
from diloco_amd.world import World  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    order = (sys.argv[3] if len(sys.argv) > 3 else "lazy,device").split(",")
    dev = torch.device("cuda", 0)
    # PLACEMENT_AB_BALLAST: "keep" -- a 4 GiB tensor allocated first and kept (the setups'
    # buffers are not the process's first device allocations); "free" -- allocated and freed
    # back to the caching allocator first; unset -- nothing
    ballast = os.environ.get("PLACEMENT_AB_BALLAST")
    if ballast in ("keep", "free"):
        held = torch.ones(1 << 30, device=dev)
        torch.cuda.synchronize()
        if ballast == "free":
            del held
    dist.init_process_group("gloo", init_method="file://" + tempfile.mktemp(prefix="dlpg"),
                            rank=0, world_size=1)
    spec = get_tree("t125")
    shapes = [s for _, s in spec.params()]
    comm = TrainingComm(World.from_default_group(1), (1, 1, spec.n_embd), None)
    setups = {}
    for name in order:
        inner = torch.nn.Module()
        inner.ps = torch.nn.ParameterList([torch.nn.Parameter(t.view(s)) for t, s in zip(
            synth.outer_tree_device(spec, dev), shapes)])
        outer = get_outer_model(inner, "device" if name == "device" else None)
        opt = get_optimizer(outer, SimpleNamespace(type="SGD", lr=0.7, momentum=0.9,
                                                   nesterov=True))
        synth.inner_tree_device([p.data.view(-1) for p in inner.parameters()], 1, 0,
                                out=[p.data.view(-1) for p in inner.parameters()])
        setups[name] = (inner, outer, opt)
    out = {k: {"gpu_ms": [], "wall_ms": []} for k in setups}
    out["order"] = order
    for r in range(rounds):
        for name, (inner, outer, opt) in setups.items():
            for _ in range(3):
                compute_pseudo_gradient(inner, outer)
                comm.sync_gradients(outer)
                opt.step()
                sync_inner_model(outer, inner)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            for _ in range(steps):
                compute_pseudo_gradient(inner, outer)
                comm.sync_gradients(outer)
                opt.step()
                sync_inner_model(outer, inner)
            e1.record()
            torch.cuda.synchronize()
            out[name]["wall_ms"].append(round((time.perf_counter() - t0) / steps * 1e3, 5))
            out[name]["gpu_ms"].append(round(e0.elapsed_time(e1) / steps, 5))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
