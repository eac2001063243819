#!/usr/bin/env python3
"""Launch each hot-path kernel a few times on a tree (for rocprofv3 counter passes)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diloco-swarm_amd"))

import torch  # noqa: E402

from diloco_amd import synth  # noqa: E402
from diloco_amd.outer import OuterSync  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402


def main():
    tree = sys.argv[1] if len(sys.argv) > 1 else "t125"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda", 0)
    spec = get_tree(tree)
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, dev), shapes)]
    eng = OuterSync(params, world_size=1)
    synth.inner_tree_device([p.view(-1) for p in params], 1, 0, out=[p.view(-1) for p in params])
    eng.step()
    for _ in range(reps):
        eng.pseudo_gradient()
    for _ in range(reps):
        eng.apply()
    fused = OuterSync(params, world_size=1, fuse_single=True)
    fused.step()
    for _ in range(reps):
        fused.step()
    kept = OuterSync(params, world_size=1, fuse_single=True, keep_wire=True)
    kept.step()
    for _ in range(reps):
        kept.step()
    # one bucket each, so every launch covers the whole tree: the int8 wire kernels and the
    # sharded step's dl_shard_sgd (one replica: the shard is the whole bucket)
    q8 = OuterSync(params, world_size=1, wire_dtype=torch.int8, bucket_cap_elems=0)
    sh = OuterSync(params, world_size=1, shard=True, bucket_cap_elems=0)
    xg = OuterSync(params, world_size=1, exchange="xgmi")  # n = 1: the fused kernel, local
    a2 = OuterSync(params, world_size=1, exchange="a2a", bucket_cap_elems=0)
    for e in (q8, sh, xg, a2):
        for _ in range(reps + 1):
            e.step()
    # dl_shard_reduce_sgd as an 8-peer rank would run it: 8 slices of an eighth of the tree
    L = (sum(p.numel() for p in params) // 8) // 64 * 64
    slices = torch.randn(8 * L, device=dev) * 1e-3
    th8, m8 = torch.randn(L, device=dev), torch.zeros(L, device=dev)
    for i in range(reps + 1):
        eng.k.shard_reduce_sgd(slices, 8, th8, m8, 0.7, 0.9, True, i == 0)
    del slices, th8, m8
    # the per-step DP gradient sync at one replica (dl_gather -> identity -> dl_unpack_avg),
    # one bucket so each launch covers the tree
    from diloco_amd.gradsync import GradSync

    grads = [torch.nn.Parameter(torch.zeros_like(p)) for p in params]
    for g in grads:
        g.grad = torch.randn_like(g)
    gs = GradSync(grads, None, 1, bucket_cap_elems=0)
    for _ in range(reps + 1):
        gs.sync()
    gs.close()
    del grads
    # the pipeline Serializer (src/serializer.py:11-15) framing the reference's message, a
    # (32, 1024, 768) activation, fp32 and bf16 payloads
    from diloco_amd.serializer import Serializer

    ser = Serializer((32, 1024, 768))
    act = torch.randn(32, 1024, 768, device=dev)
    for x in (act, act.bfloat16()):
        for _ in range(reps + 1):
            ser.serialize(x, (3, 7))
    # last: exchange="xgmi_inner" moves `params` into its own arena
    xi = OuterSync(params, world_size=1, exchange="xgmi_inner")
    for e in (xi,):
        for _ in range(reps + 1):
            e.step()
    torch.cuda.synchronize()
    print(f"kernel_driver: {tree} x{reps} done")


if __name__ == "__main__":
    main()
