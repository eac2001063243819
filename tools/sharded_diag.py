#!/usr/bin/env python3
"""Localise a wrong average in config #4 (1.3B, DP = 8, fp32, sharded exchange behind the
reference's calls; eight gloo processes on the one GPU, no host wait before the collectives).

Per rank and step, on bucket 1 (wpe and the first block's tensors):
  pack   the packed wire right after dl_delta_pack(1) (a clone on the same stream) against
         this rank's exact delta (bit-exact; wrong 4096-element chunks reported by index mod 8)
  sum    this rank's slice of the wire right before dl_shard_sgd(1) -- after the bucket's
         reduce_scatter Work was waited on -- against the sum of every rank's delta
         (normwise 1e-6: gloo's order); wrong 4096-element chunks reported
A wrong pack = the producer lost work; a right pack everywhere and a wrong sum = the exchange
or its ordering against the SGD pass.

    python tools/sharded_diag.py RUNS [MAX_FAILS]
"""
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(HERE, "tests"), HERE, os.path.join(HERE, "diloco-swarm_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

TENSORS = (1, 4)  # wpe (2 Mi) and c_attn.weight (12 Mi), both in bucket 1 of T1.3B
WORLD = 8


def _chunks(bad, base):
    if bad.size == 0:
        return None
    ch = np.unique((base + bad) // 4096)
    return {"n": int(bad.size), "chunks": int(ch.size),
            "phase": np.bincount(ch % 8, minlength=8).tolist(), "first": int(base + bad[0])}


def _worker(rank, world, port, out):
    os.environ["DILOCO_DP_BACKEND"] = "gloo"
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    from conftest import inner_tree_device_verified
    from diloco_amd import synth
    from diloco_amd.comm import TrainingComm
    from diloco_amd.trees import get_tree
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)
    from diloco_amd.world import World
    from test_dropin_gpu import SGD_CFG

    spec = get_tree("t1.3b")
    shapes = [sh for _, sh in spec.params()]
    inner = torch.nn.Module()
    inner.ps = torch.nn.ParameterList(
        [torch.nn.Parameter(x.view(sh)) for x, sh in zip(synth.outer_tree_device(spec, "cuda:0"),
                                                          shapes)])
    outer = get_outer_model(inner, "device")
    opt = get_optimizer(outer, SGD_CFG)
    comm = TrainingComm(World.from_default_group(1), (1, 1, spec.n_embd), None)
    m = outer._diloco_mirror
    k = m.k
    offs, numels = m.offs, m.numels
    blo, bhi = m.tree.bucket_ranges[1]
    snaps = {}
    orig_dp, orig_ss = k.delta_pack, k.shard_sgd

    def delta_pack(tree, b, slot, theta, wire):
        orig_dp(tree, b, slot, theta, wire)
        if b == 1:
            for t in TENSORS:
                snaps[("pack", t)] = wire[offs[t]:offs[t] + numels[t]].clone()

    def shard_sgd(wire, div, theta, mom, *a):
        base = (wire.data_ptr() - m.d_wire.data_ptr()) // 4
        if blo <= base < bhi:
            snaps["sum"] = (base, wire.clone())
        orig_ss(wire, div, theta, mom, *a)

    k.delta_pack, k.shard_sgd = delta_pack, shard_sgd
    ops, ips = list(outer.parameters()), list(inner.parameters())
    rec = {}
    for s in (1, 2):
        snaps.clear()
        theta0 = {t: ops[t].detach().view(-1).cpu().numpy().copy() for t in TENSORS}
        th = [p.detach().view(-1) for p in ops]
        inner_tree_device_verified(th, s, rank, [p.data.view(-1) for p in ips])
        compute_pseudo_gradient(inner, outer)
        comm.sync_gradients(outer)
        opt.step()
        sync_inner_model(outer, inner)
        torch.cuda.synchronize()
        r = {}
        base, sl = snaps["sum"]
        sl = sl.cpu().numpy()
        for t in TENSORS:
            th0 = theta0[t]
            d = []
            for q in range(world):
                u = synth.uniform(synth.noise_seed(s, q), t, th0.size)
                x = (np.float32(0.0) + u * np.float32(synth.NOISE_SCALE)).astype(np.float32)
                d.append((th0 - (x + th0).astype(np.float32)).astype(np.float32))
            got = snaps[("pack", t)].cpu().numpy()
            bad = np.flatnonzero(got != d[rank])
            if bad.size:
                r[f"pack_t{t}"] = _chunks(bad, offs[t])
            # this rank's slice ∩ tensor t
            lo, hi = max(base, offs[t]), min(base + sl.size, offs[t] + numels[t])
            if lo < hi:
                want = np.sum(np.stack(d).astype(np.float64), axis=0)[lo - offs[t]:hi - offs[t]]
                g = sl[lo - base:hi - base].astype(np.float64)
                err = np.abs(g - want)
                tol = 1e-6 * max(np.abs(want).max(), 1e-30)
                badc = np.flatnonzero(err > tol)
                if badc.size:
                    r[f"sum_t{t}"] = _chunks(badc, lo)
                    r[f"sum_t{t}"]["worst_rel"] = float(err.max() / np.abs(want).max())
        if r:
            rec[f"s{s}"] = r
    np.save(os.path.join(out, f"r{rank}.npy"), np.array([repr(rec)]))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    import test_dropin_gpu as tdg

    runs = int(sys.argv[1])
    max_fails = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    fails = 0
    for i in range(runs):
        t0 = time.time()
        out = tempfile.mkdtemp()
        mp.spawn(_worker, args=(WORLD, tdg._free_port(), out), nprocs=WORLD, join=True)
        recs = {r: str(np.load(os.path.join(out, f"r{r}.npy"))[0]) for r in range(WORLD)}
        bad = {r: v for r, v in recs.items() if v != "{}"}
        print(i, f"{time.time() - t0:.0f}s", bad if bad else "clean", flush=True)
        fails += bool(bad)
        if fails >= max_fails:
            break
