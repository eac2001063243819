"""Capture golden fixtures for the outer-step path FROM THE REFERENCE ITSELF.

Runs only in the build container (needs /root/reference); the GPU box and CI read the
committed fixtures. The reference code is imported read-only with four offline stubs
(tests/golden/stubs: pydantic_config, wandb, dotenv, autorootcwd) and
PYTHONDONTWRITEBYTECODE=1 so nothing is written under /root/reference.

Outputs (tests/golden/):
  trees.json         parameters() names/shapes of the micro/tiny/t125/t1.3b trees
                     (src/model.py GPT2 built on the meta device)
  micro_n{1,2,4,8}.npz full fp32 bytes of the reference's outer step on the micro tree:
                     compute_pseudo_gradient (src/utils.py:218) -> TrainingComm.sync_gradients
                     over gloo (src/comm.py:117) -> SGD-Nesterov from get_optimizer
                     (src/utils.py:59, lr 0.7, m 0.9) -> sync_inner_model (src/utils.py:223),
                     2 outer steps, run under torchrun --nproc_per_node n
  tiny_digests.json  per-tensor sha256 / sum / L2 of the same on the tiny (13.8M) tree
  serializer.json    Serializer.serialize/deserialize (src/serializer.py) on small inputs
  plan_tables.json   the build's planner tables (rule restated in oracle/oracle.py)
Inputs come from diloco_amd.synth (counter-based; regenerable on any host or on the GPU).

Usage: python tests/golden/make_golden.py
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
STUBS = os.path.join(HERE, "stubs")
PKG = os.path.join(REPO, "diloco-swarm_amd")

MICRO = dict(n_layer=2, n_head=2, n_embd=32, vocab_size=96, block_size=16, parameter_sharing=True)
TINY = dict(n_layer=4, n_head=4, n_embd=128, parameter_sharing=False)
T125 = dict(n_layer=12, n_head=12, n_embd=768, parameter_sharing=True)
T13B = dict(n_layer=24, n_head=16, n_embd=2048, parameter_sharing=True)
TREE_CFG = {"micro": MICRO, "tiny": TINY, "t125": T125, "t1.3b": T13B}


def _ref_env():
    env = dict(os.environ)
    env["PYTHONDONTWRITEBYTECODE"] = "1"
    env["PYTHONPATH"] = os.pathsep.join([STUBS, REF, PKG])
    env.setdefault("OMP_NUM_THREADS", "1")
    return env


def _import_ref():
    sys.dont_write_bytecode = True
    for p in (PKG, REF, STUBS):
        if p not in sys.path:
            sys.path.insert(0, p)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()


# ---------------------------------------------------------------------------------------------
def capture_trees(out):
    _import_ref()
    import torch
    from src.model import GPT2, GPT2Config

    res = {}
    for name, cfg in TREE_CFG.items():
        with torch.device("meta"):
            m = GPT2(GPT2Config(**cfg))
        params = [(n, list(p.shape)) for n, p in m.named_parameters()]
        res[name] = {"config": cfg, "params": params,
                     "total": int(sum(int(np.prod(s)) for _, s in params))}
    res["torch"] = torch.__version__
    with open(os.path.join(out, "trees.json"), "w") as f:
        json.dump(res, f, indent=1)


def capture_serializer(out):
    _import_ref()
    import torch
    from src.serializer import Serializer

    cases = []
    for shape, meta, dtype in [((2, 3), (0, 1), torch.float32), ((4,), (7, 123), torch.float32),
                               ((2, 2, 3), (3, 16777216), torch.float32),
                               ((3, 5), (1, 2), torch.bfloat16)]:
        g = torch.Generator().manual_seed(7)
        x = torch.randn(*shape, generator=g).to(dtype)
        s = Serializer(shape)
        y = s.serialize(x, meta)
        t, m = s.deserialize(y)
        cases.append({
            "shape": list(shape), "meta": list(meta), "dtype": str(dtype).split(".")[-1],
            "x": x.float().flatten().tolist(), "serializer_shape": list(s.shape),
            "out_shape": list(y.shape), "out_dtype": str(y.dtype).split(".")[-1],
            "meta_plane": y[0].flatten()[:2].tolist(), "payload": y[1].flatten().tolist(),
            "deser_shape": list(t.shape), "deser_meta": list(m),
            "deser_payload_equal": bool(torch.equal(t, y[1])),
        })
    with open(os.path.join(out, "serializer.json"), "w") as f:
        json.dump(cases, f, indent=1)


def capture_plans(out):
    sys.path.insert(0, REPO)
    from oracle.oracle import plan_tables_py

    with open(os.path.join(out, "trees.json")) as f:
        trees = json.load(f)
    caps = {"micro": [0, 4096, 8192], "tiny": [0, 1 << 20, 64 << 20],
            "t125": [0, 16 << 20, 64 << 20], "t1.3b": [0, 64 << 20, 256 << 20]}
    res = {}
    for name, caplist in caps.items():
        numels = [int(np.prod(s)) for _, s in trees[name]["params"]]
        res[name] = {"numels": numels, "plans": []}
        for cap in caplist:
            seg, bnd = plan_tables_py(numels, cap, 64)
            res[name]["plans"].append({"cap": cap, "align": 64, "seg_off": seg, "bkt_bounds": bnd})
    # edge cases
    edge = [[], [0], [1], [3, 0, 5], [64, 64, 1], [100000, 1, 1, 100000]]
    res["edge"] = [{"numels": e, "cap": c, "align": 64,
                    "seg_off": plan_tables_py(e, c, 64)[0], "bkt_bounds": plan_tables_py(e, c, 64)[1]}
                   for e in edge for c in (0, 64, 100)]
    with open(os.path.join(out, "plan_tables.json"), "w") as f:
        json.dump(res, f)


# ---------------------------------------------------------------------------------------------
def worker(tree: str, outdir: str, steps: int, full: bool):
    """Runs under torchrun: the reference's own outer step on this rank."""
    _import_ref()
    import torch
    from diloco_amd import synth
    from diloco_amd.trees import get_tree
    from src.comm import TrainingComm
    from src.config import OptimizerConfig, SwarmConfig
    from src.model import GPT2, GPT2Config
    from src.utils import compute_pseudo_gradient, get_optimizer, get_outer_model, sync_inner_model
    from src.world import World

    torch.set_num_threads(1)
    world = World(SwarmConfig(num_stages=1, sync_every_n_steps=1))
    rank, n = world.rank, world.world_size
    spec = get_tree(tree)
    cfg = TREE_CFG[tree]
    inner = GPT2(GPT2Config(**cfg))
    names = [nm for nm, _ in inner.named_parameters()]
    assert names == [nm for nm, _ in spec.params()], "trees.TreeSpec order differs from reference"
    theta0 = synth.outer_tree(spec.numels(), spec.init_spec())
    with torch.no_grad():
        for p, v in zip(inner.parameters(), theta0):
            p.copy_(torch.from_numpy(v).view(p.shape))
    outer = get_outer_model(inner)
    opt = get_optimizer(outer, OptimizerConfig(type="SGD", lr=0.7, momentum=0.9, nesterov=True))
    comm = TrainingComm(world, (1, 1, cfg["n_embd"]), None)

    flat = lambda ts: np.concatenate([t.detach().reshape(-1).numpy() for t in ts]).astype(np.float32)
    rec = {"theta0": np.concatenate(theta0)}
    digests = {}
    for s in range(1, steps + 1):
        prev = [p.detach().numpy().reshape(-1).copy() for p in outer.parameters()]
        vals = synth.inner_tree(prev, s, rank)
        with torch.no_grad():
            for p, v in zip(inner.parameters(), vals):
                p.copy_(torch.from_numpy(v).view(p.shape))
        if s == 1:
            rec["inner_s1"] = np.concatenate(vals)
        compute_pseudo_gradient(inner, outer)
        rec[f"delta_s{s}"] = flat(p.grad for p in outer.parameters())
        comm.sync_gradients(outer)
        rec[f"avg_s{s}"] = flat(p.grad for p in outer.parameters())
        opt.step()
        rec[f"theta_s{s}"] = flat(outer.parameters())
        rec[f"buf_s{s}"] = flat(opt.state[p]["momentum_buffer"] for p in outer.parameters())
        sync_inner_model(outer, inner)
        post = flat(inner.parameters())
        assert np.array_equal(post, rec[f"theta_s{s}"]), "sync_inner_model must copy exactly"
        if not full:
            for key in (f"delta_s{s}", f"avg_s{s}", f"theta_s{s}", f"buf_s{s}"):
                digests[key] = _tensor_digests(rec[key], spec.numels())
    if full:
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), **rec)
    else:
        del rec  # the tiny tree keeps digests only
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
            json.dump(digests, f)
    import torch.distributed as dist

    dist.barrier()


def _tensor_digests(flat: np.ndarray, numels):
    out, o = [], 0
    for n in numels:
        a = flat[o:o + n]
        out.append({"sha256": sha(a), "sum": float(a.astype(np.float64).sum()),
                    "l2": float(np.sqrt((a.astype(np.float64) ** 2).sum())),
                    "maxabs": float(np.abs(a).max()) if n else 0.0})
        o += n
    return out


def run_outer(tree: str, n: int, steps: int, full: bool, port: int):
    with tempfile.TemporaryDirectory() as td:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
               os.path.abspath(__file__), "--worker", "--tree", tree, "--out", td,
               "--steps", str(steps)] + (["--full"] if full else [])
        subprocess.run(cmd, check=True, env=_ref_env(), cwd="/tmp")
        recs, digs = None, None
        if full:
            recs = [dict(np.load(os.path.join(td, f"rank{r}.npz"))) for r in range(n)]
        else:
            digs = [json.load(open(os.path.join(td, f"rank{r}.json"))) for r in range(n)]
        return recs, digs


def capture_micro(n: int, port: int):
    """micro_n<n>.npz: the reference's 2 outer steps with n DP peers (gloo), full bytes."""
    recs, _ = run_outer("micro", n, 2, True, port)
    out = {"theta0": recs[0]["theta0"], "inner_s1_r0": recs[0]["inner_s1"]}
    for s in (1, 2):
        out[f"delta_s{s}_r0"] = recs[0][f"delta_s{s}"]
        out[f"delta_s{s}_rlast"] = recs[-1][f"delta_s{s}"]
        out[f"avg_s{s}"] = recs[0][f"avg_s{s}"]
        out[f"theta_s{s}"] = recs[0][f"theta_s{s}"]
        out[f"buf_s{s}"] = recs[0][f"buf_s{s}"]
        for r in range(1, n):  # every rank holds the same averaged state
            assert np.array_equal(recs[r][f"avg_s{s}"], out[f"avg_s{s}"])
            assert np.array_equal(recs[r][f"theta_s{s}"], out[f"theta_s{s}"])
    np.savez_compressed(os.path.join(HERE, f"micro_n{n}.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--tree", default="micro")
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--micro-n", type=int, nargs="*", default=None,
                    help="only (re)capture micro_n<N>.npz for these peer counts")
    a = ap.parse_args()
    if a.worker:
        worker(a.tree, a.out, a.steps, a.full)
        return
    if not os.path.isdir(REF):
        raise SystemExit("the reference is not mounted; fixtures are committed under tests/golden")
    if a.micro_n:
        port = 29711
        for n in a.micro_n:
            capture_micro(n, port)
            port += 11
        return
    # the reference is imported only in child processes (stubs on PYTHONPATH, no bytecode)
    subprocess.run([sys.executable, "-c",
                    f"import sys; sys.path.insert(0, {HERE!r}); import make_golden as m; "
                    f"m.capture_trees({HERE!r}); m.capture_serializer({HERE!r})"],
                   check=True, env=_ref_env(), cwd="/tmp")
    capture_plans(HERE)
    port = 29611
    for n in (1, 2, 4, 8):
        capture_micro(n, port)
        port += 7
    tiny = {}
    for n in (1, 2, 4):
        recs, digs = run_outer("tiny", n, 2, False, port)
        port += 7
        tiny[str(n)] = {"rank0": digs[0], "rank_last_delta_s1": digs[-1]["delta_s1"]}
    import torch

    tiny["torch"] = torch.__version__
    with open(os.path.join(HERE, "tiny_digests.json"), "w") as f:
        json.dump(tiny, f)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
