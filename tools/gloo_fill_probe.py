#!/usr/bin/env python3
"""Does gloo traffic on device tensors make another kernel lose one XCD's stores?

The eight-process config #4/#5 tests lost, on one rank, every store of the workgroups one XCD
ran in a completed kernel (the input fill, profiles/r05_stripe_diag.txt; dl_delta_pack,
profiles/r05_gpu_tests_final_a.txt). The stresses without gloo never did: eight processes with
D2H copies (profiles/r05_wave_loss.txt), an oversubscribed runlist, forced queue evictions,
both together, H2D + D2H copies (tools/queue_oversub_probe.py, profiles/r06_queue_probe.txt).
This probe keeps the fill and the verification of tools/queue_oversub_probe.py and puts gloo's
collective on device tensors beside it -- nothing of the outer step:

  P processes, one gloo group; every iteration each process fills a T1.3B-wte-sized fp32
  tensor with dl_fill_synth (alternating two seeds), all_reduces a bucket of --bucket-mb on
  the device through gloo (its staging copies on gloo's own streams, its CPU reduction on its
  threads), synchronizes and compares the fill with its reference; a mismatch is reported by
  the phases (block index mod 8 = XCD) of the wrong 256-element blocks.

    python tools/gloo_fill_probe.py [--procs 8] [--seconds 60] [--bucket-mb 256] [--async-op]
"""
import argparse
import json
import os
import socket
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "diloco-swarm_amd"))
sys.path.insert(0, os.path.join(HERE, "tools"))
sys.path.insert(0, os.path.join(HERE, "tests"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

N = 103_022_592  # T1.3B wte


def _blocks(bad):
    nb = N // 256
    blk = bad[:nb * 256].view(nb, 256).any(1)
    idx = torch.nonzero(blk).flatten().cpu()
    return {"blocks": int(idx.numel()), "elems": int(bad.sum()),
            "phase": torch.bincount(idx % 8, minlength=8).tolist() if idx.numel() else None}


def worker(rank, world, port, args, out):
    from diloco_amd import synth
    from gpu_platform import gpu_state

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    refs = []
    for seed in (11, 12):
        r = torch.empty(N, device="cuda")
        synth.fill_device(r, seed, 0, 0.0, 0.02)
        refs.append(r)
    x = torch.empty(N, device="cuda")
    bucket = torch.ones((args.bucket_mb << 20) // 4, device="cuda")
    torch.cuda.synchronize()
    st0 = gpu_state()
    it, fails, t_end = 0, [], time.time() + args.seconds
    go = torch.zeros(1)
    while True:
        go[0] = float(time.time() < t_end)
        dist.all_reduce(go, op=dist.ReduceOp.MIN)  # every rank stops at the same iteration
        if go[0] == 0:
            break
        k = it & 1
        synth.fill_device(x, (11, 12)[k], 0, 0.0, 0.02)
        w = dist.all_reduce(bucket, async_op=args.async_op)
        if args.async_op:
            w.wait()
        bucket.fill_(1.0)
        torch.cuda.synchronize()
        bad = x != refs[k]
        if bool(bad.any()):
            r = _blocks(bad)
            r["iter"] = it
            fails.append(r)
        it += 1
    rec = {"rank": rank, "iters": it, "n_fails": len(fails), "fails": fails[:6],
           "gpu_start": st0, "gpu_end": gpu_state()}
    with open(os.path.join(out, f"r{rank}.json"), "w") as f:
        json.dump(rec, f)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=60)
    ap.add_argument("--bucket-mb", type=int, default=256)
    ap.add_argument("--async-op", action="store_true")
    args = ap.parse_args()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tempfile.mkdtemp(prefix="gloo_fill_")
    t0 = time.time()
    ctx = mp.start_processes(worker, args=(args.procs, port, args, out), nprocs=args.procs,
                             join=False, start_method="spawn")
    while not ctx.join(timeout=20):
        print(f"... {time.time() - t0:.0f} s", flush=True)
    recs = [json.load(open(os.path.join(out, f"r{r}.json"))) for r in range(args.procs)]
    print(json.dumps({"procs": args.procs, "seconds": args.seconds, "bucket_mb": args.bucket_mb,
                      "async_op": args.async_op, "iters": sum(r["iters"] for r in recs),
                      "n_fails": sum(r["n_fails"] for r in recs), "per_rank": recs,
                      "wall_s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
