#!/usr/bin/env python3
"""Config #5 through the reference's calls (eight gloo processes on one GPU,
tests/test_dropin_gpu.py::_bf16_dropin_codec_check) K times per variant: every run's worst
error / bound and mismatches -- to localise an intermittent missing contribution.
Variants: base (the product: no host wait); sync_pack (the current stream synchronized after each bucket's pack, before
its all_reduce); sync_wait (synchronized after each bucket's wait, before its SGD pass).

    python tools/bf16_n8_repeat.py K variant [variant ...]
"""
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(HERE, "tests"), HERE, os.path.join(HERE, "diloco-swarm_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _patch(variant):
    from diloco_amd import mirror

    if variant == "base":
        return
    elif variant == "sync_pack":
        orig = mirror.DeviceOuterMirror._launch_reductions

        def launch(self, pack, view, group):
            def pack_sync(b):
                pack(b)
                torch.cuda.current_stream().synchronize()
            return orig(self, pack_sync if pack is not None else None, view, group)
        mirror.DeviceOuterMirror._launch_reductions = launch
    elif variant == "sync_wait":
        import torch.distributed.distributed_c10d as c10d  # noqa: F401

        orig_ar = dist.all_reduce

        class W:
            def __init__(self, w):
                self.w = w

            def wait(self):
                self.w.wait()
                torch.cuda.synchronize()

        def ar(*a, **k):
            w = orig_ar(*a, **k)
            return W(w) if k.get("async_op") else w
        mirror.dist.all_reduce = ar


def _worker(rank, world, port, variant, out):
    os.environ["DILOCO_DP_BACKEND"] = "gloo"
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    _patch(variant)
    import test_dropin_gpu as t

    rec = t._bf16_dropin_codec_check(rank, world)
    np.savez(os.path.join(out, f"r{rank}.npz"), **rec)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    import test_dropin_gpu as t

    import time

    k = int(sys.argv[1])
    for i in range(k):  # variants interleaved, so a drift of the box hits each alike
        for variant in sys.argv[2:]:
            t0 = time.time()
            out = tempfile.mkdtemp()
            mp.spawn(_worker, args=(8, t._free_port(), variant, out), nprocs=8, join=True)
            recs = [dict(np.load(os.path.join(out, f"r{r}.npz"))) for r in range(8)]
            bad = [str(b)[:400] for r in recs[:1] for b in r["bad"] if str(b) != "none"]
            print(variant, i, round(float(recs[0]["worst"]), 4), len(bad), bad[:1],
                  f"{time.time() - t0:.0f}s", flush=True)
