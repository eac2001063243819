#!/usr/bin/env python3
"""Is a kernel's write visible to the next kernel on the same stream? Per iteration: the
library's dl_fill_synth writes R (plain stores), then dl_copy reads R into Y right behind it
on the same stream (variant "direct"), or after a dl_sys_fence (every XCD's L2 written back
and invalidated; variant "fenced"); "_nt": the copies with non-temporal loads and stores. Y is then checked against a reference fill R2 made long
before, behind a host synchronize and a sys_fence. Run several copies at once (torchrun
--nproc-per-node P, no process group) to load the GPU as the multi-process tests do.

    python tools/xcd_stale.py [iters] [mib]
"""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "diloco-swarm_amd"))

import torch  # noqa: E402

from diloco_amd import _lib, synth  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    mib = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(0)
    _lib.load()
    n = (mib << 20) // 4
    R, Y, R2 = (torch.empty(n, device="cuda") for _ in range(3))
    s = torch.cuda.current_stream().cuda_stream
    out = {}
    for variant in ("direct", "fenced", "direct_nt", "fenced_nt"):
        fl = 1 if variant.endswith("_nt") else 0  # dl_copy: non-temporal loads and stores
        bad_iters, bad_elems = 0, 0
        for it in range(iters):
            seed = 1000 * rank + it
            synth.fill_device(R2, seed, 7, 0.0, 1.0)
            torch.cuda.synchronize()
            _lib.call("dl_sys_fence", s)
            synth.fill_device(R, 99, 7, 0.0, 1.0)  # stale content first
            torch.cuda.synchronize()
            _lib.call("dl_copy", R.data_ptr(), Y.data_ptr(), 4 * n, fl, s)  # R's lines cached
            synth.fill_device(R, seed, 7, 0.0, 1.0)
            if variant.startswith("fenced"):
                _lib.call("dl_sys_fence", s)
            _lib.call("dl_copy", R.data_ptr(), Y.data_ptr(), 4 * n, fl, s)
            torch.cuda.synchronize()
            _lib.call("dl_sys_fence", s)
            torch.cuda.synchronize()
            k = int((Y != R2).sum())
            bad_elems += k
            bad_iters += int(k > 0)
        out.setdefault(variant, []).append((bad_iters, bad_elems))
    print({"rank": rank, "iters": iters, "mib": mib, "stale": out}, flush=True)


if __name__ == "__main__":
    main()
