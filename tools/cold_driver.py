#!/usr/bin/env python3
"""Launch the one-replica hot-path kernels cold, for rocprofv3 counter passes: each launch
follows a 512 MiB default-policy dl_copy that evicts the Infinity Cache (bench.Scrubber), as
the H inner steps of training do. Kernels: dl_delta_pack, dl_unpack_sgd (whole-range),
dl_delta_sgd, dl_delta_pack_sgd, dl_delta_pack with two chunks per workgroup (DL_TUNE_PAIRS,
k_walk_pairs in the trace), and dl_copy of T125's size with NT policy (the copy ceiling).

    python tools/cold_driver.py [tree] [reps]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diloco-swarm_amd"))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

from bench import Scrubber  # noqa: E402
from diloco_amd import _lib, synth  # noqa: E402
from diloco_amd.outer import OuterSync  # noqa: E402
from diloco_amd.trees import get_tree  # noqa: E402


def main():
    tree = sys.argv[1] if len(sys.argv) > 1 else "t125"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda", 0)
    spec = get_tree(tree)
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, dev), shapes)]
    synth.inner_tree_device([p.view(-1) for p in params], 1, 0, out=[p.view(-1) for p in params])
    scrub = Scrubber(dev)
    two = OuterSync(params, world_size=1, fuse_single=False, tile_chunks=0)
    one = OuterSync(params, world_size=1, fuse_single=True)
    kept = OuterSync(params, world_size=1, fuse_single=True, keep_wire=True)
    pairs = None
    if _lib.load().dl_tuning_build():  # DL_TUNE_PAIRS exists in the tuning build only
        pairs = OuterSync(params, world_size=1, fuse_single=False, tile_chunks=0)
        # AUTO's store policy for a whole-tree dl_delta_pack (NT above 2^28 elements), paired
        big = pairs.tree.total >= (1 << 28)
        pairs.tree.tune(0, _lib.TUNE_NT_LOADS | _lib.TUNE_PAIRS
                        | (_lib.TUNE_NT_STORES if big else 0))
    for e in (two, one, kept) + ((pairs,) if pairs else ()):
        e.step()  # steady-state SGD mode from here on
    n = spec.total() // 4 * 4
    a = torch.ones(n, device=dev)
    b = torch.empty(n, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream

    def copy():
        _lib.call("dl_copy", a.data_ptr(), b.data_ptr(), 4 * n, _lib.TUNE_NT_LOADS, st)

    for _ in range(reps):
        for fn in (two.pseudo_gradient, two.apply, one.step, kept.step,
                   pairs.pseudo_gradient if pairs else None, copy):
            if fn is None:
                continue
            scrub()
            fn()
    torch.cuda.synchronize()
    print(f"cold_driver: {tree} x{reps} done")


if __name__ == "__main__":
    main()
