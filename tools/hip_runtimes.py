#!/usr/bin/env python3
"""Which HIP runtime libraries a process that imports torch and loads libdiloco_hip.so has
mapped (one libamdhip64 expected: the library's NEEDED libamdhip64.so.7 resolves to the copy
torch already loaded)."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "diloco-swarm_amd"))

import torch  # noqa: E402

from diloco_amd import _lib  # noqa: E402

if __name__ == "__main__":
    torch.zeros(1, device="cuda")
    _lib.load()
    with open("/proc/self/maps") as f:
        libs = sorted({ln.split()[-1] for ln in f if "amdhip64" in ln or "hsa-runtime" in ln})
    print(libs)
