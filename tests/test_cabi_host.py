"""The C-ABI from a non-Python host: tests/cabi/host_step.c (plain C + the HIP runtime +
libdiloco_hip.so, no Python, no torch) runs four outer steps on a ragged tree -- the one-pass
kernel, the two-kernel pair, the bucketed all-reduce and the sharded reduce-scatter / shard SGD
/ all-gather / scatter step over a one-rank RCCL communicator the library creates -- and
compares them bit for bit with the C oracle. On the GPU it must pass; without a GPU it must fail
loudly (the library reports hipErrorNoDevice), never succeed silently."""
import os
import subprocess

import pytest

from conftest import REPO

BIN = os.path.join(REPO, "tests", "cabi", "host_step")


def _run():
    if not os.path.exists(BIN):
        pytest.fail("tests/cabi/host_step is not built (run __graft_entry__.build())")
    return subprocess.run([BIN], capture_output=True, text=True, timeout=120)


def test_cabi_host_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present (tests/test_cabi_host.py::test_cabi_host_step_on_gpu)")
    p = _run()
    assert p.returncode != 0
    assert "dl_tree_create" in p.stderr and "device" in p.stderr.lower()


@pytest.mark.gpu
def test_cabi_host_step_on_gpu():
    p = _run()
    assert p.returncode == 0, p.stdout + p.stderr
    assert "bit-exact vs oracle" in p.stdout
