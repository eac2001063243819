"""diloco_amd.staging: which groups stage device tensors through the host (gloo), and that the
answer follows the group object, not its id or the default group's past backend."""
import subprocess
import sys

from conftest import PKG

_SCRIPT = r"""
import os, sys
sys.path.insert(0, sys.argv[1])
import torch
import torch.distributed as dist
from diloco_amd import staging

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[2])
dist.init_process_group("gloo", rank=0, world_size=1)
g = dist.new_group(backend="gloo")
assert staging.host_staged(None) and staging.host_staged(g) and staging.host_staged(g)
assert g in staging._GLOO and None not in staging._GLOO  # the default group is never cached
t = torch.ones(4)
staging.before_collective(g, t)  # host tensors: nothing to wait for
out = staging.collective(dist.all_reduce, g, t, group=g)
assert out is None and t.tolist() == [1.0] * 4
# a fake group object of another backend gets its own answer, not a cached one
staging._GLOO[object()] = True
class Other: pass
assert staging.host_staged(Other()) is False
print("ok")
"""


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_host_staged_follows_the_group_object():
    r = subprocess.run([sys.executable, "-c", _SCRIPT, PKG, str(_free_port())],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().endswith("ok")
