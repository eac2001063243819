"""Collectives over gloo on device tensors: finish the producing kernels first.

gloo stages a CUDA tensor through pinned host memory: the work copies it to the host on a
stream of its own that waits for an event recorded on the caller's stream, runs the exchange
on the host, and copies the result back. With eight processes on one GPU exchanging
1.3B-parameter bf16 buckets, that copy occasionally saw a bucket before the pack kernel had
written it -- the sum missed one rank's contribution, on every replica alike
(tests/test_dropin_gpu.py::test_t13b_eight_peers_dropin_device_bf16_wire_within_codec_bound
failed 4 times in 19 runs; tools/bf16_n8_repeat.py). Synthetic producers
(torch fills, the library's copies, a long kernel ahead of them) never reproduced it
(tools/gloo_race.py). So before a gloo collective on device tensors the caller's stream is
synchronized: the data is on the device when gloo copies it, at the cost of one host wait per
collective on a transport that stages through the host anyway. RCCL collectives run on a
stream ordered behind the producers and are untouched: gloo on device tensors is the
test / one-GPU-rehearsal transport (DILOCO_DP_BACKEND=gloo)."""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.distributed as dist

# keyed by the group object itself (held here, so a destroyed group's id cannot be reused by a
# new group of another backend and inherit its answer); None = the default group, which
# destroy_process_group + init_process_group can replace, so it is never cached
_GLOO: Dict[dist.ProcessGroup, bool] = {}


def host_staged(group: Optional[dist.ProcessGroup]) -> bool:
    """The group's collectives stage device tensors through host memory (gloo)."""
    v = None if group is None else _GLOO.get(group)
    if v is None:
        try:
            v = dist.get_backend(group) == "gloo"
        except (RuntimeError, ValueError):
            v = False
        if group is not None:
            _GLOO[group] = v
    return v


def before_collective(group: Optional[dist.ProcessGroup], t: torch.Tensor) -> None:
    """Call right before issuing a collective that reads `t`: over gloo, the kernels queued
    on the caller's stream (the producers of `t`) finish first."""
    if t.is_cuda and host_staged(group):
        torch.cuda.current_stream(t.device).synchronize()


def collective(fn, pg: Optional[dist.ProcessGroup], t: torch.Tensor, /, *args, **kw):
    """fn(t, *args, **kw) -- a collective over pg that reads t -- after before_collective."""
    before_collective(pg, t)
    return fn(t, *args, **kw)
