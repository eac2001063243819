"""The reference's CPU outer step restated per tensor with torch (TEST INFRASTRUCTURE).

Only bench.py's cpu_baseline leg and tests/ use this. It is the sequence of
src/train.py:261-269 with the reference's own per-parameter loops:
    compute_pseudo_gradient  src/utils.py:218-221  po.grad = (po.data - pi.data).clone()
    sync_gradients           src/comm.py:117-123   per-tensor all_reduce(SUM) + /= n (n > 1)
    outer_optimizer.step()   torch.optim.SGD(lr, momentum, nesterov) (src/utils.py:62-63)
    sync_inner_model         src/utils.py:223-226  pi.data.copy_(po)
"""
from __future__ import annotations

import time
from typing import List, Optional

import torch
import torch.distributed as dist


class TorchOuterStep:
    def __init__(self, inner: List[torch.Tensor], lr=0.7, momentum=0.9, nesterov=True,
                 group: Optional[dist.ProcessGroup] = None):
        self.inner = inner
        self.outer = [torch.nn.Parameter(t.detach().clone()) for t in inner]  # get_outer_model
        self.opt = torch.optim.SGD(self.outer, lr=lr, momentum=momentum, nesterov=nesterov)
        self.group = group
        self.n = dist.get_world_size(group) if group is not None else 1

    def step(self):
        for po, pi in zip(self.outer, self.inner):
            po.grad = (po.data - pi.data).clone()
        if self.n > 1:
            for po in self.outer:
                dist.all_reduce(po.grad, op=dist.ReduceOp.SUM, group=self.group)
                po.grad /= self.n
        self.opt.step()
        for po, pi in zip(self.outer, self.inner):
            pi.data.copy_(po.detach())


def time_steps(numels, steps=2, threads=1, seed=0, budget_s=None):
    """Seconds per outer step of the per-tensor torch CPU path on a tree of `numels`.

    With budget_s, keeps stepping (at least `steps` times) until budget_s seconds elapsed.
    Returns (seconds_per_step, steps_timed)."""
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(seed)
    inner = [torch.empty(n).uniform_(-0.03, 0.03, generator=g) for n in numels]
    st = TorchOuterStep(inner)
    for t in inner:
        t.add_(torch.empty_like(t).uniform_(-1e-3, 1e-3, generator=g))
    st.step()  # first step allocates the momentum buffers (not timed)
    t0 = time.perf_counter()
    done = 0
    while done < steps or (budget_s is not None and time.perf_counter() - t0 < budget_s):
        st.step()
        done += 1
    return (time.perf_counter() - t0) / done, done
