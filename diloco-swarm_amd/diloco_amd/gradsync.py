"""DP average of device gradients: the reference's per-tensor loop in one bucketed pass.

`TrainingComm.sync_gradients(model)` (src/comm.py:117-123) on a model whose gradients live on
the GPU -- plain DP / SWARM without an outer optimizer, called every sync step at
src/train.py:249-251:

    for p in model.parameters():
        all_reduce(p.grad, SUM); p.grad /= num_peers

becomes, per bucket: dl_gather (grads -> packed wire) -> RCCL all_reduce(SUM) ->
dl_unpack_avg (wire / n -> grads), pipelined across buckets (outer.pipelined_buckets).
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch
import torch.distributed as dist

from .kernels import default_kernels
from .outer import _Done, pipelined_buckets
from .plan import DEFAULT_BUCKET_CAP_ELEMS, SLOT_GRAD


class GradSync:
    def __init__(self, params: Sequence[torch.Tensor], group: Optional[dist.ProcessGroup],
                 world_size: int, wire_dtype: torch.dtype = torch.float32,
                 bucket_cap_elems: int = DEFAULT_BUCKET_CAP_ELEMS, kernels=None):
        self.params = list(params)
        self.k = kernels or default_kernels()
        self.device = self.params[0].device
        self.group, self.world_size = group, int(world_size)
        self.numels = [p.numel() for p in self.params]
        self.tree = self.k.tree(self.numels, self.device, bucket_cap_elems)
        self.wire = torch.zeros(self.tree.total, dtype=wire_dtype, device=self.device)
        # own stream, joined back into the caller's (see OuterSync.stream)
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None

    def matches(self, params: Sequence[torch.Tensor]) -> bool:
        return len(params) == len(self.params) and all(
            a is b for a, b in zip(params, self.params))

    def sync(self) -> None:
        if self.stream is None:
            self._sync()
            return
        cur = torch.cuda.current_stream(self.device)
        if cur == self.stream:
            self._sync()
            return
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self._sync()
        cur.wait_stream(self.stream)

    def _sync(self) -> None:
        grads = [p.grad for p in self.params]
        for i, g in enumerate(grads):
            if g.dtype != torch.float32 or not g.is_contiguous():
                raise TypeError(f"grad {i}: {g.dtype}, contiguous={g.is_contiguous()}; "
                                "the DP sync kernels take contiguous fp32 gradients")
        self.k.bind(self.tree, SLOT_GRAD, grads, self.device)

        def view(b):
            lo, hi = self.tree.bucket_ranges[b]
            return self.wire[lo:hi]

        # one replica with no process group: the all-reduce is the identity (the rebinding,
        # gather and /1 still run, so the path is exercised on a one-GPU machine)
        local = self.world_size == 1 and not dist.is_initialized()
        pipelined_buckets(
            self.tree.n_buckets,
            lambda b: self.k.gather(self.tree, b, SLOT_GRAD, self.wire),
            lambda b: _Done() if local else dist.all_reduce(
                view(b), op=dist.ReduceOp.SUM, group=self.group, async_op=True),
            lambda b: self.k.unpack_avg(self.tree, b, self.wire, self.world_size, SLOT_GRAD),
        )

    def close(self) -> None:
        self.tree.close()
