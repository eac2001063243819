"""DP average of device gradients: the reference's per-tensor loop in one bucketed pass.

`TrainingComm.sync_gradients(model)` (src/comm.py:117-123) on a model whose gradients live on
the GPU -- plain DP / SWARM without an outer optimizer, called every sync step at
src/train.py:249-251:

    for p in model.parameters():
        all_reduce(p.grad, SUM); p.grad /= num_peers

becomes, per bucket: dl_gather (grads -> packed wire) -> RCCL all_reduce(SUM) ->
dl_unpack_avg (wire / n -> grads), pipelined across buckets (outer.pipelined_buckets).

exchange="a2a" (as OuterSync's): per bucket dl_gather -> RCCL all_to_all of the wire slices ->
dl_shard_reduce_avg (Σ in rank order in fp32, / n, into this peer's shard) -> RCCL all_gather
of the averaged shards -> dl_unpack_avg (a copy): the same bus bytes as the all-reduce, an
average that does not depend on RCCL's algorithm and is bit-exact against oracle/or_sum_avg at
every n.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch
import torch.distributed as dist

from .kernels import default_kernels
from . import _lib
from .outer import _Done, pipelined_buckets
from .plan import DEFAULT_BUCKET_CAP_ELEMS, SLOT_GRAD


class GradSync:
    def __init__(self, params: Sequence[torch.Tensor], group: Optional[dist.ProcessGroup],
                 world_size: int, wire_dtype: torch.dtype = torch.float32,
                 bucket_cap_elems: int = DEFAULT_BUCKET_CAP_ELEMS, kernels=None,
                 exchange: str = "rccl"):
        self.params = list(params)
        self.k = kernels or default_kernels()
        self.device = self.params[0].device
        self.group, self.world_size = group, int(world_size)
        if exchange not in ("rccl", "a2a"):
            raise ValueError(f"exchange {exchange!r}: 'rccl' or 'a2a'")
        self.a2a = exchange == "a2a"
        if dist.is_initialized() and self.world_size > 1:
            gs = dist.get_world_size(group)
            if gs != self.world_size:  # the collectives would reduce over the wrong ranks
                raise ValueError(f"GradSync(world_size={self.world_size}) on a process group "
                                 f"of {gs} ranks")
        # one replica: the all-reduce is the identity -- with no process group, or a group of
        # other ranks this replica does not average with (OuterSync._local's rule); a one-rank
        # group carries it (the single-rank RCCL transport test)
        self.local = self.world_size == 1 and (
            not dist.is_initialized() or dist.get_world_size(group) != 1)
        if self.a2a and wire_dtype != torch.float32:
            raise ValueError("GradSync(exchange='a2a') averages the fp32 grads")
        self.numels = [p.numel() for p in self.params]
        # a2a: buckets split into n equal 64-element-aligned shards
        balign = _lib.ALIGN_ELEMS * (self.world_size if self.a2a else 1)
        self.tree = self.k.tree(self.numels, self.device, bucket_cap_elems, balign)
        self.wire = torch.zeros(self.tree.total, dtype=wire_dtype, device=self.device)
        if self.a2a:
            n = self.world_size
            smax = max((hi - lo) // n for lo, hi in self.tree.bucket_ranges) if \
                self.tree.n_buckets else 0
            z = dict(dtype=torch.float32, device=self.device)
            # landing buffers and averaged shards, one per bucket in flight
            self.a2a_recv = [torch.zeros(n * smax, **z) for _ in range(2)]
            self.a2a_avg = [torch.zeros(smax, **z) for _ in range(2)]
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

        # one replica (self.local): the all-reduce is the identity (the rebinding, gather and
        # /1 still run, so the path is exercised on a one-GPU machine)
        local = self.local
        if self.a2a and not local:
            self._sync_a2a()
            return
        pipelined_buckets(
            self.tree.n_buckets,
            lambda b: self.k.gather(self.tree, b, SLOT_GRAD, self.wire),
            lambda b: _Done() if local else dist.all_reduce(
                view(b), op=dist.ReduceOp.SUM, group=self.group, async_op=True),
            lambda b: self.k.unpack_avg(self.tree, b, self.wire, self.world_size, SLOT_GRAD),
        )

    def _sync_a2a(self) -> None:
        """gather(b) -> all_to_all(b) | rank-order average(b) -> all_gather(b) | copy back(b),
        overlapped across buckets like OuterSync's sharded step."""
        n, nb = self.world_size, self.tree.n_buckets

        def shard(b):
            lo, hi = self.tree.bucket_ranges[b]
            return (hi - lo) // n

        def a2a(b):
            lo, hi = self.tree.bucket_ranges[b]
            self.k.gather(self.tree, b, SLOT_GRAD, self.wire)
            return dist.all_to_all_single(self.a2a_recv[b % 2][:n * shard(b)], self.wire[lo:hi],
                                          group=self.group, async_op=True)

        if nb == 0:
            return
        x, ag = [None] * nb, [None] * nb
        x[0] = a2a(0)
        for b in range(nb):
            if b + 1 < nb:
                x[b + 1] = a2a(b + 1)
            x[b].wait()
            s = shard(b)
            self.k.shard_reduce_avg(self.a2a_recv[b % 2][:n * s], n, self.a2a_avg[b % 2][:s])
            lo, hi = self.tree.bucket_ranges[b]
            ag[b] = dist.all_gather_into_tensor(self.wire[lo:hi], self.a2a_avg[b % 2][:s],
                                                group=self.group, async_op=True)
            if b >= 1:
                ag[b - 1].wait()
                self.k.unpack_avg(self.tree, b - 1, self.wire, 1, SLOT_GRAD)
        ag[nb - 1].wait()
        self.k.unpack_avg(self.tree, nb - 1, self.wire, 1, SLOT_GRAD)

    def close(self) -> None:
        self.tree.close()
