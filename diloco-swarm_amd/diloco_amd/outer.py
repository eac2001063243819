"""Device-resident DiLoCo outer step: packed θ_outer / momentum in HBM, HIP kernels, RCCL.

One `OuterSync` per DP replica (one process per GPU). It performs, for the whole tree, what
`src/train.py:261-269` does per tensor on the CPU:

    compute_pseudo_gradient   (src/utils.py:218-221)  -> dl_delta_pack   wire = θ_outer - inner
    sync_gradients            (src/comm.py:117-123)   -> RCCL all_reduce(SUM) of each bucket
    outer_optimizer.step()    (src/train.py:267)      -> dl_unpack_sgd   g = wire/n; Nesterov SGD
    sync_inner_model          (src/utils.py:223-226)  -> (fused in dl_unpack_sgd) inner = θ

Layout in HBM (DESIGN.md "Data layout"): θ_outer, momentum and the wire buffer are packed
fp32 (wire optionally bf16) arrays in parameters() order with 256-B-aligned segments; the
inner parameters stay where PyTorch allocated them and are reached through a device pointer
table. With n > 1 replicas the buckets are pipelined: pack(b+1) and unpack(b-1) run on the
compute stream while RCCL reduces bucket b on its own stream.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist

from . import _lib
from .plan import DEFAULT_BUCKET_CAP_ELEMS, SLOT_INNER, PackedTree

_WIRE = {torch.float32: _lib.DL_F32, torch.bfloat16: _lib.DL_BF16}


def _stream_handle(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class OuterSync:
    """Device-resident outer state of one replica + the fused outer step."""

    def __init__(
        self,
        params: Sequence[torch.Tensor],
        *,
        lr: float = 0.7,
        momentum: float = 0.9,
        nesterov: bool = True,
        group: Optional[dist.ProcessGroup] = None,
        world_size: Optional[int] = None,
        wire_dtype: torch.dtype = torch.float32,
        bucket_cap_elems: int = DEFAULT_BUCKET_CAP_ELEMS,
    ):
        self.params: List[torch.Tensor] = [p.data if isinstance(p, torch.nn.Parameter) else p
                                           for p in params]
        if not self.params:
            raise ValueError("OuterSync needs at least one parameter")
        self.device = self.params[0].device
        if self.device.type != "cuda":
            raise ValueError("OuterSync keeps the outer state in HBM: parameters must be on a GPU")
        if wire_dtype not in _WIRE:
            raise ValueError(f"wire dtype {wire_dtype} (supported: float32, bfloat16)")
        if nesterov and momentum == 0:
            raise ValueError("Nesterov momentum requires a momentum")  # torch.optim.SGD's check
        self.lr, self.momentum, self.nesterov = float(lr), float(momentum), bool(nesterov)
        self.wire_dtype = wire_dtype
        self.group = group
        if world_size is None:
            world_size = dist.get_world_size(group) if dist.is_initialized() else 1
        self.world_size = int(world_size)
        with torch.cuda.device(self.device):
            self.tree = PackedTree([p.numel() for p in self.params], bucket_cap_elems)
            s = _stream_handle(self.device)
            self.tree.bind(SLOT_INNER, self.params, s)
            # a1 get_outer_model (src/utils.py:213-216): θ_outer starts as a copy of inner.
            # zeros, so the alignment padding of every packed buffer stays zero forever.
            self.theta = torch.zeros(self.tree.total, dtype=torch.float32, device=self.device)
            self.mom = (torch.zeros(self.tree.total, dtype=torch.float32, device=self.device)
                        if self.momentum != 0 else None)
            self.wire = torch.zeros(self.tree.total, dtype=wire_dtype, device=self.device)
            _lib.call("dl_gather", self.tree.handle, _lib.ALL_BUCKETS, SLOT_INNER,
                      self.theta.data_ptr(), _lib.DL_F32, s)
        self.steps_done = 0

    # ---- building blocks (each stream-ordered on the current stream) ----------------------
    def _rebind(self, s: int) -> None:
        self.tree.bind(SLOT_INNER, self.params, s)

    def pseudo_gradient(self, bucket: int = _lib.ALL_BUCKETS) -> None:
        """wire[bucket] = θ_outer - inner (a2)."""
        s = _stream_handle(self.device)
        self._rebind(s)
        _lib.call("dl_delta_pack", self.tree.handle, bucket, SLOT_INNER, self.theta.data_ptr(),
                  self.wire.data_ptr(), _WIRE[self.wire_dtype], s)

    def bucket_view(self, bucket: int) -> torch.Tensor:
        if bucket == _lib.ALL_BUCKETS:
            return self.wire
        lo, hi = self.tree.bucket_ranges[bucket]
        return self.wire[lo:hi]

    def all_reduce(self, bucket: int, async_op: bool = True):
        """SUM all-reduce of one wire bucket over the DP group (RCCL), a3 minus the /n."""
        return dist.all_reduce(self.bucket_view(bucket), op=dist.ReduceOp.SUM, group=self.group,
                               async_op=async_op)

    def apply(self, bucket: int = _lib.ALL_BUCKETS, write_inner: bool = True) -> None:
        """g = wire/n; Nesterov SGD on θ_outer; inner = θ_outer (a3 /n, a4, a5)."""
        s = _stream_handle(self.device)
        _lib.call(
            "dl_unpack_sgd", self.tree.handle, bucket, self.wire.data_ptr(),
            _WIRE[self.wire_dtype], self.world_size, self.theta.data_ptr(),
            self.mom.data_ptr() if self.mom is not None else None,
            self.lr, self.momentum, int(self.nesterov), int(self.steps_done == 0),
            SLOT_INNER if write_inner else -1, s,
        )

    # ---- the outer step ---------------------------------------------------------------------
    def step(self, mark: Optional[Callable[[str], None]] = None) -> None:
        """One DiLoCo outer step over the whole tree (src/train.py:261-269).

        `mark(name)` (optional) is called between phases, e.g. to record HIP events.
        """
        m = mark or (lambda _n: None)
        if self.world_size == 1:
            # src/comm.py:118-119: one peer -> no all-reduce and no division
            m("delta_pack")
            self.pseudo_gradient(_lib.ALL_BUCKETS)
            m("unpack_sgd")
            self.apply(_lib.ALL_BUCKETS)
            m("end")
        else:
            nb = self.tree.n_buckets
            works = [None] * nb
            m("pipeline")
            for b in range(nb):
                self.pseudo_gradient(b)
                works[b] = self.all_reduce(b, async_op=True)
                if b >= 1:
                    works[b - 1].wait()
                    self.apply(b - 1)
            works[nb - 1].wait()
            self.apply(nb - 1)
            m("end")
        self.steps_done += 1

    def state_tensors(self):
        """(θ_outer, momentum) packed views, for checkpoints and tests."""
        return self.theta, self.mom

    def unpacked(self, packed: torch.Tensor) -> List[torch.Tensor]:
        """Per-tensor views into a packed buffer (shapes of the inner params)."""
        out = []
        for i, p in enumerate(self.params):
            lo = int(self.tree.seg_off[i])
            out.append(packed[lo:lo + p.numel()].view(p.shape))
        return out

    def close(self) -> None:
        self.tree.close()
