"""Device-resident DiLoCo outer step: packed θ_outer / momentum in HBM, HIP kernels, RCCL.

One `OuterSync` per DP replica (one process per GPU). It performs, for the whole tree, what
`src/train.py:261-269` does per tensor on the CPU:

    compute_pseudo_gradient   (src/utils.py:218-221)  -> dl_delta_pack   wire = θ_outer - inner
    sync_gradients            (src/comm.py:117-123)   -> the exchange below (Σ over replicas, /n)
    outer_optimizer.step()    (src/train.py:267)      -> Nesterov SGD (torch's arithmetic)
    sync_inner_model          (src/utils.py:223-226)  -> inner = θ

Exchange variants, all bucketed and pipelined across buckets:
  one replica        dl_delta_sgd: delta, SGD and copy-back in one pass (24 B/param);
                     keep_wire=True: dl_delta_pack_sgd, the same pass also storing the packed
                     pseudo-gradient (outer.grad; 28 B/param); fuse_single=False: the
                     two-kernel dl_delta_pack -> dl_unpack_sgd pipeline, tile by tile
  sharded            (default for n > 1 with the fp32 wire) RCCL reduce-scatter ->
                     dl_shard_sgd on this peer's 1/n (θ and momentum shards) -> RCCL all-gather
                     of θ -> dl_scatter; HBM 20 + 20/n B/param, momentum 4P/n
  sharded, ordered   exchange="a2a": the reduce-scatter becomes an RCCL all_to_all of the wire
                     slices + dl_shard_reduce_sgd (Σ in rank order in fp32, /n, SGD): the same
                     bus bytes, a result that does not depend on RCCL's algorithm, bit-exact
                     against the oracle at every n; a bf16 wire is summed in fp32
  replicated         (shard=False; the bf16 wire's default) RCCL all-reduce -> dl_unpack_sgd
                     (/n + SGD + copy-back, 24 B/param) on every replica
  int8 wire          dl_delta_q8 -> all_to_all -> dl_q8_reduce -> all_gather -> dl_unpack_sgd_q8
  direct (xgmi)      exchange="xgmi": IPC-mapped peers, one dl_xgmi_reduce_sgd per rank;
                     exchange="xgmi_inner": no wire -- the inner params live in one packed
                     arena the peers read, dl_xgmi_delta_sgd forms θ - inner_q itself

Layout in HBM: θ_outer, momentum and the wire are packed arrays in
parameters() order with 256-B-aligned segments; the inner parameters stay where PyTorch
allocated them and are reached through a device pointer table.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist

from . import _lib
from .kernels import Q8_SLOT, default_kernels
from .plan import DEFAULT_BUCKET_CAP_ELEMS, SLOT_INNER

ALL = _lib.ALL_BUCKETS
# Tile of dl_pack_sgd_tiled: 8192 chunks = 32 Mi elements, 128 MiB per stream (wire + θ of a
# tile = 256 MiB, the Infinity Cache). Measured cold -- the Infinity Cache scrubbed before
# every step, as after H inner steps (tools/cold_sweep.py, profiles/r02_cold_sweep_*.json):
# T1.3B 8.01 ms whole-range, 7.33 ms at 4096, 6.96 ms at 8192 (the unpack re-reads the tile's
# wire and θ from the Infinity Cache); T125 0.723 / 0.742 / 0.709 ms. Smaller tiles lose:
# every extra launch boundary costs ≈ 2 µs (1024-chunk tiles: T125 0.876 ms).
DEFAULT_TILE_CHUNKS = 8192


def pipelined_buckets(n_buckets: int, pack: Callable[[int], None],
                      reduce: Callable[[int], object], unpack: Callable[[int], None]) -> None:
    """pack(b) -> async reduce(b) -> wait -> unpack(b), overlapped across buckets.

    Issue order: pack(0) red(0) pack(1) red(1) [wait 0, unpack(0)] pack(2) red(2) [wait 1,
    unpack(1)] ...: the collective stream always has the next bucket queued behind the
    current one, while the compute stream packs ahead and unpacks behind it.
    """
    works = [None] * n_buckets
    for b in range(n_buckets):
        pack(b)
        works[b] = reduce(b)
        if b >= 1:
            works[b - 1].wait()
            unpack(b - 1)
    if n_buckets:
        works[n_buckets - 1].wait()
        unpack(n_buckets - 1)


U_BF16 = 2.0 ** -8   # unit roundoff of bf16 (8-bit significand, round to nearest even)
U_F32 = 2.0 ** -24


def bf16_codec_bound(sabs, n: int, exchange: str = "rccl"):
    """The bf16 wire's error contract (config #5): per element, |g_bf16 - g_fp32| <= this, for
    the averaged pseudo-gradient g of n peers, given sabs = Σ_r |d_r| over the peers' deltas
    (numpy array or tensor). Each delta is rounded to bf16 (relative error <= u). exchange
    "rccl" (the replicated bf16 all-reduce): n - 1 partial sums rounded to bf16 in whatever
    order RCCL's ring adds them, each |S_k| <= (1+u)^n Σ|d_r|; "a2a" (the ordered exchange):
    the bf16 slices summed in fp32 in rank order, never re-rounded. Then / n in fp32. First
    order in u, plus the fp32 terms. The update θ_{s-1} - θ_s of Nesterov SGD carries
    lr·((1+m)·bound_s + m²·bound_{s-1}) of it."""
    if exchange == "a2a":
        c = U_BF16 * (1.0 + n * U_F32) + (n + 1) * U_F32
    else:
        c = U_BF16 * (1.0 + (n - 1) * (1.0 + U_BF16) ** n) + (n + 1) * U_F32
    return sabs * (c / n)


class _Done:
    """Handle of a collective that completed synchronously (one replica, no process group)."""

    def wait(self) -> None:
        pass


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
        kernels=None,
        fuse_single: bool = True,
        side_stream: Optional[bool] = None,
        shard: Optional[bool] = None,
        rank: Optional[int] = None,
        exchange: str = "rccl",
        tile_chunks: int = DEFAULT_TILE_CHUNKS,
        keep_wire: bool = False,
    ):
        self._objs = list(params)  # the caller's objects (exchange="xgmi_inner" relays them)
        self.params: List[torch.Tensor] = [p.data if isinstance(p, torch.nn.Parameter) else p
                                           for p in params]
        if not self.params:
            raise ValueError("OuterSync needs at least one parameter")
        if nesterov and momentum == 0:
            raise ValueError("Nesterov momentum requires a momentum")  # torch.optim.SGD's check
        self.k = kernels or default_kernels()
        self.device = self.params[0].device
        self.lr, self.momentum, self.nesterov = float(lr), float(momentum), bool(nesterov)
        self.wire_dtype = wire_dtype
        # one replica: delta + SGD + copy-back in one pass (dl_delta_sgd), no wire round trip
        self.fuse_single = bool(fuse_single)
        # ... and with keep_wire, store the pseudo-gradient into the wire in the same pass
        # (dl_delta_pack_sgd): the reference's outer.grad stays observable after the step
        self.keep_wire = bool(keep_wire)
        # one replica, two-kernel pipeline: pack/step tile by tile (dl_pack_sgd_tiled) so the
        # step re-reads the wire and θ from the Infinity Cache; 0 = whole-range launches
        if tile_chunks < 0:
            raise ValueError(f"tile_chunks {tile_chunks} < 0")
        self.tile_chunks = int(tile_chunks)
        self.group = group
        if world_size is None:
            world_size = dist.get_world_size(group) if dist.is_initialized() else 1
        self.world_size = int(world_size)
        if rank is None:  # this peer's index in the DP group (which shard it owns)
            rank = dist.get_rank(group) if dist.is_initialized() and self.world_size > 1 else 0
        self.rank = int(rank)
        if wire_dtype not in (torch.float32, torch.bfloat16, torch.int8):
            raise ValueError(f"wire dtype {wire_dtype}: float32, bfloat16 or int8")
        self.q8 = wire_dtype == torch.int8
        shard_given = shard
        if shard is None:
            # fp32 wire: same bus bytes as the all-reduce, fewer HBM bytes. bf16 wire: the
            # fp32 all-gather of θ would move 6(n-1)/n B/param against the bf16 all-reduce's
            # 4(n-1)/n, so the replicated step stays the default there.
            shard = self.world_size > 1 and wire_dtype == torch.float32
        if shard and self.q8:
            raise ValueError("the int8 wire has its own exchange; shard=True needs f32/bf16")
        if exchange not in ("rccl", "a2a", "xgmi", "xgmi_inner"):
            raise ValueError(f"exchange {exchange!r}: 'rccl', 'a2a', 'xgmi' or 'xgmi_inner'")
        # a2a: the sharded step with an all_to_all of the wire slices and a rank-order reduce
        # (dl_shard_reduce_sgd) in place of the SUM reduce-scatter
        self.a2a = exchange == "a2a"
        if self.a2a:
            if self.q8:
                raise ValueError("exchange='a2a' exchanges the f32 or bf16 wire")
            if shard_given is False:
                raise ValueError("exchange='a2a' is a sharded step (shard=False contradicts it)")
            shard = True
        # xgmi: the direct peer-access exchange (dl_xgmi_reduce_sgd) over IPC-mapped buffers
        # xgmi_inner: the same with no wire -- the inner parameters move into one packed arena
        # that the peers read, and the exchange kernel forms θ_outer - inner_q itself
        # (dl_xgmi_delta_sgd): no dl_delta_pack pass, no wire buffer
        self.xgmi = exchange in ("xgmi", "xgmi_inner")
        self.xgmi_inner = exchange == "xgmi_inner"
        if self.xgmi and wire_dtype != torch.float32:
            raise ValueError(f"exchange={exchange!r} sends the fp32 wire")
        self.sharded = bool(shard) and not self.xgmi
        # sharded / xgmi: buckets (and the tree) align to 64·n elements -> n equal aligned shards
        balign = _lib.ALIGN_ELEMS * (self.world_size if (self.sharded or self.xgmi) else 1)
        self.tree = self.k.tree([p.numel() for p in self.params], self.device, bucket_cap_elems,
                                balign)
        self.k.bind(self.tree, SLOT_INNER, self.params, self.device)
        # a1 get_outer_model (src/utils.py:213-216): θ_outer starts as a copy of inner.
        # zeros, so the alignment padding of every packed buffer stays zero forever.
        z = dict(device=self.device)
        self.theta = torch.zeros(self.tree.total, dtype=torch.float32, **z)
        self.mom = (torch.zeros(self.tree.total, dtype=torch.float32, **z)
                    if self.momentum != 0 and not (self.sharded or self.xgmi) else None)
        if self.q8:
            # int8 codec: one Q8_SLOT-byte slot per chunk; bucket b's slots padded to a
            # multiple of the peer count so both exchanges split evenly (dl_q8.hip)
            n = self.world_size
            self.q8_plan, base, mmax = [], 0, 1
            for c0, c1 in self.tree.bucket_chunks:
                m = max(1, -(-(c1 - c0) // n))
                self.q8_plan.append((c1 - c0, m, base))
                base += n * m
                mmax = max(mmax, m)
            self.wire = None
            self.q_slots = torch.zeros(base * Q8_SLOT, dtype=torch.uint8, **z)
            self.q_recv = torch.zeros(n * mmax * Q8_SLOT, dtype=torch.uint8, **z)
            self.q_red = torch.zeros(mmax * Q8_SLOT, dtype=torch.uint8, **z)
        elif self.xgmi_inner:
            self.wire = None
        else:
            self.wire = torch.zeros(self.tree.total, dtype=wire_dtype, **z)
        self.k.gather(self.tree, ALL, SLOT_INNER, self.theta)
        if self.sharded:
            # shard b of this peer: θ[lo + r·s, lo + (r+1)·s) with s = (hi - lo)/n, kept in
            # contiguous shard buffers at offset shard_off[b]
            n, r = self.world_size, self.rank
            self.shard_off, off = [], 0
            for lo, hi in self.tree.bucket_ranges:
                assert (hi - lo) % n == 0
                self.shard_off.append(off)
                off += (hi - lo) // n
            self.shard_total = off
            self.th_shard = torch.empty(off, dtype=torch.float32, **z)
            for b in range(self.tree.n_buckets):
                self.th_shard_view(b).copy_(self.theta_shard_of(b))
            self.g_shard = None if self.a2a else torch.zeros(off, dtype=wire_dtype, **z)
            self.mom_shard = (torch.zeros(off, dtype=torch.float32, **z)
                              if self.momentum != 0 else None)
            # exchange="a2a": all_to_all landing buffers, made on first use (a one-replica
            # engine without a process group never exchanges)
            self.a2a_recv: Optional[List[torch.Tensor]] = None
        if self.xgmi:
            from .xgmi import PeerMap

            n = self.world_size
            self.x_len = self.tree.total // n
            self.x_lo = self.rank * self.x_len
            self.mom_x = (torch.zeros(self.x_len, dtype=torch.float32, **z)
                          if self.momentum != 0 else None)
            self._flag = torch.zeros(1, dtype=torch.float32, **z)
            if self.xgmi_inner:
                self._relay_inner()
            src = self.inner_arena if self.xgmi_inner else self.wire
            self.peers = PeerMap({"src": src, "theta": self.theta},
                                 group if n > 1 else None, self.device)
            if not self.peers.ok:
                raise RuntimeError(f"exchange='xgmi' unavailable: {self.peers.reason}")
        self.steps_done = 0
        self._step_bound = False
        # step() runs on its own stream, ordered after the caller's current stream and joined
        # back into it: work other threads put on the default stream meanwhile (the
        # reference's p2p send threads copy activations with .to("cpu"), src/comm.py:38)
        # overlaps the outer step instead of queueing behind it.
        # side_stream=None (auto): a side stream wherever the step has stages to order against
        # the collectives; the one-replica fused step is ONE kernel, so it launches on the
        # caller's stream -- the two joins would add two cross-queue hops (22 us of a 0.61 ms
        # step, profiles/r02_stream_ab.json) and the join back orders the caller behind the
        # kernel anyway.
        if side_stream is None:
            side_stream = not (self.world_size == 1 and self.fuse_single and not self.q8
                               and not self.xgmi and not self.sharded)
        self.stream = (torch.cuda.Stream(self.device)
                       if side_stream and self.device.type == "cuda" else None)

    # ---- building blocks (each stream-ordered on the current stream) ----------------------
    def _relay_inner(self) -> None:
        """exchange="xgmi_inner": move every inner parameter's storage into one packed arena
        (same layout as θ; values, Parameter objects, autograd and optimizer state unchanged),
        so the peers map ONE allocation per rank and read the inner values directly."""
        z = dict(dtype=torch.float32, device=self.device)
        self.inner_arena = torch.zeros(self.tree.total, **z)
        with torch.no_grad():
            for i, o in enumerate(self._objs):
                lo = int(self.tree.seg_off[i])
                v = self.inner_arena[lo:lo + o.numel()].view(o.shape)
                v.copy_(o.data if isinstance(o, torch.nn.Parameter) else o)
                o.data = v
        self.params = [o.data if isinstance(o, torch.nn.Parameter) else o for o in self._objs]
        self._arena_ptrs = [o.data_ptr() for o in self._objs]
        self.k.bind(self.tree, SLOT_INNER, self.params, self.device)

    def _bind_inner(self) -> None:
        """Point the tree's inner slot at the inner params' current storage (a no-op when
        unchanged). step() binds once up front; the per-bucket building blocks bind when they
        are called on their own (checking 292 addresses per bucket would cost ~1 ms of host
        time per T1.3B step)."""
        if not self._step_bound:
            self.k.bind(self.tree, SLOT_INNER, self.params, self.device)

    def pseudo_gradient(self, bucket: int = ALL) -> None:
        """wire[bucket] = θ_outer - inner (a2); int8 wire: its quantised slots."""
        if self.xgmi_inner:
            raise RuntimeError("exchange='xgmi_inner' has no wire: the exchange kernel forms "
                               "the pseudo-gradient; use step()")
        self._bind_inner()
        if self.q8:
            self.k.delta_q8(self.tree, bucket, SLOT_INNER, self.theta, self.q8_region(bucket))
        else:
            self.k.delta_pack(self.tree, bucket, SLOT_INNER, self.theta, self.wire)

    def q8_region(self, bucket: int) -> torch.Tensor:
        """The int8 slots of one bucket (n * m slots, chunk order, zero padding at the end)."""
        if bucket == ALL:
            if self.tree.n_buckets != 1:
                raise ValueError("the int8 wire works bucket by bucket")
            bucket = 0
        _nch, m, base = self.q8_plan[bucket]
        return self.q_slots[base * Q8_SLOT:(base + self.world_size * m) * Q8_SLOT]

    def q8_exchange(self, bucket: int):
        """all_to_all -> dl_q8_reduce (Σ_r in rank order, / n, re-quantise) -> async all_gather
        of the averaged slots back into the bucket's region; returns the all_gather handle."""
        _nch, m, _base = self.q8_plan[bucket]
        n = self.world_size
        region = self.q8_region(bucket)
        recv = self.q_recv[:n * m * Q8_SLOT]
        dist.all_to_all_single(recv, region, group=self.group, async_op=True).wait()
        red = self.q_red[:m * Q8_SLOT]
        self.k.q8_reduce(recv, n, m, n, red)
        return dist.all_gather_into_tensor(region, red, group=self.group, async_op=True)

    # ---- sharded variant --------------------------------------------------------
    def _shard_len(self, bucket: int) -> int:
        lo, hi = self.tree.bucket_ranges[bucket]
        return (hi - lo) // self.world_size

    def theta_shard_of(self, bucket: int) -> torch.Tensor:
        """This peer's slice of the full packed θ in one bucket."""
        lo, _ = self.tree.bucket_ranges[bucket]
        s = self._shard_len(bucket)
        return self.theta[lo + self.rank * s:lo + (self.rank + 1) * s]

    def _shard(self, buf: Optional[torch.Tensor], bucket: int) -> Optional[torch.Tensor]:
        if buf is None:
            return None
        o = self.shard_off[bucket]
        return buf[o:o + self._shard_len(bucket)]

    def th_shard_view(self, bucket: int) -> torch.Tensor:
        return self._shard(self.th_shard, bucket)

    def _local(self) -> bool:
        # one replica: both collectives are identities (plain copies) -- unless a one-rank
        # process group is there to carry them (the single-rank RCCL transport test)
        if self.world_size != 1:
            return False
        return not dist.is_initialized() or dist.get_world_size(self.group) != 1

    def _a2a_slices(self, bucket: int) -> torch.Tensor:
        if self.a2a_recv is None:
            # one buffer per bucket in flight (the step overlaps the exchange of bucket b+1
            # with the reduce of bucket b): n slices of the largest shard
            smax = max(self._shard_len(b) for b in range(self.tree.n_buckets))
            self.a2a_recv = [torch.zeros(self.world_size * smax, dtype=self.wire_dtype,
                                         device=self.device) for _ in range(2)]
        return self.a2a_recv[bucket % 2][:self.world_size * self._shard_len(bucket)]

    def reduce_scatter(self, bucket: int, async_op: bool = True):
        """SUM reduce-scatter of one wire bucket: this peer receives the sum of its 1/n.
        exchange="a2a": an all_to_all instead -- this peer receives the n ranks' copies of its
        1/n, summed in rank order by shard_apply."""
        if self.a2a:
            if self._local():  # one replica: the bucket itself is the one slice
                return _Done()
            return dist.all_to_all_single(self._a2a_slices(bucket), self.bucket_view(bucket),
                                          group=self.group, async_op=async_op)
        if self._local():
            self._shard(self.g_shard, bucket).copy_(self.bucket_view(bucket))
            return _Done()
        return dist.reduce_scatter_tensor(self._shard(self.g_shard, bucket),
                                          self.bucket_view(bucket), op=dist.ReduceOp.SUM,
                                          group=self.group, async_op=async_op)

    def shard_apply(self, bucket: int) -> None:
        """g = Σ/n; Nesterov SGD on this peer's θ and momentum shards (a3 /n, a4)."""
        if self.a2a:
            slices = self.bucket_view(bucket) if self._local() else self._a2a_slices(bucket)
            self.k.shard_reduce_sgd(slices, self.world_size, self.th_shard_view(bucket),
                                    self._shard(self.mom_shard, bucket), self.lr, self.momentum,
                                    self.nesterov, self.steps_done == 0)
            return
        self.k.shard_sgd(self._shard(self.g_shard, bucket), self.world_size,
                         self.th_shard_view(bucket), self._shard(self.mom_shard, bucket),
                         self.lr, self.momentum, self.nesterov, self.steps_done == 0)

    def all_gather(self, bucket: int, async_op: bool = True):
        """Every peer's updated θ shard -> the full packed θ of the bucket."""
        lo, hi = self.tree.bucket_ranges[bucket]
        if self._local():
            self.theta[lo:hi].copy_(self.th_shard_view(bucket))
            return _Done()
        return dist.all_gather_into_tensor(self.theta[lo:hi], self.th_shard_view(bucket),
                                           group=self.group, async_op=async_op)

    def write_inner(self, bucket: int) -> None:
        """a5: inner = θ_outer for one bucket (dl_scatter)."""
        self._bind_inner()
        self.k.scatter(self.tree, bucket, self.theta, SLOT_INNER)

    def momentum_full(self) -> Optional[torch.Tensor]:
        """The packed momentum of the whole tree (sharded: all-gathered; for checks/export)."""
        if self.xgmi:
            if self.mom_x is None:
                return None
            out = torch.empty(self.tree.total, dtype=torch.float32, device=self.device)
            if self.world_size > 1:
                dist.all_gather_into_tensor(out, self.mom_x, group=self.group)
            else:
                out.copy_(self.mom_x)
            return out
        if not self.sharded or self.mom_shard is None:
            return self.mom
        out = torch.zeros(self.tree.total, dtype=torch.float32, device=self.device)
        for b in range(self.tree.n_buckets):
            lo, hi = self.tree.bucket_ranges[b]
            if self._local():
                out[lo:hi].copy_(self._shard(self.mom_shard, b))
            else:
                dist.all_gather_into_tensor(out[lo:hi], self._shard(self.mom_shard, b),
                                            group=self.group)
        return out

    def bucket_view(self, bucket: int) -> torch.Tensor:
        if bucket == ALL:
            return self.wire
        lo, hi = self.tree.bucket_ranges[bucket]
        return self.wire[lo:hi]

    def _replicated_only(self, what: str) -> None:
        if self.xgmi:
            raise RuntimeError(f"{what}: this engine exchanges through IPC (exchange='xgmi'); "
                               "use step()")
        if self.sharded:
            raise RuntimeError(f"{what}: this engine runs the sharded step (shard=True); use "
                               "step() or reduce_scatter / shard_apply / all_gather / write_inner")

    def all_reduce(self, bucket: int, async_op: bool = True):
        """SUM all-reduce of one wire bucket over the DP group (RCCL), a3 minus the /n."""
        self._replicated_only("all_reduce")
        return dist.all_reduce(self.bucket_view(bucket), op=dist.ReduceOp.SUM, group=self.group,
                               async_op=async_op)

    def apply(self, bucket: int = ALL, write_inner: bool = True) -> None:
        """g = wire/n; Nesterov SGD on θ_outer; inner = θ_outer (a3 /n, a4, a5)."""
        self._replicated_only("apply")
        slot = SLOT_INNER if write_inner else -1
        if self.q8:  # the slots already hold the average
            self.k.unpack_sgd_q8(self.tree, bucket, self.q8_region(bucket), self.theta, self.mom,
                                 self.lr, self.momentum, self.nesterov, self.steps_done == 0,
                                 slot)
            return
        self.k.unpack_sgd(self.tree, bucket, self.wire, self.world_size, self.theta, self.mom,
                          self.lr, self.momentum, self.nesterov, self.steps_done == 0, slot)

    # ---- the outer step ---------------------------------------------------------------------
    def step(self, pipeline: Optional[bool] = None) -> None:
        """One DiLoCo outer step over the whole tree (src/train.py:261-269).

        pipeline=True runs the bucketed collective path even for a single replica (an
        identity all-reduce): it validates the transport on a one-GPU machine."""
        if self.stream is None:
            self._step(pipeline)
            return
        cur = torch.cuda.current_stream(self.device)
        if cur == self.stream:  # the caller already runs on the engine's stream
            self._step(pipeline)
            return
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self._step(pipeline)
        cur.wait_stream(self.stream)

    def _step(self, pipeline: Optional[bool]) -> None:
        if pipeline is None:
            pipeline = self.world_size > 1
        if not self.xgmi_inner:
            self.k.bind(self.tree, SLOT_INNER, self.params, self.device)
        self._step_bound = True
        try:
            self._step_body(pipeline)
        finally:
            self._step_bound = False
        self.steps_done += 1

    def _step_body(self, pipeline: bool) -> None:
        if self.q8:
            self._step_q8(pipeline)
        elif self.xgmi:
            self._step_xgmi()
        elif self.sharded:
            self._step_sharded()
        elif pipeline:
            pipelined_buckets(self.tree.n_buckets, self.pseudo_gradient,
                              lambda b: self.all_reduce(b, async_op=True), self.apply)
        elif self.fuse_single and self.keep_wire:
            # src/comm.py:118-119: one peer -> no all-reduce and no division
            self.k.delta_pack_sgd(self.tree, ALL, SLOT_INNER, self.theta, self.wire, self.mom,
                                  self.lr, self.momentum, self.nesterov, self.steps_done == 0)
        elif self.fuse_single:
            self.k.delta_sgd(self.tree, ALL, SLOT_INNER, self.theta, self.mom, self.lr,
                             self.momentum, self.nesterov, self.steps_done == 0)
        elif self.tile_chunks:
            self.k.pack_sgd_tiled(self.tree, ALL, SLOT_INNER, self.theta, self.wire, self.mom,
                                  self.lr, self.momentum, self.nesterov, self.steps_done == 0,
                                  self.tile_chunks)
        else:
            self.pseudo_gradient(ALL)
            self.apply(ALL)

    def _step_sharded(self) -> None:
        """pack(b) -> RS(b) | shard SGD(b) -> AG(b) | scatter(b), overlapped across buckets:
        the collective stream runs RS(0) RS(1) AG(0) RS(2) AG(1) ... while the compute stream
        packs ahead, steps the shard in between and writes the inner params behind."""
        nb = self.tree.n_buckets
        rs, ag = [None] * nb, [None] * nb
        self.pseudo_gradient(0)
        rs[0] = self.reduce_scatter(0)
        for b in range(nb):
            if b + 1 < nb:
                self.pseudo_gradient(b + 1)
                rs[b + 1] = self.reduce_scatter(b + 1)
            rs[b].wait()
            self.shard_apply(b)
            ag[b] = self.all_gather(b)
            if b >= 1:
                ag[b - 1].wait()
                self.write_inner(b - 1)
        ag[nb - 1].wait()
        self.write_inner(nb - 1)

    def _barrier(self) -> None:
        """All ranks' preceding work on their streams is complete (a stream-ordered 4-B
        all-reduce with RCCL; gloo blocks the host)."""
        if self.world_size > 1:
            dist.all_reduce(self._flag, group=self.group)

    def _step_xgmi(self) -> None:
        """delta_pack -> barrier -> dl_xgmi_reduce_sgd (peers' wires summed in rank order, SGD
        on this rank's shard, θ shard stored into every peer) -> barrier -> inner = θ."""
        if self.xgmi_inner:
            if any(o.data_ptr() != e for o, e in zip(self._objs, self._arena_ptrs)):
                raise RuntimeError("exchange='xgmi_inner': an inner parameter's storage was "
                                   "replaced after the engine moved it into its packed arena, "
                                   "which the peers read")
        else:
            self.pseudo_gradient(ALL)
        # every XCD's L2 written back / invalidated around each barrier (dl_sys_fence): peers
        # read this wire (or inner arena) and write this θ over xGMI, outside this GPU's L2
        self.k.sys_fence(self.device)
        self._barrier()
        self.k.sys_fence(self.device)
        step = self.k.xgmi_delta_sgd if self.xgmi_inner else self.k.xgmi_reduce_sgd
        step(self.peers.table("src"), self.peers.table("theta"), self.world_size, self.rank,
             self.x_lo, self.x_len, self.mom_x, self.lr, self.momentum, self.nesterov,
             self.steps_done == 0, self.device)
        self.k.sys_fence(self.device)
        self._barrier()
        self.k.sys_fence(self.device)
        if self.xgmi_inner:  # inner = θ: one flat copy of the arena (padding stays zero)
            self.inner_arena.copy_(self.theta)
        else:
            self.k.scatter(self.tree, ALL, self.theta, SLOT_INNER)

    def _step_q8(self, pipeline: bool) -> None:
        nb = self.tree.n_buckets
        if not pipeline and self.world_size == 1:
            # one replica: the average of one is its own re-quantised slots. At n = 1 no bucket
            # is padded, so the buckets' slots are the tree's chunks in order and each kernel
            # covers the whole tree in one launch
            self.k.delta_q8(self.tree, ALL, SLOT_INNER, self.theta, self.q_slots)
            self.k.q8_reduce(self.q_slots, 1, self.tree.n_chunks, 1, self.q_slots)
            self.k.unpack_sgd_q8(self.tree, ALL, self.q_slots, self.theta, self.mom, self.lr,
                                 self.momentum, self.nesterov, self.steps_done == 0, SLOT_INNER)
            return
        if not pipeline:  # no exchange requested: each replica re-quantises its own slots
            for b in range(nb):
                self.pseudo_gradient(b)
                nch, m, _ = self.q8_plan[b]
                region = self.q8_region(b)
                self.k.q8_reduce(region, 1, m, 1, region)
                self.apply(b)
            return
        # pack(b+1) and its all_to_all overlap all_gather(b) and unpack(b)
        self.pseudo_gradient(0)
        for b in range(nb):
            gather = self.q8_exchange(b)
            if b + 1 < nb:
                self.pseudo_gradient(b + 1)
            gather.wait()
            self.apply(b)

    # ---- checkpoint / resume -----------------------------------------------------------------
    def state_dict(self) -> dict:
        """Outer state in parameters() order, independent of layout and world size: per-tensor
        θ_outer and momentum (sharded: all-gathered; collective over the group) and the step
        count (the first step creates the momentum, torch.optim.SGD's rule)."""
        mom = self.momentum_full()
        return {"theta": [t.clone() for t in self.unpacked(self.theta)],
                "momentum": None if mom is None else [t.clone() for t in self.unpacked(mom)],
                "steps": self.steps_done, "lr": self.lr, "momentum_factor": self.momentum,
                "nesterov": self.nesterov}

    def load_state_dict(self, state: dict, write_inner: bool = True) -> None:
        """Restore a state_dict() (from any world size / bucket layout). write_inner: also set
        the inner parameters to θ_outer, as after an outer step."""
        th = state["theta"]
        if len(th) != len(self.params) or any(a.numel() != p.numel()
                                               for a, p in zip(th, self.params)):
            raise ValueError("state_dict does not match this engine's parameter tree")
        if int(state["steps"]) > 0 and self.momentum != 0 and state.get("momentum") is None:
            raise ValueError("state_dict after step >= 1 must carry the momentum")
        with torch.no_grad():
            for dst, src in zip(self.unpacked(self.theta), th):
                dst.copy_(src.view(dst.shape))
            mom = state.get("momentum")
            if self.momentum != 0 and mom is not None:
                full = torch.zeros(self.tree.total, dtype=torch.float32, device=self.device)
                for dst, src in zip(self.unpacked(full), mom):
                    dst.copy_(src.view(dst.shape))
                if self.xgmi:
                    self.mom_x.copy_(full[self.x_lo:self.x_lo + self.x_len])
                elif self.sharded:
                    for b in range(self.tree.n_buckets):
                        lo, _ = self.tree.bucket_ranges[b]
                        s = self._shard_len(b)
                        self._shard(self.mom_shard, b).copy_(
                            full[lo + self.rank * s:lo + (self.rank + 1) * s])
                else:
                    self.mom.copy_(full)
            if self.sharded:
                for b in range(self.tree.n_buckets):
                    self.th_shard_view(b).copy_(self.theta_shard_of(b))
        self.steps_done = int(state["steps"])
        if write_inner:
            self.k.bind(self.tree, SLOT_INNER, self.params, self.device)
            self.k.scatter(self.tree, ALL, self.theta, SLOT_INNER)

    def unpacked(self, packed: torch.Tensor) -> List[torch.Tensor]:
        """Per-tensor views into a packed buffer (shapes of the inner params)."""
        out = []
        for i, p in enumerate(self.params):
            lo = int(self.tree.seg_off[i])
            out.append(packed[lo:lo + p.numel()].view(p.shape))
        return out

    def close(self) -> None:
        if getattr(self, "peers", None) is not None:
            if self.world_size > 1:  # nobody still reads a buffer this rank is about to unmap
                torch.cuda.synchronize(self.device)
                dist.barrier(group=self.group)
            self.peers.close()
            self.peers = None
        self.tree.close()
