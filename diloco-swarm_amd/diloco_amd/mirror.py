"""Device mirror of the reference's host-resident outer model.

The reference keeps θ_outer on the CPU (`get_outer_model` -> deepcopy(inner).to("cpu"),
src/utils.py:213-216) and works on it per tensor with pageable copies. The drop-in functions
keep that host-visible state exact -- outer params, outer.grad and the optimizer's momentum
buffers are ordinary CPU tensors holding the reference's values -- but lay them out as views
into three pinned, packed host arenas and mirror them in HBM:

    host (pinned, packed)        device (HBM, packed)
    h_theta  <- params' storage   d_theta
    h_grad   <- .grad views       d_wire   (fp32: the reference's fp32 all-reduce)
    h_mom    <- momentum views    d_mom

so every host<->device transfer is ONE DMA of the whole arena over PCIe, and the compute is the
HIP segment-walker kernels. Coherence is tracked with PyTorch's per-tensor version counters:
a host tensor modified in place by torch code (e.g. the reference's CPU SGD) has a new
`_version`, and the device copy is re-uploaded before its next use. Writes through `.data`
bypass version counters; call `invalidate()` after such writes.

Write-back (`write_back=`): "sync" (default) ends every call with the host tensors holding
the new values, as the reference does. "deferred" (pinned write-back) keeps
the device copy authoritative through the outer step and writes every arena the step changed
back to the host in ONE batch of DMAs, issued at the end of `copy_to_inner`
(sync_inner_model, src/train.py:269) on a side stream and not waited for: the PCIe transfer
overlaps the next inner steps instead of sitting on the outer step's critical path. Until it
completes the host tensors are stale; the next mirror call (and `flush()`, the outer model's
`state_dict()`, `OuterSGD.state_dict()`) waits for it. A host tensor modified while its
device copy is newer is an error, not a silent overwrite.
"""
from __future__ import annotations

import warnings
import weakref
from collections import OrderedDict
from operator import is_
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from . import _lib
from .kernels import default_kernels
from .outer import pipelined_buckets
from .plan import DEFAULT_BUCKET_CAP_ELEMS, SLOT_GRAD, SLOT_INNER

ALL = _lib.ALL_BUCKETS
S_CHUNK = _lib.CHUNK_ELEMS  # elements per tree chunk (one int8 slot each)


def _check_host_params(params: Sequence[torch.Tensor]) -> None:
    for i, p in enumerate(params):
        if p.device.type != "cpu":
            raise ValueError(f"outer parameter {i} is on {p.device}; the outer copy lives on the "
                             "host (src/utils.py:216)")
        if p.dtype != torch.float32:
            raise TypeError(f"outer parameter {i}: {p.dtype}, the outer step is fp32")


WRITE_BACKS = ("lazy", "sync", "deferred")
OUTER_WIRES = ("f32", "bf16", "int8")
# The DP exchange behind sync_gradients for the device outer model at N > 1:
#   "sharded"     per bucket RCCL reduce_scatter -> Nesterov SGD on this rank's 1/n of θ and
#                 the momentum -> RCCL all_gather of θ (20 + 20/n B/param of HBM)
#   "replicated"  per bucket RCCL all_reduce -> the SGD pass on the whole tree on every rank
#   "a2a"         "sharded" with an all_to_all + rank-order sum (bit-exact at every n)
OUTER_EXCHANGES = ("sharded", "replicated", "a2a")
# get_outer_model's default per placement (round 6): the reference's
# outer.grad and momentum buffers are local CPU tensors (src/utils.py:218-221, torch SGD state
# at src/train.py:267), so the host placement defaults to "replicated" -- every rank holds the
# whole average and momentum after each step, every read is local, at the same bus bytes as the
# sharded form (an all_reduce is a reduce_scatter + all_gather) and a full SGD pass per rank.
# The device placement keeps "sharded": its reads of .grad / the momentum at N > 1 are
# collectives, guarded by collective_read() so that a one-rank read raises instead of hanging.
DEFAULT_EXCHANGE = {"host": "replicated", "device": "sharded"}


def _none():
    return None


def collective_read(group, what: str) -> None:
    """Entry of a read that is a collective over the DP group (under the sharded exchange a
    rank holds 1/n of the averaged .grad and of the momentum; reading either gathers the rest
    from its peers). Before the all_gathers start, the ranks agree through the job's
    rendezvous store that every one of them is making this read: the k-th read of `what` on
    this group counts its arrivals, and the last arrival sets the read's state to "go"; a rank
    still waiting after DILOCO_COLLECTIVE_READ_TIMEOUT seconds (default 30) sets it to "abort".
    compare_set makes the two outcomes exclusive, so a read either runs on every rank or raises
    RuntimeError on every rank that enters it -- also a peer arriving after the deadline --
    instead of leaving one rank blocked in an all_gather its peers never make."""
    import os
    from datetime import timedelta

    if not dist.is_initialized():  # no job, no rendezvous store (a group emulated in-process)
        return
    if group is None:
        group = dist.group.WORLD
    n = dist.get_world_size(group)
    if n <= 1:
        return
    from torch.distributed import distributed_c10d as c10d

    get_store = getattr(c10d, "_get_default_store", None)
    if get_store is None:
        raise RuntimeError("torch.distributed has no rendezvous store to agree on a collective "
                           "read; use exchange='replicated' (every read local)")
    store = get_store()
    ranks = ",".join(map(str, dist.get_process_group_ranks(group)))
    base = f"diloco/collective_read/{what}/{ranks}"
    # this rank's count of such reads, kept in the store itself: a new process group (a new
    # store) starts every rank at 1 again
    seq = store.add(f"{base}/seq/{dist.get_rank()}", 1)
    key = f"{base}/{seq}"
    timeout = float(os.environ.get("DILOCO_COLLECTIVE_READ_TIMEOUT", "30"))
    if store.add(key + "/arrived", 1) >= n:
        state = store.compare_set(key + "/state", "", "go")
    else:
        try:
            store.wait([key + "/state"], timedelta(seconds=timeout))
        except Exception:  # the deadline passed: decided below, atomically
            pass
        state = store.compare_set(key + "/state", "", "abort")
    if bytes(state) != b"go":
        raise RuntimeError(
            f"reading the outer model's {what} at N > 1 under the sharded exchange is a "
            f"collective over the DP group (ranks [{ranks}]), and not every rank made this "
            f"read within {timeout:g} s (DILOCO_COLLECTIVE_READ_TIMEOUT). Read it on every "
            "rank, call flush_outer_model(outer_model) on every rank first, or use "
            "exchange='replicated' (the host placement's default: every read local)")


def ordered_average(k, tree, wire: torch.Tensor, recv: torch.Tensor, group, n: int,
                    rank: int) -> None:
    """wire <- the rank-order average of every peer's wire, bucket by bucket (the ordered
    form of src/comm.py:120-123, DILOCO_DP_EXCHANGE=a2a): all_to_all hands this rank every
    peer's copy of its 1/n, dl_shard_reduce_avg sums them in rank order and divides into this
    rank's slice of the wire, an in-place all_gather returns the other slices. `recv`: a
    landing buffer the wire's size."""
    for lo, hi in tree.bucket_ranges:
        s = (hi - lo) // n
        dist.all_to_all_single(recv[lo:hi], wire[lo:hi], group=group)
        k.shard_reduce_avg(recv[lo:hi], n, wire[lo + rank * s:lo + (rank + 1) * s])
        dist.all_gather_into_tensor(wire[lo:hi], wire[lo + rank * s:lo + (rank + 1) * s],
                                    group=group)


def dp_bucket_align() -> int:
    """Bucket alignment of an outer model's packed tree: 64 elements times the job's world
    size, so that any DP group -- its size divides the world size, src/world.py:96-97 -- splits
    every bucket into equal 256-B-aligned slices. 64 at one process."""
    if dist.is_available() and dist.is_initialized():
        ws = dist.get_world_size()
    else:
        import os

        ws = int(os.environ.get("WORLD_SIZE", "1") or 1)
    return _lib.ALIGN_ELEMS * max(1, ws)


def shardable(tree, n: int) -> bool:
    """Every bucket splits into n equal slices of whole 16-B vectors (the tree was planned
    with buckets aligned to 64 elements times a multiple of n)."""
    return all((hi - lo) % n == 0 and ((hi - lo) // n) % 4 == 0 for lo, hi in tree.bucket_ranges)


class HostOuterMirror:
    def __init__(self, outer_model: torch.nn.Module, device: torch.device, kernels=None,
                 bucket_cap_elems: int = DEFAULT_BUCKET_CAP_ELEMS, write_back: str = "sync"):
        if write_back not in ("sync", "deferred"):
            raise ValueError(f"write_back {write_back!r}: one of {WRITE_BACKS}")
        self.params: List[torch.nn.Parameter] = list(outer_model.parameters())
        if not self.params:
            raise ValueError("outer model has no parameters")
        _check_host_params(self.params)
        self.k = kernels or default_kernels()
        self.device = torch.device(device)
        self.numels = [p.numel() for p in self.params]
        self.tree = self.k.tree(self.numels, self.device, bucket_cap_elems, dp_bucket_align())
        self.offs = [int(o) for o in self.tree.seg_off[:-1]]
        total = self.tree.total
        pin = self.device.type == "cuda"
        self.h_theta = torch.zeros(total, dtype=torch.float32, pin_memory=pin)
        self.h_grad = torch.zeros(total, dtype=torch.float32, pin_memory=pin)
        self.h_mom: Optional[torch.Tensor] = None
        self.d_theta = torch.zeros(total, dtype=torch.float32, device=self.device)
        self.d_wire = torch.zeros(total, dtype=torch.float32, device=self.device)
        self.d_mom: Optional[torch.Tensor] = None
        self._theta_key = None
        self._grad_key = None
        self._mom_key = None
        # deferred write-back: arenas whose device copy is newer than the host, and the event
        # of the write-back DMAs in flight
        self.deferred = write_back == "deferred"
        self._dirty: set = set()
        self._wb_event = None
        self._mom_bufs: Optional[List[torch.Tensor]] = None
        self._wb_stream = (torch.cuda.Stream(self.device)
                           if self.deferred and self.device.type == "cuda" else None)
        self._relay_params()

    # ---- host arenas ---------------------------------------------------------------------
    def _view(self, arena: torch.Tensor, i: int) -> torch.Tensor:
        o = self.offs[i]
        return arena[o:o + self.numels[i]].view(self.params[i].shape)

    def _relay_params(self) -> None:
        """Move every outer parameter's storage into h_theta (values unchanged)."""
        with torch.no_grad():
            for i, p in enumerate(self.params):
                v = self._view(self.h_theta, i)
                if p.data.data_ptr() != v.data_ptr():
                    v.copy_(p.data)
                    p.data = v
        self._theta_key = None

    def _param_key(self):
        return tuple((p._version, p.data_ptr()) for p in self.params)

    def _grad_key_now(self):
        return tuple(None if p.grad is None else (p.grad.data_ptr(), p.grad._version)
                     for p in self.params)

    def _stream_sync(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()

    def invalidate(self) -> None:
        """Forget every device copy (after host writes that bypass version counters)."""
        self._theta_key = self._grad_key = self._mom_key = None

    # ---- coherence ------------------------------------------------------------------------
    def theta_to_device(self) -> None:
        if any(p.data_ptr() != self._view(self.h_theta, i).data_ptr()
               for i, p in enumerate(self.params)):
            self._relay_params()
        key = self._param_key()
        if key != self._theta_key:
            self._conflict("theta", "outer parameters")
            self.d_theta.copy_(self.h_theta, non_blocking=True)
            self._theta_key = key

    def _set_grad_views(self) -> None:
        for i, p in enumerate(self.params):
            v = self._view(self.h_grad, i)
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v

    def grads_to_device(self, zero_fill_missing: bool) -> None:
        """Make d_wire equal the host gradients (missing ones per the caller's rule)."""
        if self._grad_key is not None and self._grad_key == self._grad_key_now():
            return
        self._conflict("grad", "outer gradients")
        with torch.no_grad():
            for i, p in enumerate(self.params):
                v = self._view(self.h_grad, i)
                if p.grad is None:
                    if not zero_fill_missing:
                        raise RuntimeError(
                            f"outer parameter {i} has no gradient: the fused outer step updates "
                            "every tensor (call compute_pseudo_gradient first)")
                    v.zero_()  # src/comm.py:121: zeros_like(param)
                elif p.grad.data_ptr() != v.data_ptr():
                    v.copy_(p.grad)
        self._set_grad_views()
        self.d_wire.copy_(self.h_grad, non_blocking=True)
        self._grad_key = self._grad_key_now()

    def _grads_to_host(self) -> None:
        self._set_grad_views()
        if self.deferred:
            self._dirty.add("grad")
        else:
            self.h_grad.copy_(self.d_wire, non_blocking=True)
            self._stream_sync()
        self._grad_key = self._grad_key_now()

    # ---- deferred write-back ----------------------------------------------------------------
    def _conflict(self, arena: str, what: str) -> None:
        if arena in self._dirty:
            raise RuntimeError(
                f"the host {what} changed while the device copy was newer (write_back="
                "'deferred' writes them back at sync_inner_model); call flush() before "
                "modifying them between the outer step's calls")

    def _settle(self) -> None:
        """Wait for the write-back DMAs in flight (host tensors valid afterwards)."""
        if self._wb_event is not None:
            self._wb_event.synchronize()
            self._wb_event = None

    def _write_back(self) -> None:
        """Every dirty arena device -> host, on the side stream after the current stream's
        work; not waited for (the next call or flush() settles it)."""
        if not self._dirty:
            return
        pairs = {"grad": (self.h_grad, self.d_wire), "theta": (self.h_theta, self.d_theta),
                 "mom": (self.h_mom, self.d_mom)}
        if self._wb_stream is None:  # a CPU mirror (tests): plain copies
            for a in self._dirty:
                pairs[a][0].copy_(pairs[a][1])
        else:
            self._wb_stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self._wb_stream):
                for a in ("grad", "theta", "mom"):
                    if a in self._dirty:
                        pairs[a][0].copy_(pairs[a][1], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._wb_stream)
            self._wb_event = ev
        # an arena write bumps the version counter its views share (.grad, momentum buffers;
        # not the parameters, whose .data was set): these writes are ours, not the user's
        if "grad" in self._dirty:
            self._grad_key = self._grad_key_now()
        if "mom" in self._dirty and self._mom_bufs is not None:
            self._mom_key = tuple((b.data_ptr(), b._version) for b in self._mom_bufs)
        self._dirty.clear()

    def flush(self) -> None:
        """Host tensors equal the device state (deferred mode; a no-op otherwise)."""
        self._write_back()
        self._settle()

    # ---- the four reference operations --------------------------------------------------
    def pseudo_gradient(self, inner_params: Sequence[torch.Tensor]) -> None:
        """outer.grad = outer - inner (src/utils.py:218-221), delta computed in HBM."""
        self._settle()
        self.theta_to_device()
        self.k.bind(self.tree, SLOT_INNER, [p.data for p in inner_params], self.device)
        self.k.delta_pack(self.tree, ALL, SLOT_INNER, self.d_theta, self.d_wire)
        self._grads_to_host()

    def all_reduce(self, group: Optional[dist.ProcessGroup], num_peers: int,
                   ordered: bool = False) -> None:
        """grad = Σ_peers grad / n (src/comm.py:120-123): RCCL on d_wire, /n in HBM.
        ordered: the rank-order average (all_to_all + dl_shard_reduce_avg + all_gather;
        DILOCO_DP_EXCHANGE=a2a), when every bucket splits into num_peers slices."""
        self._settle()
        self.grads_to_device(zero_fill_missing=True)
        if ordered and shardable(self.tree, num_peers):
            recv = torch.empty_like(self.d_wire)
            ordered_average(self.k, self.tree, self.d_wire, recv, group, num_peers,
                            dist.get_rank(group))
            self._grads_to_host()
            return

        def view(b):
            lo, hi = self.tree.bucket_ranges[b]
            return self.d_wire[lo:hi]

        pipelined_buckets(
            self.tree.n_buckets, lambda b: None,
            lambda b: dist.all_reduce(view(b), op=dist.ReduceOp.SUM, group=group,
                                      async_op=True),
            lambda b: self.k.unpack_avg(self.tree, b, self.d_wire, num_peers, -1, self.d_wire),
        )
        self._grads_to_host()

    def sgd_step(self, lr: float, momentum: float, nesterov: bool,
                 host_bufs: Optional[List[Optional[torch.Tensor]]]) -> List[Optional[torch.Tensor]]:
        """torch.optim.SGD._single_tensor_sgd over the whole tree (src/train.py:267).

        host_bufs: the optimizer's current momentum buffers (None = not created yet, i.e.
        the first step). Returns the momentum buffers to store in the optimizer state
        (views of the pinned h_mom arena)."""
        self._settle()
        self.theta_to_device()
        self.grads_to_device(zero_fill_missing=False)
        first = True
        if momentum != 0:
            if self.h_mom is None:
                pin = self.device.type == "cuda"
                self.h_mom = torch.zeros_like(self.h_theta, pin_memory=pin)
                self.d_mom = torch.zeros_like(self.d_theta)
            have = [b is not None for b in host_bufs]
            if any(have) and not all(have):
                raise RuntimeError("momentum buffers exist for some outer parameters only")
            first = not any(have)
            if not first:
                views = [self._view(self.h_mom, i) for i in range(len(self.params))]
                key = tuple((b.data_ptr(), b._version) for b in host_bufs)
                if key != self._mom_key:
                    self._conflict("mom", "momentum buffers")
                    with torch.no_grad():
                        for b, v in zip(host_bufs, views):
                            if b.data_ptr() != v.data_ptr():
                                v.copy_(b)
                    self.d_mom.copy_(self.h_mom, non_blocking=True)
        self.k.unpack_sgd(self.tree, ALL, self.d_wire, 1, self.d_theta,
                          self.d_mom if momentum != 0 else None, lr, momentum, nesterov, first, -1)
        bufs: List[Optional[torch.Tensor]] = [None] * len(self.params)
        if momentum != 0:
            bufs = [self._view(self.h_mom, i) for i in range(len(self.params))]
        if self.deferred:
            self._dirty.add("theta")
            if momentum != 0:
                self._dirty.add("mom")
        else:
            self.h_theta.copy_(self.d_theta, non_blocking=True)
            if momentum != 0:
                self.h_mom.copy_(self.d_mom, non_blocking=True)
            self._stream_sync()
        self._theta_key = self._param_key()  # arena writes do not bump parameter versions
        if momentum != 0:
            self._mom_key = tuple((b.data_ptr(), b._version) for b in bufs)
            self._mom_bufs = bufs
        return bufs

    def copy_to_inner(self, inner_params: Sequence[torch.Tensor]) -> None:
        """inner = outer (src/utils.py:223-226), scattered from HBM; deferred mode: then the
        step's write-back to the host, in flight when this returns."""
        self._settle()
        self.theta_to_device()
        self.k.bind(self.tree, SLOT_INNER, [p.data for p in inner_params], self.device)
        self.k.scatter(self.tree, ALL, self.d_theta, SLOT_INNER)
        if self.deferred:
            self._write_back()

    def close(self) -> None:
        self.flush()
        self.tree.close()

    def __deepcopy__(self, memo):  # a copied outer model starts without a mirror
        return None

    def __reduce_ex__(self, proto):  # ... and so does a pickled one
        return (_none, ())



# The C-level `.grad` / `.data` of every tensor: the mirror reads and assigns them through
# these descriptors, bypassing OuterParameter's properties (no recursion, no extra Python call).
_GRAD = torch._C.TensorBase.grad
_DATA = torch._C.TensorBase.data


_DATA_PTR = torch._C.TensorBase.data_ptr
_VERSION = torch._C.TensorBase._version.__get__


def _ptrs(ts: Sequence[torch.Tensor]) -> List[int]:
    return list(map(_DATA_PTR, ts))


def _vers(ts: Sequence[torch.Tensor]) -> List[int]:
    """Version counters: any in-place torch write bumps them (kernel writes through the packed
    arenas and writes through `.data` do not)."""
    return list(map(_VERSION, ts))


def module_params(model: torch.nn.Module) -> List[torch.nn.Parameter]:
    """list(model.parameters()), same order (modules in named_modules() order, each module's
    parameters in registration order, a shared parameter at its first occurrence), with the
    duplicates found by identity instead of Tensor.__hash__ (a Python call per lookup: the
    per-call cost of the drop-in functions on a 148-tensor tree). The modules are walked here
    as named_modules() walks them (pre-order, a shared module at its first occurrence) without
    its generator chain and prefix strings, which were half of this function's time; the
    duplicates go in one C-level dict build (keys keep their first position)."""
    ps: list = []
    mods: set = set()

    def walk(m: torch.nn.Module) -> None:
        mods.add(id(m))
        ps.extend(m._parameters.values())
        for c in m._modules.values():
            if c is not None and id(c) not in mods:
                walk(c)

    walk(model)
    uniq = dict(zip(map(id, ps), ps))
    uniq.pop(id(None), None)  # parameters registered as None
    return list(uniq.values())


class OuterParameter(torch.nn.Parameter):
    """A parameter of a fused device outer model (get_outer_model(..., placement="device")).

    Its mirror defers work the reference does eagerly: compute_pseudo_gradient records the
    delta instead of computing it, and sync_gradients leaves the packed .grad holding the Σ
    with the /n pending, so the outer SGD can run all of it in one pass. Reading or assigning
    `.grad` first completes whatever is pending, so every value a caller observes equals the
    reference's (src/utils.py:221, src/comm.py:122-123). Assigning `.grad` or `.data` also
    tells the mirror that its packed views may have been replaced, so a step in which nobody
    assigned them skips the per-tensor address checks."""

    def _mirror(self):
        r = self.__dict__.get("_dl_mirror")
        return r() if r is not None else None

    @property
    def grad(self):
        m = self._mirror()
        if m is not None and m.pending:
            m.settle_grads()
        return _GRAD.__get__(self)

    @grad.setter
    def grad(self, value):
        m = self._mirror()
        if m is not None:
            if m.pending:
                m.settle_grads()
            m.grads_touched = True
        _GRAD.__set__(self, value)

    @grad.deleter
    def grad(self):
        m = self._mirror()
        if m is not None:
            if m.pending:
                m.settle_grads()
            m.grads_touched = True
        _GRAD.__delete__(self)

    @property
    def data(self):
        return _DATA.__get__(self)

    @data.setter
    def data(self, value):
        m = self._mirror()
        if m is not None:
            m.theta_touched = True
        _DATA.__set__(self, value)

    def __reduce_ex__(self, proto):  # pickles as a plain Parameter (the mirror stays behind),
        # over its own storage (a view would carry the whole packed arena)
        return (torch._utils._rebuild_parameter,
                (_DATA.__get__(self).clone(), self.requires_grad, OrderedDict()))

    def __deepcopy__(self, memo):  # ... and deep-copies as one (a clone of the values)
        if id(self) in memo:
            return memo[id(self)]
        out = torch.nn.Parameter(_DATA.__get__(self).clone(), self.requires_grad)
        memo[id(self)] = out
        return out


# Tensor functions that read metadata only: they never make a sharded momentum gather
_META = frozenset([
    torch.Tensor.data_ptr, torch.Tensor.size, torch.Tensor.dim, torch.Tensor.numel,
    torch.Tensor.stride, torch.Tensor.storage_offset, torch.Tensor.is_contiguous,
    torch.Tensor.element_size, torch.Tensor.nelement, torch.Tensor.ndimension,
    torch.Tensor.shape.__get__, torch.Tensor.dtype.__get__, torch.Tensor.device.__get__,
    torch.Tensor.ndim.__get__, torch.Tensor._version.__get__, torch.Tensor.is_cuda.__get__,
    torch.Tensor.layout.__get__, torch.Tensor.requires_grad.__get__,
    torch.Tensor.is_leaf.__get__, torch.Tensor.grad.__get__, torch.Tensor.__len__,
])


def _gather_momentum_of(args, kwargs) -> None:
    seen = set()

    def visit(x):
        if isinstance(x, MomentumBuffer):
            r = x.__dict__.get("_dl_mirror")
            m = r() if r is not None else None
            if m is not None and id(m) not in seen:
                seen.add(id(m))
                m.gather_momentum()
        elif isinstance(x, (list, tuple)):
            for y in x:
                visit(y)

    visit(args)
    if kwargs:
        visit(tuple(kwargs.values()))


class MomentumBuffer(torch.Tensor):
    """`outer_optimizer.state[p]["momentum_buffer"]` of a fused device outer model (a view of
    its packed momentum arena). Under the sharded exchange every rank's SGD pass updates only
    its own 1/n of the momentum; the rest of the arena is gathered from the peers
    the first time anything reads the values -- any torch function on a buffer other than a
    metadata query, its pickling and its deep copy -- so every value a caller observes is the
    reference's full, replicated momentum (src/utils.py:62-63, torch SGD's state). That gather
    is an all_gather over the DP group: like reading .grad under the sharded exchange, it is a
    collective, made by every rank of the group (as torch.save of the optimizer state in the
    reference's multi-rank runs is). Results of operations are plain tensors."""

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        if func not in _META:
            _gather_momentum_of(args, kwargs)
        with torch._C.DisableTorchFunctionSubclass():
            return func(*args, **(kwargs or {}))

    def _plain(self) -> torch.Tensor:
        _gather_momentum_of((self,), None)
        with torch._C.DisableTorchFunctionSubclass():
            return self.detach().clone()

    def __deepcopy__(self, memo):
        if id(self) in memo:
            return memo[id(self)]
        out = self._plain()
        memo[id(self)] = out
        return out

    def __reduce_ex__(self, proto):  # pickles as a plain tensor of the gathered values
        return self._plain().__reduce_ex__(proto)


class DeviceOuterMirror:
    """Device-resident outer model: the outer parameters, their .grad and
    the optimizer's momentum buffers ARE views into packed HBM arenas, so the reference's
    compute_pseudo_gradient -> sync_gradients -> outer SGD -> sync_inner_model sequence runs
    with no host round trip and no host synchronisation (everything is ordered on the current
    stream). A host copy is made only when asked for (`.cpu()`, `state_dict()`): torch copies
    lazily. Chosen by get_outer_model(..., placement="device") or DILOCO_OUTER_PLACEMENT=device.

    fused=False (eager) runs every call as the reference does, one kernel each:
        dl_delta_pack -> RCCL all_reduce + dl_unpack_avg -> dl_unpack_sgd -> dl_scatter
        = 12 + (8) + 20 + 8 B per parameter (48 at N > 1, 40 at one peer).
    fused=True (the default for this placement, DILOCO_OUTER_FUSED=0 turns it off) keeps the
    observable values and runs the sequence in as few HBM passes as the data flow allows:
      - compute_pseudo_gradient records the delta (inner params, their addresses and version
        counters) instead of computing it;
      - sync_gradients packs each bucket just before its RCCL all_reduce and leaves the /n
        pending (the packed .grad holds the Σ);
      - OuterSGD.step runs ONE pass: at one peer dl_delta_pack_sgd (delta, .grad, SGD, θ and
        the inner params: 28 B/param, the engine's headline kernel); at N > 1 dl_unpack_sgd with
        the divisor and the inner write (24 B after the 12 B pack);
      - sync_inner_model verifies that the inner params still hold θ (same tensors at the same
        addresses, no version bump on either side since that write) and does nothing; anything
        else -> dl_scatter as in eager mode.
    Reading or assigning an outer parameter's .grad completes the pending work first
    (OuterParameter), so .grad always shows the reference's value. Two consequences differ from
    the reference and are the price of the fusion: the inner params receive θ_new during
    OuterSGD.step() rather than in sync_inner_model (train.py reads neither in between), and
    changing the inner params or θ in place between compute_pseudo_gradient and the call that
    consumes the delta raises instead of being silently used (writes through an inner tensor's
    `.data` bypass version counters: call invalidate() after them)."""

    def __init__(self, outer_model: torch.nn.Module, device: torch.device, kernels=None,
                 bucket_cap_elems: int = DEFAULT_BUCKET_CAP_ELEMS, fused: bool = False,
                 wire: str = "f32", exchange: str = "sharded", keep_params: bool = False):
        """keep_params: the outer model's Parameter objects stay the ones it has (their class
        switched to OuterParameter in place) -- for an outer model that got its device only
        at its first compute_pseudo_gradient, after get_optimizer took references to them.
        Its parameters may then still be the CPU tensors the model was built with: each is
        copied straight into its view of the θ arena (and a CPU .grad into the wire arena), so
        the HBM never holds a second whole copy of the model."""
        if wire not in OUTER_WIRES:
            raise ValueError(f"wire {wire!r}: one of {OUTER_WIRES}")
        if exchange not in OUTER_EXCHANGES:
            raise ValueError(f"exchange {exchange!r}: one of {OUTER_EXCHANGES}")
        self.exchange = exchange
        self.params: List[torch.nn.Parameter] = module_params(outer_model)
        if not self.params:
            raise ValueError("outer model has no parameters")
        self.k = kernels or default_kernels()
        self.device = torch.device(device)
        for i, p in enumerate(self.params):
            if p.device != self.device and not (keep_params and p.device.type == "cpu"):
                raise ValueError(f"outer parameter {i} is on {p.device}, expected {self.device}")
            if p.dtype != torch.float32:
                raise TypeError(f"outer parameter {i}: {p.dtype}, the outer step is fp32")
        self.fused = fused
        self.numels = [p.numel() for p in self.params]
        self.tree = self.k.tree(self.numels, self.device, bucket_cap_elems, dp_bucket_align())
        self.offs = [int(o) for o in self.tree.seg_off[:-1]]
        z = dict(dtype=torch.float32, device=self.device)
        self.d_theta = torch.zeros(self.tree.total, **z)
        self.d_wire = torch.zeros(self.tree.total, **z)
        self.d_mom: Optional[torch.Tensor] = None
        # wire="bf16" (BASELINE config #5 behind the drop-in calls): at N > 1 the deltas cross
        # the wire in bf16 (cast in the pack kernel, RCCL's bf16 SUM) and the SGD pass reads
        # them from it; .grad shows the decoded average (the codec's value, not fp32's)
        self.wire = wire
        self.d_wire16 = (torch.zeros(self.tree.total, dtype=torch.bfloat16, device=self.device)
                         if wire == "bf16" else None)
        self._sum16 = False  # the pending Σ is in d_wire16 (.grad's arena is stale)
        # fused, N > 1: the bucket all_reduces sync_gradients left in flight (the SGD pass of
        # bucket b waits for its own collective only, so it overlaps bucket b+1's)
        self._works: Optional[list] = None
        # per-tensor views of each arena and their addresses, made once: the per-step checks
        # compare raw addresses (an outer step must not cost a Python tensor per parameter)
        self._views = {"theta": self._make_views(self.d_theta),
                       "wire": self._make_views(self.d_wire)}
        self._ptrs = {k: [v.data_ptr() for v in vs] for k, vs in self._views.items()}
        # fused mode: OuterParameter flags assignments of .grad / .data, so the address checks
        # run only after one (or after a version bump on θ)
        self.theta_touched = True
        self.grads_touched = True
        self._theta_ver = None
        # the outer parameters share d_theta's version counter (OuterParameters made over its
        # views): θ's version is one integer; parameters kept in place keep their own counters
        self._shared_ver = fused and not keep_params
        host_grads = None
        if any(p.device != self.device for p in self.params):  # keep_params on CPU tensors
            host_grads = [_GRAD.__get__(p) for p in self.params]
            for p in self.params:
                _GRAD.__set__(p, None)
            self._relay("theta", "data", force=True)
        self._relay_theta()
        if host_grads is not None:
            with torch.no_grad():
                for p, g, v in zip(self.params, host_grads, self._views["wire"]):
                    if g is not None:
                        v.copy_(g)
                        _GRAD.__set__(p, v)
        if fused:
            self._install_outer_parameters(outer_model, keep_params)
        self._delta = None   # pending pseudo-gradient: (inner params, ptrs, versions, θ versions)
        self._div = 1        # pending /n: d_wire holds the Σ of the peers' deltas
        self._target = None  # (inner params, ptrs, versions) of the last compute_pseudo_gradient
        self._synced = None  # (inner params, ptrs, versions, θ versions): inner holds θ
        self._mom_src: Optional[List[torch.Tensor]] = None  # the buffers the last step returned
        # sharded exchange state (fused, N > 1): the wire after the collectives ("sharded":
        # this rank's slice of each bucket holds the Σ -- or, after an a2a reduce, the average
        # -- the rest this rank's own deltas; "a2a": the n slices are still in d_recv), the DP
        # group, its size and this rank's index in it; the momentum arena holds this rank's
        # slices only (the rest gathered on first read, MomentumBuffer)
        self._xmode: Optional[str] = None
        self._xgroup, self._xn, self._xrank = None, 1, 0
        self._mom_stale = False
        self._mom_shard = None  # (group, n, rank) of the steps that left it sharded
        self.d_recv: Optional[torch.Tensor] = None  # a2a landing arena (the wire's size)
        self._warned = False

    def _momentum_buffer(self, view: torch.Tensor) -> "MomentumBuffer":
        t = view.as_subclass(MomentumBuffer)
        t.__dict__["_dl_mirror"] = weakref.ref(self)
        return t

    def __deepcopy__(self, memo):  # a copied outer model starts without a mirror
        return None

    def __reduce_ex__(self, proto):  # ... and so does a pickled one
        return (_none, ())

    def _install_outer_parameters(self, model: torch.nn.Module, keep: bool = False) -> None:
        """Fused mode: every parameter of the outer model becomes an OuterParameter created
        over its view of the θ arena (shared parameters stay shared). A tensor made from a view
        shares its base's version counter, so every in-place write to any outer parameter
        bumps d_theta's one counter: the per-call check that θ is unchanged reads one integer
        instead of 148 (or 292) version counters. keep: the same Parameter objects, their class
        switched in place (their data already are the arena's views, _relay_theta)."""
        ref = weakref.ref(self)
        if keep:
            for p in self.params:
                p.__class__ = OuterParameter
                p.__dict__["_dl_mirror"] = ref
            self._theta_ver = self._theta_version()
            return
        index = {id(p): i for i, p in enumerate(self.params)}
        new: List[Optional[OuterParameter]] = [None] * len(self.params)
        for mod in model.modules():
            for name, p in list(mod._parameters.items()):
                if p is None:
                    continue
                i = index[id(p)]
                if new[i] is None:
                    q = OuterParameter(self._views["theta"][i], p.requires_grad)
                    q.__dict__["_dl_mirror"] = ref
                    new[i] = q
                mod._parameters[name] = new[i]
        self.params = new
        self._theta_ver = self._theta_version()

    def _theta_version(self):
        """fused: d_theta's version counter, shared by every outer parameter (one integer);
        eager, or parameters kept in place: the parameters' own counters."""
        return self.d_theta._version if self._shared_ver else _vers(self.params)

    def _make_views(self, arena: torch.Tensor) -> List[torch.Tensor]:
        return [arena[o:o + n].view(p.shape)
                for o, n, p in zip(self.offs, self.numels, self.params)]

    def _view(self, arena: torch.Tensor, i: int) -> torch.Tensor:
        o = self.offs[i]
        return arena[o:o + self.numels[i]].view(self.params[i].shape)

    def _in_place(self, kind: str, what: str) -> bool:
        exp = self._ptrs[kind]
        if what == "data":
            return _ptrs(self.params) == exp
        for p, e in zip(self.params, exp):
            g = _GRAD.__get__(p)
            if g is None or g.data_ptr() != e:
                return False
        return True

    def _relay(self, kind: str, what: str, zero_fill_missing: bool = True,
               force: bool = False) -> bool:
        """Make every parameter's `what` ("data" or "grad") the view of arena `kind`; True if
        any arena content was replaced. force: skip the address check (parameters on another
        device: empty tensors' addresses can coincide across devices)."""
        if not force and self._in_place(kind, what):
            return False
        views = self._views[kind]
        with torch.no_grad():
            for i, p in enumerate(self.params):
                v = views[i]
                cur = _DATA.__get__(p) if what == "data" else _GRAD.__get__(p)
                if cur is not None and cur.data_ptr() == v.data_ptr() and cur.device == v.device:
                    continue
                if cur is None:
                    if not zero_fill_missing:
                        raise RuntimeError(
                            f"outer parameter {i} has no gradient: the fused outer step updates "
                            "every tensor (call compute_pseudo_gradient first)")
                    v.zero_()  # src/comm.py:121: zeros_like(param)
                else:
                    v.copy_(cur)
                if what == "data":
                    _DATA.__set__(p, v)
                else:
                    _GRAD.__set__(p, v)
        return True

    def _relay_theta(self, ver=None):
        """θ's packed arena holds every outer parameter (relayed if one was replaced); returns
        θ's version (_theta_version; `ver`: read by the caller just before). Skips the address
        checks in fused mode when no `.data` was assigned and the version did not move since
        the last call."""
        if ver is None:
            ver = self._theta_version()
        if not self.fused or self.theta_touched or ver != self._theta_ver:
            if self._relay("theta", "data"):
                self._synced = None  # θ's arena content changed: the inner no longer holds it
                ver = self._theta_version()  # the relay's own copies bumped it
            self.theta_touched = False
            self._theta_ver = ver
        return ver

    def _relay_grads(self, zero_fill_missing: bool) -> None:
        if not self.fused or self.grads_touched:
            self._relay("wire", "grad", zero_fill_missing)
            self.grads_touched = False

    def invalidate(self) -> None:
        """After writes through `.data` (no version bump): forget that the inner params hold θ
        and re-check every address at the next call."""
        self._synced = None
        self._target = None
        self.theta_touched = self.grads_touched = True

    # ---- deferred work (fused mode) ------------------------------------------------------
    @property
    def pending(self) -> bool:
        return (self._delta is not None or self._div != 1 or self._sum16
                or self._works is not None or self._xmode is not None)

    # ---- the sharded exchange (fused, N > 1) ---------------------------------------------
    def _own(self, b: int, n: int, rank: int):
        """[a, e): this rank's slice of bucket b when the bucket is split n ways."""
        lo, hi = self.tree.bucket_ranges[b]
        s = (hi - lo) // n
        return lo + rank * s, lo + (rank + 1) * s

    def _exchange_mode(self, n: int, ordered: bool) -> str:
        mode = "a2a" if ordered else self.exchange
        if self.wire == "bf16":
            if ordered and not self._warned:
                self._warned = True
                warnings.warn("the bf16 outer wire reduces with RCCL's bf16 all_reduce; "
                              "DILOCO_DP_EXCHANGE=a2a applies to the fp32 wire only")
            return "replicated"
        if mode == "sharded" and not self.fused:
            return "replicated"  # eager: .grad holds the full average right after the call
        if mode != "replicated" and not shardable(self.tree, n):
            if not self._warned:
                self._warned = True
                warnings.warn(f"outer-model buckets do not split into {n} equal slices (the "
                              "tree was planned for another world size): replicated exchange")
            return "replicated"
        return mode

    def _gather_wire(self) -> None:
        """The pending sharded wire -> every bucket's full Σ (or average) on every rank: the
        a2a slices reduced in rank order, then an in-place all_gather per bucket."""
        collective_read(self._xgroup, "grad")
        mode, self._xmode = self._xmode, None
        n, r, g = self._xn, self._xrank, self._xgroup
        for b in range(self.tree.n_buckets):
            lo, hi = self.tree.bucket_ranges[b]
            a, e = self._own(b, n, r)
            if mode == "a2a":
                self.k.shard_reduce_avg(self.d_recv[lo:hi], n, self.d_wire[a:e])
            dist.all_gather_into_tensor(self.d_wire[lo:hi], self.d_wire[a:e], group=g)

    def gather_momentum(self) -> None:
        """The momentum arena whole again after sharded steps (each rank updated its own
        slices): an in-place all_gather per bucket over the DP group of those steps."""
        if not self._mom_stale:
            return
        g, n, r = self._mom_shard
        collective_read(g, "momentum")
        self._mom_stale = False
        for b in range(self.tree.n_buckets):
            lo, hi = self.tree.bucket_ranges[b]
            a, e = self._own(b, n, r)
            dist.all_gather_into_tensor(self.d_mom[lo:hi], self.d_mom[a:e], group=g)

    def _sharded_sgd(self, mom, lr, momentum, nesterov, first, target) -> None:
        """Per bucket: wait for its reduce_scatter (a2a: all_to_all, then dl_shard_reduce_avg
        into this rank's slice of the wire), dl_shard_sgd on this rank's slice of θ and the
        momentum (/n, torch's Nesterov arithmetic), an in-place RCCL all_gather of θ, and --
        one bucket behind -- dl_scatter of the gathered θ into the inner params."""
        works, self._works = self._works, None
        mode, n, r, g = self._xmode, self._xn, self._xrank, self._xgroup
        write = target is not None
        if write:
            self.k.bind(self.tree, SLOT_INNER, target[0], self.device, key=tuple(target[1]))
        nb = self.tree.n_buckets
        ags = [None] * nb
        for b in range(nb):
            if works is not None:
                works[b].wait()
            lo, hi = self.tree.bucket_ranges[b]
            a, e = self._own(b, n, r)
            if mode == "a2a":
                self.k.shard_reduce_avg(self.d_recv[lo:hi], n, self.d_wire[a:e])
            self.k.shard_sgd(self.d_wire[a:e], 1 if mode == "a2a" else n, self.d_theta[a:e],
                             None if mom is None else mom[a:e], lr, momentum, nesterov, first)
            ags[b] = dist.all_gather_into_tensor(self.d_theta[lo:hi], self.d_theta[a:e],
                                                 group=g, async_op=True)
            if b >= 1:
                ags[b - 1].wait()
                if write:
                    self.k.scatter(self.tree, b - 1, self.d_theta, SLOT_INNER)
        ags[nb - 1].wait()
        if write:
            self.k.scatter(self.tree, nb - 1, self.d_theta, SLOT_INNER)
        # the wire keeps this rank's slices (Σ; after an a2a reduce the average) for a later
        # .grad read; the momentum holds this rank's slices only
        self._xmode = "sharded"
        if mode == "a2a":
            self._div = 1
        if mom is not None:
            self._mom_stale = True
            self._mom_shard = (g, n, r)

    def _take_delta(self, tver_now=None) -> List[torch.Tensor]:
        """The pending delta's inner params, checked unchanged since compute_pseudo_gradient
        and bound to SLOT_INNER (tver_now: θ's version, if the caller has it)."""
        inner, iptrs, ivers, tver = self._delta
        self._delta = None
        if tver_now is None:
            tver_now = self._theta_version()
        if (_ptrs(inner) != iptrs or _vers(inner) != ivers or self.theta_touched
                or tver_now != tver):
            raise RuntimeError(
                "the inner or the outer parameters were modified after compute_pseudo_gradient "
                "and before the pseudo-gradient was used; the fused device outer model computes "
                "it when it is first needed (get_outer_model(..., fused=False) or "
                "DILOCO_OUTER_FUSED=0 computes it eagerly)")
        self.k.bind(self.tree, SLOT_INNER, inner, self.device, key=tuple(iptrs))
        return inner

    def _join(self) -> None:
        """The current stream waits for every collective still in flight on the wire."""
        works, self._works = self._works, None
        for w in works or ():
            w.wait()

    def settle_grads(self) -> None:
        """Complete the pending work so the packed .grad holds the reference's values."""
        self._join()
        if self._delta is not None:
            self._take_delta()
            self.k.delta_pack(self.tree, ALL, SLOT_INNER, self.d_theta, self.d_wire)
        if self._xmode == "q8":  # the averaged int8 slots, decoded into .grad's arena
            self._decode_q8()
        elif self._xmode is not None:  # sharded: a collective over the DP group (class doc)
            self._gather_wire()
        if self._sum16:  # bf16 wire: the decoded average (/n in fp32) into .grad's arena
            div, self._div, self._sum16 = self._div, 1, False
            self.k.unpack_avg(self.tree, ALL, self.d_wire16, div, -1, self.d_wire)
        elif self._div != 1:
            div, self._div = self._div, 1
            self.k.unpack_avg(self.tree, ALL, self.d_wire, div, -1, self.d_wire)

    def flush(self) -> None:
        """No host copy to write back (torch copies to the host on demand); completes the
        deferred .grad work and gathers a sharded momentum (collectives under the sharded
        exchange)."""
        if self.fused:
            self.settle_grads()
            self.gather_momentum()

    def _grad_views(self) -> None:
        if not self.fused or self.grads_touched:
            for p, v, e in zip(self.params, self._views["wire"], self._ptrs["wire"]):
                g = _GRAD.__get__(p)
                if g is None or g.data_ptr() != e:
                    _GRAD.__set__(p, v)
            self.grads_touched = False

    # ---- the four reference operations --------------------------------------------------
    def pseudo_gradient(self, inner_params: Sequence[torch.Tensor]) -> None:
        """outer.grad = outer - inner (src/utils.py:218-221); .grad are views of d_wire."""
        inner = list(inner_params)
        self._join()  # a collective still reading / writing the wire finishes first
        tver = self._relay_theta()
        iptrs = _ptrs(inner)
        self.k.bind(self.tree, SLOT_INNER, inner, self.device, key=tuple(iptrs))
        self._div = 1  # the wire is overwritten: a /n still pending is moot
        self._sum16 = False
        self._xmode = None
        if self.fused:
            ivers = _vers(inner)
            self._delta = (inner, iptrs, ivers, tver)
            self._target = (inner, iptrs, ivers)
        else:
            self.k.delta_pack(self.tree, ALL, SLOT_INNER, self.d_theta, self.d_wire)
        self._grad_views()

    def all_reduce(self, group: Optional[dist.ProcessGroup], num_peers: int,
                   ordered: bool = False) -> None:
        """grad = Σ_peers grad / n (src/comm.py:120-123), in place on the packed .grad.
        ordered (DILOCO_DP_EXCHANGE=a2a): the rank-order sum, bit-exact at every n."""
        if self.wire == "int8":  # its exchange sums in rank order already (dl_q8_reduce)
            self._all_reduce_q8(group, num_peers)
            return
        mode = self._exchange_mode(num_peers, ordered)
        if self.wire == "bf16":
            self._all_reduce_bf16(group, num_peers)
            return
        if mode != "replicated":
            self._all_reduce_sharded(group, num_peers, mode)
            return
        pack = None
        if self._delta is not None:  # fused: each bucket packed just before its collective
            self._take_delta()
            self._relay_theta()
            self._grad_views()

            def pack(b):
                self.k.delta_pack(self.tree, b, SLOT_INNER, self.d_theta, self.d_wire)
        else:
            if self.pending:
                self.settle_grads()  # a second sync_gradients reduces the averages
            self._relay_grads(zero_fill_missing=True)

        def view(b):
            lo, hi = self.tree.bucket_ranges[b]
            return self.d_wire[lo:hi]

        if self.fused:  # every bucket's collective in flight; the SGD pass waits per bucket
            self._launch_reductions(pack, view, group)
            self._div = num_peers
            return
        pipelined_buckets(
            self.tree.n_buckets, pack or (lambda b: None),
            lambda b: dist.all_reduce(view(b), op=dist.ReduceOp.SUM, group=group,
                                      async_op=True),
            lambda b: self.k.unpack_avg(self.tree, b, self.d_wire, num_peers, -1, self.d_wire),
        )

    def _all_reduce_bf16(self, group: Optional[dist.ProcessGroup], num_peers: int) -> None:
        """The bf16 wire: per bucket, the deltas (a pending delta: dl_delta_pack straight to
        bf16; else .grad's fp32 arena cast by dl_gather) -> RCCL all_reduce (bf16 SUM). Fused:
        the Σ stays on the wire for the SGD pass (.grad decodes it when read); eager: decoded
        into .grad with the /n at once (dl_unpack_avg)."""
        w16 = self.d_wire16
        if self._delta is not None:
            self._take_delta()
            self._relay_theta()
            self._grad_views()

            def pack(b):
                self.k.delta_pack(self.tree, b, SLOT_INNER, self.d_theta, w16)
        else:
            if self.pending:
                self.settle_grads()  # a second sync_gradients reduces the averages
            self._relay_grads(zero_fill_missing=True)
            self.k.bind(self.tree, SLOT_GRAD, self._views["wire"], self.device,
                        key=tuple(self._ptrs["wire"]))

            def pack(b):
                self.k.gather(self.tree, b, SLOT_GRAD, w16)

        def view(b):
            lo, hi = self.tree.bucket_ranges[b]
            return w16[lo:hi]

        if self.fused:
            self._launch_reductions(pack, view, group)
            self._div, self._sum16 = num_peers, True
            return
        pipelined_buckets(
            self.tree.n_buckets, pack,
            lambda b: dist.all_reduce(view(b), op=dist.ReduceOp.SUM, group=group,
                                      async_op=True),
            lambda b: self.k.unpack_avg(self.tree, b, w16, num_peers, -1, self.d_wire),
        )

    def _all_reduce_sharded(self, group, n: int, mode: str) -> None:
        """Fused: per bucket pack (the pending delta) then an asynchronous in-place RCCL
        reduce_scatter into this rank's slice of the bucket (mode "a2a": an all_to_all of the
        bucket into d_recv); none waited for here -- OuterSGD.step waits bucket by bucket, a
        .grad read gathers the whole average first. Eager (mode "a2a" only): the rank-order
        average of every bucket into .grad at once."""
        pack = None
        if self._delta is not None:
            self._take_delta()
            self._relay_theta()
            self._grad_views()

            def pack(b):
                self.k.delta_pack(self.tree, b, SLOT_INNER, self.d_theta, self.d_wire)
        else:
            if self.pending:
                self.settle_grads()  # a second sync_gradients reduces the averages
            self._relay_grads(zero_fill_missing=True)
        rank = dist.get_rank(group)
        if mode == "a2a" and self.d_recv is None:
            self.d_recv = torch.empty_like(self.d_wire)
        if not self.fused:
            ordered_average(self.k, self.tree, self.d_wire, self.d_recv, group, n, rank)
            return
        works = []
        for b in range(self.tree.n_buckets):
            if pack is not None:
                pack(b)
            lo, hi = self.tree.bucket_ranges[b]
            a, e = self._own(b, n, rank)
            if mode == "a2a":
                works.append(dist.all_to_all_single(self.d_recv[lo:hi], self.d_wire[lo:hi],
                                                    group=group, async_op=True))
            else:
                works.append(dist.reduce_scatter_tensor(self.d_wire[a:e], self.d_wire[lo:hi],
                                                        op=dist.ReduceOp.SUM, group=group,
                                                        async_op=True))
        self._works = works
        self._xmode, self._xgroup, self._xn, self._xrank = mode, group, n, rank
        self._div = n if mode == "sharded" else 1

    # ---- the int8 wire behind the reference's calls ------------------------
    def _q8_buffers(self, n: int) -> dict:
        """Slot regions of every bucket (n·m slots of Q8_SLOT bytes: the bucket's chunks in
        order, zero padding to a multiple of n), two all_to_all landing buffers, one reduced
        region per bucket (so every bucket's all_gather may stay in flight)."""
        q = getattr(self, "_q8", None)
        if q is not None and q["n"] == n:
            return q
        from .kernels import Q8_SLOT

        plan, base, rbase, mmax = [], 0, 0, 1
        for c0, c1 in self.tree.bucket_chunks:
            m = max(1, -(-(c1 - c0) // n))
            plan.append((c1 - c0, m, base, rbase))
            base += n * m
            rbase += m
            mmax = max(mmax, m)
        z = dict(dtype=torch.uint8, device=self.device)
        segs = []
        for lo, hi in self.tree.bucket_ranges:
            segs.append([i for i, o in enumerate(self.offs) if lo <= o < hi])
        self._q8 = q = {"n": n, "plan": plan, "S": Q8_SLOT, "segs": segs,
                        "slots": torch.zeros(base * Q8_SLOT, **z),
                        "red": torch.zeros(rbase * Q8_SLOT, **z),
                        "recv": [torch.zeros(n * mmax * Q8_SLOT, **z) for _ in range(2)]}
        return q

    def _q8_region(self, q: dict, b: int) -> torch.Tensor:
        nch, m, base, _ = q["plan"][b]
        return q["slots"][base * q["S"]:(base + q["n"] * m) * q["S"]]

    def _all_reduce_q8(self, group, n: int) -> None:
        """Per bucket: dl_delta_q8 (the pending delta quantised straight from θ and the inner
        params; else .grad's fp32 arena) -> all_to_all -> dl_q8_reduce (Σ over the peers in rank
        order, / n, re-quantised) -> all_gather of the averaged slots, left in flight (the
        next bucket's pack and all_to_all are issued before this one's reduce). Fused: the SGD
        pass dequantises inside dl_unpack_sgd_q8; .grad shows the decoded average when read.
        Eager: decoded into .grad at once."""
        if self._delta is not None:
            self._take_delta()
            self._relay_theta()
            self._grad_views()
            theta, slot = self.d_theta, SLOT_INNER
        else:
            if self.pending:
                self.settle_grads()  # a second sync_gradients reduces the averages
            self._relay_grads(zero_fill_missing=True)
            # the deltas are .grad itself: quantise (wire - 0) -> θ slot holds the wire,
            # the "inner" slot zeros (a zero arena bound in the auxiliary slot)
            if getattr(self, "_q8_zero", None) is None:
                self._q8_zero = [torch.zeros_like(v) for v in self._views["wire"]]
                from .plan import SLOT_AUX
                self.k.bind(self.tree, SLOT_AUX, self._q8_zero, self.device)
            from .plan import SLOT_AUX
            theta, slot = self.d_wire, SLOT_AUX
        q = self._q8_buffers(n)
        S, nb = q["S"], self.tree.n_buckets

        def pack(b):
            self.k.delta_q8(self.tree, b, slot, theta, self._q8_region(q, b))

        def a2a(b):
            nch, m, _, _ = q["plan"][b]
            return dist.all_to_all_single(q["recv"][b % 2][:n * m * S], self._q8_region(q, b),
                                          group=group, async_op=True)

        works, pend = [None] * nb, [None] * nb
        pack(0)
        pend[0] = a2a(0)
        for b in range(nb):
            if b + 1 < nb:
                pack(b + 1)
                pend[b + 1] = a2a(b + 1)
            pend[b].wait()
            nch, m, _, rb = q["plan"][b]
            red = q["red"][rb * S:(rb + m) * S]
            self.k.q8_reduce(q["recv"][b % 2][:n * m * S], n, m, n, red)
            works[b] = dist.all_gather_into_tensor(self._q8_region(q, b), red, group=group,
                                                   async_op=True)
        self._works = works
        self._xmode, self._div = "q8", 1
        if not self.fused:
            self._decode_q8()

    def _decode_q8(self) -> None:
        """The averaged slots -> .grad's fp32 arena: g = q · s per chunk (the product
        dl_unpack_sgd_q8 forms in registers), chunk j of a tensor covering its elements
        [4096·j, 4096·(j+1))."""
        self._join()
        self._xmode = None
        q = self._q8
        S, C = q["S"], S_CHUNK
        for b in range(self.tree.n_buckets):
            nch, m, base, _ = q["plan"][b]
            sl = q["slots"][base * S:(base + nch) * S].view(nch, S)
            g = sl[:, S - C:].contiguous().view(torch.int8).float() * \
                sl[:, :4].contiguous().view(torch.float32)
            r = 0
            for i in q["segs"][b]:
                n_i = self.numels[i]
                k = -(-n_i // C)
                self.d_wire[self.offs[i]:self.offs[i] + n_i].copy_(g[r:r + k].reshape(-1)[:n_i])
                r += k

    def _q8_sgd(self, mom, lr, momentum, nesterov, first, target) -> None:
        """Per bucket: wait for its all_gather, then dl_unpack_sgd_q8 (g = q·s, Nesterov SGD
        on θ and the momentum, the inner params written when the last delta's are bound)."""
        works, self._works = self._works, None
        q = self._q8
        write = target is not None
        if write:
            self.k.bind(self.tree, SLOT_INNER, target[0], self.device, key=tuple(target[1]))
        for b in range(self.tree.n_buckets):
            if works is not None:
                works[b].wait()
            self.k.unpack_sgd_q8(self.tree, b, self._q8_region(q, b), self.d_theta, mom, lr,
                                 momentum, nesterov, first, SLOT_INNER if write else -1)
        # the slots keep the average for a later .grad read (_xmode stays "q8")

    def _launch_reductions(self, pack, view, group) -> None:
        """Fused N > 1: pack(b) then an asynchronous all_reduce(SUM) of bucket b, for every
        bucket, none waited for here (OuterSGD.step waits bucket by bucket, anything that reads
        or rewrites the wire first joins them all)."""
        works = []
        for b in range(self.tree.n_buckets):
            if pack is not None:
                pack(b)
            works.append(dist.all_reduce(view(b), op=dist.ReduceOp.SUM, group=group,
                                         async_op=True))
        self._works = works

    def sgd_step(self, lr: float, momentum: float, nesterov: bool,
                 host_bufs: Optional[List[Optional[torch.Tensor]]]) -> List[Optional[torch.Tensor]]:
        """torch.optim.SGD._single_tensor_sgd over the whole tree; returns the momentum
        buffers (views of d_mom) for the optimizer state."""
        tver = self._theta_version()
        delta = self._take_delta(tver) if self._delta is not None else None
        tver = self._relay_theta(tver)
        if delta is None:
            self._relay_grads(zero_fill_missing=False)
        first = True
        bufs: List[Optional[torch.Tensor]] = [None] * len(self.params)
        if momentum != 0:
            if self.d_mom is None:
                self.d_mom = torch.zeros_like(self.d_theta)
                plain = self._make_views(self.d_mom)
                self._views["mom_plain"] = plain
                self._views["mom"] = [self._momentum_buffer(v) for v in plain]
                self._ptrs["mom"] = [v.data_ptr() for v in plain]
            bufs = self._views["mom"]
            src = self._mom_src
            if not (src is not None and len(host_bufs) == len(src)
                    and all(map(is_, host_bufs, src))):
                have = [b is not None for b in host_bufs]
                if any(have) and not all(have):
                    raise RuntimeError("momentum buffers exist for some outer parameters only")
                first = not any(have)
                if not first:
                    copied = 0
                    with torch.no_grad():
                        for b, v, e in zip(host_bufs, self._views["mom_plain"],
                                           self._ptrs["mom"]):
                            if _DATA_PTR(b) != e:
                                v.copy_(b)  # e.g. a state_dict loaded into the optimizer
                                copied += 1
                    if copied == len(host_bufs):
                        self._mom_stale = False  # every slice written from the caller's
            else:
                first = False  # the buffers this mirror returned last step
            self._mom_src = bufs
        mom = self.d_mom if momentum != 0 else None
        sharded = delta is None and self._xmode in ("sharded", "a2a")
        q8 = delta is None and self._xmode == "q8"
        if (mom is not None and self._mom_stale and not first
                and not (sharded and self._mom_shard == (self._xgroup, self._xn, self._xrank))):
            self.gather_momentum()  # a whole-tree update needs every slice of the momentum
        # the inner params of the last compute_pseudo_gradient take θ_new in the same pass
        # (fused mode). The record of that write keeps their addresses and versions from then:
        # if they moved or were written since, sync_inner_model sees it and scatters again
        target, self._target = self._target, None
        write = target is not None
        if delta is not None:  # one peer: the delta never leaves registers
            self.k.delta_pack_sgd(self.tree, ALL, SLOT_INNER, self.d_theta, self.d_wire, mom,
                                  lr, momentum, nesterov, first)
            self._mom_stale = False
        elif sharded:  # N > 1, sharded exchange: this rank's 1/n, then all_gather(θ)
            self._sharded_sgd(mom, lr, momentum, nesterov, first, target)
        elif q8:  # N > 1, int8 wire: the averaged slots of each bucket, SGD fused in
            self._mom_stale = False
            self._q8_sgd(mom, lr, momentum, nesterov, first, target)
        else:
            self._mom_stale = False
            if write:
                self.k.bind(self.tree, SLOT_INNER, target[0], self.device, key=tuple(target[1]))
            # a pending /n stays pending: the wire keeps the Σ, .grad settles it when read
            wire = self.d_wire16 if self._sum16 else self.d_wire
            slot = SLOT_INNER if write else -1
            works, self._works = self._works, None
            if works is None:
                self.k.unpack_sgd(self.tree, ALL, wire, self._div, self.d_theta, mom, lr,
                                  momentum, nesterov, first, slot)
            else:  # bucket b's SGD waits for bucket b's collective only
                for b, w in enumerate(works):
                    w.wait()
                    self.k.unpack_sgd(self.tree, b, wire, self._div, self.d_theta, mom, lr,
                                      momentum, nesterov, first, slot)
        self._synced = (target + (tver,)) if write else None
        return bufs

    def copy_to_inner(self, inner_params: Sequence[torch.Tensor]) -> None:
        """inner = outer (src/utils.py:223-226): verified no-op after a fused step that
        already wrote these inner params, else scattered from HBM."""
        inner = list(inner_params)
        self._target = None
        if self._delta is not None:  # the inner params are about to change: use them first
            self._take_delta()
            self.k.delta_pack(self.tree, ALL, SLOT_INNER, self.d_theta, self.d_wire)
        tver = self._relay_theta()
        s = self._synced
        iptrs = _ptrs(inner)
        if (s is not None and len(s[0]) == len(inner)
                and all(map(is_, s[0], inner))
                and iptrs == s[1] and _vers(inner) == s[2] and tver == s[3]):
            return
        self.k.bind(self.tree, SLOT_INNER, inner, self.device, key=tuple(iptrs))
        self.k.scatter(self.tree, ALL, self.d_theta, SLOT_INNER)
        if self.fused:
            self._synced = (inner, iptrs, _vers(inner), tver)

    def close(self) -> None:
        self._join()
        self.tree.close()


# ---- the reference's host placement, kept lazily (write_back="lazy", the default) ----------------
_NO_TF = torch._C.DisableTorchFunctionSubclass


def _host_args(args, kwargs) -> list:
    """The lazy host objects among a torch function's arguments, as (tensor, mirror, arena),
    each arena made current first."""
    found, seen = [], set()

    def visit(x):
        if isinstance(x, (HostParameter, HostTensor)):
            d = x.__dict__
            r = d.get("_dl_mirror")
            m = r() if r is not None else None
            if m is not None:
                arena = d["_dl_arena"]
                found.append((x, m, arena))
                if (id(m), arena) not in seen:
                    seen.add((id(m), arena))
                    m.to_host(arena)
        elif isinstance(x, (list, tuple)):
            for y in x:
                visit(y)

    visit(args)
    if kwargs:
        visit(tuple(kwargs.values()))
    return found


def _host_function(func, args, kwargs):
    """HostParameter / HostTensor __torch_function__: metadata queries pass through; anything
    else first brings the arenas of its lazy host arguments up to date from HBM, runs on the
    plain tensors, and reports every argument it wrote (its version counter moved) to its
    mirror, which uploads that arena before the next outer-step call."""
    kwargs = kwargs or {}
    if func in _META:
        with _NO_TF():
            return func(*args, **kwargs)
    found = _host_args(args, kwargs)
    with _NO_TF():
        vers = [x._version for x, _, _ in found]
        out = func(*args, **kwargs)
        for (x, m, arena), v in zip(found, vers):
            if x._version != v:
                m.host_written(arena)
    return out


def _to_host_of(args, kwargs) -> None:
    _host_args(args, kwargs)


class HostTensor(torch.Tensor):
    """`.grad` or `outer_optimizer.state[p]["momentum_buffer"]` of the host-placed outer model
    under write_back="lazy": a CPU tensor (a view of a pinned host arena) whose values are
    copied from HBM the first time anything reads them after the device changed them -- any
    torch function other than a metadata query, pickling, deep copy -- and whose writes are
    uploaded before the next outer-step call. Results of operations are plain tensors."""

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        return _host_function(func, args, kwargs)

    def _plain(self) -> torch.Tensor:
        _to_host_of((self,), None)
        with _NO_TF():
            return self.detach().clone()

    def __deepcopy__(self, memo):
        if id(self) in memo:
            return memo[id(self)]
        out = self._plain()
        memo[id(self)] = out
        return out

    def __reduce_ex__(self, proto):
        return self._plain().__reduce_ex__(proto)


class HostParameter(torch.nn.Parameter):
    """A parameter of the host-placed outer model (src/utils.py:216: a CPU tensor) under
    write_back="lazy". The outer step runs on its HBM twin (mirror.LazyHostOuterMirror); this
    object -- the same Parameter object get_outer_model returned, its class switched in place,
    so the optimizer's references stay valid -- holds a view of a pinned host arena that is
    brought up to date from HBM when it is read: any torch function on it other than a metadata
    query, `.data`, `.grad`, pickling, deep copy. Writes (in place, through `.data`, assigning
    `.data` or `.grad`) are uploaded before the next outer-step call. Writes through a `.data`
    alias kept from earlier bypass every version counter: call invalidate() after them (as for
    every placement)."""

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        return _host_function(func, args, kwargs)

    def _m(self):
        r = self.__dict__.get("_dl_mirror")
        return r() if r is not None else None

    @property
    def data(self):
        m = self._m()
        if m is not None:
            m.to_host("theta")
        with _NO_TF():
            return _DATA.__get__(self)

    @data.setter
    def data(self, value):
        m = self._m()
        if m is not None:
            m.to_host("theta")
            m.theta_touched = True
        with _NO_TF():
            _DATA.__set__(self, value)

    @property
    def grad(self):
        m = self._m()
        if m is not None:
            m.to_host("grad")
        with _NO_TF():
            return _GRAD.__get__(self)

    @grad.setter
    def grad(self, value):
        m = self._m()
        if m is not None:
            m.to_host("grad")
            m.grads_touched = True
        with _NO_TF():
            _GRAD.__set__(self, value)

    @grad.deleter
    def grad(self):
        m = self._m()
        if m is not None:
            m.to_host("grad")
            m.grads_touched = True
        with _NO_TF():
            _GRAD.__delete__(self)

    def __reduce_ex__(self, proto):  # pickles as a plain Parameter of the current values,
        # over its own storage (a view would carry the whole pinned arena)
        return (torch._utils._rebuild_parameter,
                (self.data.clone(), self.requires_grad, OrderedDict()))

    def __deepcopy__(self, memo):
        if id(self) in memo:
            return memo[id(self)]
        out = torch.nn.Parameter(self.data.clone(), self.requires_grad)
        memo[id(self)] = out
        return out


_ARENAS = ("grad", "theta", "mom")


class LazyHostOuterMirror:
    """The reference's host-resident outer model (get_outer_model -> deepcopy(inner).to("cpu"),
    src/utils.py:213-216) stepped at device speed: write_back="lazy", the default placement.

    The outer model's parameters stay the CPU Parameters the reference returns, their .grad
    and the optimizer's momentum buffers CPU tensors -- views of three pinned host arenas
    (θ, grad, momentum) laid out like the device's. The outer step itself runs on an HBM twin
    of the outer model (a DeviceOuterMirror: the fused one-pass kernel at one peer, the RCCL
    exchange at N > 1 -- replicated by default, so .grad and the momentum stay local on every
    rank -- no PCIe traffic per step). A host arena is copied from HBM (one
    DMA) only when something reads one of its tensors after the device changed it
    (HostParameter / HostTensor intercept every read), and host-side writes are uploaded before
    the next outer-step call (detected by the arenas' version counters and by assignments of
    `.data` / `.grad`). So every value a caller observes is the reference's, on the CPU,
    while an outer step that nobody observes costs what the device placement costs. Under an
    opted-in sharded exchange at N > 1, reading `.grad` or the momentum is a collective over
    the DP group, as for the device placement (collective_read guards it)."""

    def __init__(self, outer_model: torch.nn.Module, device: torch.device, kernels=None,
                 bucket_cap_elems: int = DEFAULT_BUCKET_CAP_ELEMS, fused: bool = True,
                 wire: str = "f32", exchange: str = DEFAULT_EXCHANGE["host"]):
        self.device = torch.device(device)
        params = module_params(outer_model)
        if not params:
            raise ValueError("outer model has no parameters")
        _check_host_params(params)
        with _NO_TF():
            twin = torch.nn.Module()
            twin.ps = torch.nn.ParameterList([
                torch.nn.Parameter(_DATA.__get__(p).to(self.device), p.requires_grad)
                for p in params])
        self.dev = DeviceOuterMirror(twin, self.device, kernels, bucket_cap_elems, fused, wire,
                                     exchange)
        self._twin = twin
        self.fused, self.wire, self.exchange = fused, wire, exchange
        self.tree, self.offs, self.numels = self.dev.tree, self.dev.offs, self.dev.numels
        # host arenas, pageable by default: pinned and pageable measured the same for the step
        # (profiles/r04_placement_ab_order.txt) -- nothing crosses PCIe unless the host reads --
        # and pageable pages of the .grad / momentum arenas are not resident until a read
        # fills them (4 B/param resident per rank instead of 12 pinned).
        # DILOCO_HOST_PIN=1 pins them (one async DMA per read)
        from .utils import env_flag

        self._pin = self.device.type == "cuda" and env_flag("DILOCO_HOST_PIN", False)
        self.h = {"theta": self._arena(zero=True), "grad": self._arena(), "mom": None}
        ref = weakref.ref(self)
        with _NO_TF(), torch.no_grad():
            self._theta_views = self._views(self.h["theta"])
            for p, v in zip(params, self._theta_views):
                v.copy_(_DATA.__get__(p))
                _DATA.__set__(p, v)
                p.__class__ = HostParameter  # same object: the optimizer's references stay
                p.__dict__["_dl_mirror"] = ref
                p.__dict__["_dl_arena"] = "theta"
            self._grad_views = [self._host_tensor(v, "grad") for v in self._views(self.h["grad"])]
        self.params = params
        self._mom_views: Optional[List[torch.Tensor]] = None
        self._ver = {"theta": self.h["theta"]._version, "grad": self.h["grad"]._version,
                     "mom": None}
        self._dirty: set = set()
        self._written: set = set()  # arenas written on the host since the last upload
        self._grads_set = False  # the API .grads are the grad arena's views
        self.theta_touched = self.grads_touched = False

    def _arena(self, zero: bool = False) -> torch.Tensor:
        """A host arena of the packed layout. Not zero: left unwritten (pageable pages stay
        unresident until a read from HBM fills the arena) except the alignment gaps between
        segments, zeroed so that an upload of the arena never carries garbage into HBM."""
        z = dict(dtype=torch.float32, pin_memory=self._pin)
        if zero:
            return torch.zeros(self.tree.total, **z)
        a = torch.empty(self.tree.total, **z)
        ends = [o + n for o, n in zip(self.offs, self.numels)]
        for e, o in zip(ends, self.offs[1:] + [self.tree.total]):
            if o > e:
                a[e:o].zero_()
        return a

    def _views(self, arena: torch.Tensor) -> List[torch.Tensor]:
        return [arena[o:o + n].view(p.shape)
                for o, n, p in zip(self.offs, self.numels, self.dev.params)]

    def _host_tensor(self, view: torch.Tensor, arena: str) -> "HostTensor":
        t = view.as_subclass(HostTensor)
        t.__dict__["_dl_mirror"] = weakref.ref(self)
        t.__dict__["_dl_arena"] = arena
        return t

    @property
    def pending(self) -> bool:
        return bool(self._dirty)

    # ---- coherence ------------------------------------------------------------------------
    def _sync_stream(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()

    def to_host(self, arena: str) -> None:
        """The host arena equals the device state (one DMA if the device changed it)."""
        if arena not in self._dirty:
            return
        with _NO_TF():
            if arena == "grad":
                self.dev.settle_grads()  # the pending delta / Σ / sharded gathers, then /n
            elif arena == "mom":
                self.dev.gather_momentum()
            src = {"theta": self.dev.d_theta, "grad": self.dev.d_wire, "mom": self.dev.d_mom}[arena]
            h = self.h[arena]
            h.copy_(src, non_blocking=self._pin)
            self._sync_stream()
            self._dirty.discard(arena)
            self._ver[arena] = h._version

    def flush(self) -> None:
        for a in _ARENAS:
            self.to_host(a)

    def invalidate(self) -> None:
        """After writes the hooks cannot see (through a `.data` alias kept from earlier):
        re-upload every host arena at the next call."""
        self.dev.invalidate()
        self.theta_touched = self.grads_touched = True
        self._written |= {"theta", "grad", "mom"}

    def host_written(self, arena: str) -> None:
        self._written.add(arena)

    def _changed(self, arena: str, what: str) -> bool:
        h = self.h[arena]
        if h is None:
            return False
        if arena in self._written:
            self._written.discard(arena)
        elif h._version == self._ver[arena]:
            return False
        if arena in self._dirty:
            raise RuntimeError(
                f"the host {what} were written while their device copy was newer (a write that "
                "bypassed the outer model's tensors); call flush_outer_model() first")
        return True

    def _push(self) -> None:
        """Host writes since the last call -> HBM (before any outer-step work)."""
        dev = self.dev
        with _NO_TF(), torch.no_grad():
            if self.theta_touched:  # a parameter's .data was assigned: back into the arena
                self.theta_touched = False
                for p, v in zip(self.params, self._theta_views):
                    cur = _DATA.__get__(p)
                    if cur.data_ptr() != v.data_ptr():
                        v.copy_(cur)
                        _DATA.__set__(p, v)
            if self._changed("theta", "outer parameters"):
                dev.d_theta.copy_(self.h["theta"], non_blocking=self._pin)
                self._ver["theta"] = self.h["theta"]._version
            if self.grads_touched:  # a .grad was assigned: values into the arena, or None
                self.grads_touched = False
                self._grads_set = False
                for i, (p, tp) in enumerate(zip(self.params, dev.params)):
                    g, v = _GRAD.__get__(p), self._grad_views[i]
                    if g is None:
                        _GRAD.__set__(tp, None)
                        dev.grads_touched = True
                        continue
                    if g is not v:
                        if g.data_ptr() != v.data_ptr():
                            v.copy_(g)
                        _GRAD.__set__(p, v)
                    if _GRAD.__get__(tp) is None:
                        _GRAD.__set__(tp, dev._views["wire"][i])
                        dev.grads_touched = True
            if self._changed("grad", "outer gradients"):
                dev.d_wire.copy_(self.h["grad"], non_blocking=self._pin)
                self._ver["grad"] = self.h["grad"]._version
                dev.grads_touched = True

    def _set_api_grads(self) -> None:
        if self._grads_set:
            return
        with _NO_TF():
            for p, v in zip(self.params, self._grad_views):
                if _GRAD.__get__(p) is not v:
                    _GRAD.__set__(p, v)
        self._grads_set = True

    # ---- the four reference operations --------------------------------------------------
    def pseudo_gradient(self, inner_params: Sequence[torch.Tensor]) -> None:
        self._push()
        self.dev.pseudo_gradient(inner_params)
        self._set_api_grads()
        self._dirty.add("grad")

    def all_reduce(self, group, num_peers: int, ordered: bool = False) -> None:
        self._push()
        self.dev.all_reduce(group, num_peers, ordered)
        self._set_api_grads()
        self._dirty.add("grad")

    def sgd_step(self, lr: float, momentum: float, nesterov: bool, host_bufs):
        self._push()
        dev = self.dev
        dev_bufs = host_bufs
        if momentum != 0 and self._mom_views is not None and len(host_bufs) == len(
                self._mom_views) and all(map(is_, host_bufs, self._mom_views)):
            if self._changed("mom", "momentum buffers"):  # written on the host: upload
                with _NO_TF():
                    dev.d_mom.copy_(self.h["mom"], non_blocking=self._pin)
                self._ver["mom"] = self.h["mom"]._version
                dev._mom_stale = False
            dev_bufs = dev._views["mom"]  # the device's own buffers: not the first step
        dev.sgd_step(lr, momentum, nesterov, dev_bufs)
        self._dirty.add("theta")
        if momentum == 0:
            return [None] * len(self.params)
        if self._mom_views is None:
            self.h["mom"] = self._arena()
            self._mom_views = [self._host_tensor(v, "mom") for v in self._views(self.h["mom"])]
            self._ver["mom"] = self.h["mom"]._version
        self._dirty.add("mom")
        return self._mom_views

    def copy_to_inner(self, inner_params: Sequence[torch.Tensor]) -> None:
        self._push()
        self.dev.copy_to_inner(inner_params)

    def close(self) -> None:
        self.flush()
        self.dev.close()

    def __deepcopy__(self, memo):  # a copied outer model starts without a mirror
        return None

    def __reduce_ex__(self, proto):
        return (_none, ())
