"""The kernel backend of the outer-step engines: libdiloco_hip.so through its C-ABI.

Every engine (OuterSync, GradSync, HostOuterMirror) calls these methods and nothing else for
compute, so the orchestration above them (bucketing, pipelining, /n, optimizer state) is one
code path. `HipKernels` is the only backend the package ships; it launches on the current
HIP stream of the tensors' device and raises if the library or the GPU is missing.
"""
from __future__ import annotations

import ctypes

from typing import Optional, Sequence

import torch

from . import _lib
from .plan import DEFAULT_BUCKET_CAP_ELEMS, PackedTree

_DT = {torch.float32: _lib.DL_F32, torch.bfloat16: _lib.DL_BF16}


Q8_SLOT = _lib.Q8_SLOT_BYTES


def wire_code(dtype: torch.dtype) -> int:
    try:
        return _DT[dtype]
    except KeyError:
        raise TypeError(f"unsupported packed dtype {dtype} (float32 or bfloat16)") from None


def _s(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


class HipKernels:
    """Segment-walker kernels of libdiloco_hip.so (DESIGN.md "Kernels")."""

    name = "hip"

    def check_device(self, device: torch.device) -> None:
        if device.type != "cuda":
            raise ValueError(f"the HIP outer-step kernels need device tensors, got {device}")
        _lib.load()

    def tree(self, numels: Sequence[int], device: torch.device,
             cap_elems: int = DEFAULT_BUCKET_CAP_ELEMS,
             bucket_align: int = _lib.ALIGN_ELEMS) -> PackedTree:
        self.check_device(device)
        with torch.cuda.device(device):
            return PackedTree(numels, cap_elems, bucket_align)

    def bind(self, tree: PackedTree, slot: int, tensors: Sequence[torch.Tensor], device,
             key=None) -> None:
        """key: tuple of the tensors' addresses, if the caller computed it (skips a pass)."""
        if key is not None and tree._bound[slot] == key:
            return
        tree.bind(slot, tensors, torch.cuda.current_stream(device).cuda_stream, key)

    def delta_pack(self, tree, bucket, inner_slot, theta, wire) -> None:
        _lib.call("dl_delta_pack", tree.handle, bucket, inner_slot, theta.data_ptr(),
                  wire.data_ptr(), wire_code(wire.dtype), _s(theta))

    def unpack_sgd(self, tree, bucket, wire, divisor, theta, mom, lr, momentum, nesterov,
                   first, inner_slot) -> None:
        _lib.call("dl_unpack_sgd", tree.handle, bucket, wire.data_ptr(), wire_code(wire.dtype),
                  int(divisor), theta.data_ptr(), _ptr(mom), float(lr), float(momentum),
                  int(nesterov), int(first), int(inner_slot), _s(theta))

    def delta_sgd(self, tree, bucket, inner_slot, theta, mom, lr, momentum, nesterov,
                  first) -> None:
        _lib.call("dl_delta_sgd", tree.handle, bucket, inner_slot, theta.data_ptr(), _ptr(mom),
                  float(lr), float(momentum), int(nesterov), int(first), _s(theta))

    def delta_pack_sgd(self, tree, bucket, inner_slot, theta, wire, mom, lr, momentum, nesterov,
                       first) -> None:
        """One peer, one pass: delta + SGD + copy-back, the pseudo-gradient kept in `wire`."""
        _lib.call("dl_delta_pack_sgd", tree.handle, bucket, inner_slot, theta.data_ptr(),
                  wire.data_ptr(), wire_code(wire.dtype), _ptr(mom), float(lr), float(momentum),
                  int(nesterov), int(first), _s(theta))

    def pack_sgd_tiled(self, tree, bucket, inner_slot, theta, wire, mom, lr, momentum,
                       nesterov, first, tile_chunks) -> None:
        """One peer: delta_pack then unpack_sgd (divisor 1) tile by tile (Infinity-Cache
        blocking); the same results as the two whole-range launches."""
        _lib.call("dl_pack_sgd_tiled", tree.handle, bucket, inner_slot, theta.data_ptr(),
                  wire.data_ptr(), wire_code(wire.dtype), _ptr(mom), float(lr), float(momentum),
                  int(nesterov), int(first), int(tile_chunks), _s(theta))

    def shard_sgd(self, wire, divisor, theta, mom, lr, momentum, nesterov, first) -> None:
        """Flat 1/n shard after a reduce-scatter (wire, theta, mom: equal-length views)."""
        _lib.call("dl_shard_sgd", wire.data_ptr(), wire_code(wire.dtype), int(divisor),
                  theta.data_ptr(), _ptr(mom), theta.numel(), float(lr), float(momentum),
                  int(nesterov), int(first), _s(theta))

    def shard_reduce_sgd(self, slices, n_slices, theta, mom, lr, momentum, nesterov,
                         first) -> None:
        """Flat 1/n shard after an all_to_all: slices = n_slices equal slices (wire dtype) of
        theta's length; Σ in rank order, /n, SGD on theta / mom (equal-length views)."""
        _lib.call("dl_shard_reduce_sgd", slices.data_ptr(), wire_code(slices.dtype),
                  int(n_slices), theta.numel(), theta.data_ptr(), _ptr(mom), float(lr),
                  float(momentum), int(nesterov), int(first), _s(theta))

    def shard_reduce_avg(self, slices, n_slices, out) -> None:
        """out = Σ of the n_slices equal slices in rank order / n (fp32 out, out's length)."""
        _lib.call("dl_shard_reduce_avg", slices.data_ptr(), wire_code(slices.dtype),
                  int(n_slices), out.numel(), out.data_ptr(), _s(out))

    def xgmi_reduce_sgd(self, wires, thetas, n, rank, lo, length, mom, lr, momentum, nesterov,
                        first, device=None) -> None:
        """Direct exchange on this rank's shard (wires / thetas: uint64 arrays of the n peers'
        device addresses, IPC-mapped)."""
        p64 = ctypes.POINTER(ctypes.c_uint64)
        _lib.call("dl_xgmi_reduce_sgd", wires.ctypes.data_as(p64), thetas.ctypes.data_as(p64),
                  int(n), int(rank), int(lo), int(length), _ptr(mom), float(lr),
                  float(momentum), int(nesterov), int(first),
                  torch.cuda.current_stream(device).cuda_stream)

    def xgmi_delta_sgd(self, inners, thetas, n, rank, lo, length, mom, lr, momentum, nesterov,
                       first, device=None) -> None:
        """Direct exchange from the peers' packed inner arenas (no wire): g formed in-kernel."""
        p64 = ctypes.POINTER(ctypes.c_uint64)
        _lib.call("dl_xgmi_delta_sgd", inners.ctypes.data_as(p64), thetas.ctypes.data_as(p64),
                  int(n), int(rank), int(lo), int(length), _ptr(mom), float(lr),
                  float(momentum), int(nesterov), int(first),
                  torch.cuda.current_stream(device).cuda_stream)

    def sys_fence(self, device=None) -> None:
        """L2 write-back + invalidate on every XCD (cross-GPU ordering of IPC-shared buffers)."""
        _lib.call("dl_sys_fence", torch.cuda.current_stream(device).cuda_stream)

    # int8 wire codec (DL_Q8_SLOT_BYTES slots, one per chunk)
    def delta_q8(self, tree, bucket, inner_slot, theta, slots) -> None:
        _lib.call("dl_delta_q8", tree.handle, bucket, inner_slot, theta.data_ptr(),
                  slots.data_ptr(), _s(theta))

    def q8_reduce(self, recv, n_peers, n_slots, divisor, out) -> None:
        _lib.call("dl_q8_reduce", recv.data_ptr(), int(n_peers), int(n_slots), int(divisor),
                  out.data_ptr(), _s(out))

    def unpack_sgd_q8(self, tree, bucket, slots, theta, mom, lr, momentum, nesterov, first,
                      inner_slot) -> None:
        _lib.call("dl_unpack_sgd_q8", tree.handle, bucket, slots.data_ptr(), theta.data_ptr(),
                  _ptr(mom), float(lr), float(momentum), int(nesterov), int(first),
                  int(inner_slot), _s(theta))

    def unpack_avg(self, tree, bucket, wire, divisor, dst_slot, dst_packed=None) -> None:
        _lib.call("dl_unpack_avg", tree.handle, bucket, wire.data_ptr(), wire_code(wire.dtype),
                  int(divisor), int(dst_slot), _ptr(dst_packed), _s(wire))

    def gather(self, tree, bucket, src_slot, packed) -> None:
        _lib.call("dl_gather", tree.handle, bucket, src_slot, packed.data_ptr(),
                  wire_code(packed.dtype), _s(packed))

    def scatter(self, tree, bucket, packed, dst_slot) -> None:
        _lib.call("dl_scatter", tree.handle, bucket, packed.data_ptr(), dst_slot, _s(packed))


_DEFAULT = None


def default_kernels():
    """The backend the engines use: HipKernels unless a test installed its own checker
    backend with set_default_kernels (tests/oracle_kernels.py; never done by the package)."""
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = HipKernels()
    return _DEFAULT


def set_default_kernels(k) -> None:
    """Test hook: route the engines through `k` (None restores HipKernels)."""
    global _DEFAULT
    _DEFAULT = k
