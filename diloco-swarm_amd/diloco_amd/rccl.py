"""RCCL through the C-ABI (dl_allreduce / dl_reduce_scatter / dl_all_gather).

The engines use torch.distributed (backend "nccl" = RCCL) for their collectives; this module
is the same exchange driven through libdiloco_hip.so, for hosts that hold an ncclComm_t of
their own or want the library's C entry points only. Two ways to get a communicator:

    Comm.from_process_group(group, device)   torch's ProcessGroupNCCL communicator (its RCCL)
    Comm.create(nranks, rank, uid)           a new one; uid = Comm.unique_id() on one rank,
                                             shared with the others by any means

Collectives are enqueued on the current HIP stream of the tensor's device.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch
import torch.distributed as dist

from . import _lib

UNIQUE_ID_BYTES = 128
_DT = {torch.float32: _lib.DL_F32, torch.bfloat16: _lib.DL_BF16, torch.float16: _lib.DL_F16,
       torch.uint8: _lib.DL_U8, torch.int8: _lib.DL_U8}


def _dtype(t: torch.Tensor) -> int:
    if t.dtype not in _DT:
        raise TypeError(f"{t.dtype}: the RCCL entry points take float32/bfloat16/float16/bytes")
    return _DT[t.dtype]  # int8 / uint8: raw bytes (int8 wire slots)


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def torch_rccl_path() -> Optional[str]:
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else None


def load(path: Optional[str] = None) -> None:
    """Select the RCCL library (default: the one already in the process, i.e. torch's)."""
    _lib.call("dl_rccl_load", path.encode() if path else None)


def version() -> int:
    v = ctypes.c_int32()
    _lib.call("dl_rccl_version", ctypes.byref(v))
    return v.value


class group:
    """RCCL group (dl_group_start / dl_group_end): the point-to-point calls inside progress
    together -- required for a send and its receive on one rank."""

    def __enter__(self):
        _lib.call("dl_group_start")
        return self

    def __exit__(self, *exc):
        _lib.call("dl_group_end")
        return False


class Comm:
    def __init__(self, handle: int, nranks: int, owned: bool):
        self.handle, self.nranks, self.owned = ctypes.c_void_p(handle), nranks, owned

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
        _lib.call("dl_comm_unique_id", buf)
        return buf.raw

    @classmethod
    def create(cls, nranks: int, rank: int, uid: bytes) -> "Comm":
        if len(uid) != UNIQUE_ID_BYTES:
            raise ValueError("unique id must be 128 bytes")
        h = ctypes.c_void_p()
        _lib.call("dl_comm_init", ctypes.byref(h), int(nranks),
                  ctypes.create_string_buffer(uid, UNIQUE_ID_BYTES), int(rank))
        return cls(h.value, nranks, owned=True)

    @classmethod
    def from_process_group(cls, group: Optional[dist.ProcessGroup],
                           device: torch.device) -> "Comm":
        """The communicator behind a torch `nccl` process group (not owned: torch frees it).
        One collective is issued first so that torch has created it."""
        group = group or dist.group.WORLD
        backend = group._get_backend(torch.device(device))
        if not hasattr(backend, "_comm_ptr"):
            raise TypeError(f"{type(backend).__name__} has no RCCL communicator")
        probe = torch.zeros(1, device=device)
        dist.all_reduce(probe, group=group)
        ptr = backend._comm_ptr()
        if not ptr:
            raise RuntimeError("the process group has no communicator on this device")
        load(torch_rccl_path())  # use the communicator with the RCCL that created it
        return cls(int(ptr), dist.get_world_size(group), owned=False)

    def all_reduce(self, t: torch.Tensor) -> None:
        """In-place SUM over the communicator (src/comm.py:122)."""
        _lib.call("dl_allreduce", t.data_ptr(), t.numel(), _dtype(t), self.handle, _stream(t))

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        if inp.numel() != out.numel() * self.nranks or inp.dtype != out.dtype:
            raise ValueError("reduce_scatter: input must be nranks x output, same dtype")
        _lib.call("dl_reduce_scatter", inp.data_ptr(), out.data_ptr(), out.numel(), _dtype(out),
                  self.handle, _stream(out))

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        if out.numel() != inp.numel() * self.nranks or inp.dtype != out.dtype:
            raise ValueError("all_gather: output must be nranks x input, same dtype")
        _lib.call("dl_all_gather", inp.data_ptr(), out.data_ptr(), inp.numel(), _dtype(inp),
                  self.handle, _stream(inp))

    def send(self, t: torch.Tensor, peer: int) -> None:
        """Point-to-point send of t to `peer` (src/comm.py:38 on the device, no host copy)."""
        _lib.call("dl_send", t.data_ptr(), t.numel(), _dtype(t), int(peer), self.handle,
                  _stream(t))

    def recv(self, t: torch.Tensor, peer: int) -> None:
        """Point-to-point receive into t from `peer` (src/comm.py:67 after the header)."""
        _lib.call("dl_recv", t.data_ptr(), t.numel(), _dtype(t), int(peer), self.handle,
                  _stream(t))

    def close(self) -> None:
        if self.owned and self.handle:
            _lib.call("dl_comm_destroy", self.handle)
        self.handle = ctypes.c_void_p()
