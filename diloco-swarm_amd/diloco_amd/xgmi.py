"""Peer mapping for the direct exchange (dl_xgmi_reduce_sgd): every rank's packed wire and θ
buffers, IPC-mapped into every rank of one node's DP group.

`PeerMap(tensors, group, device)` is collective. Each rank exports its tensors (the handle of
the allocation holding each one + its byte offset), the group exchanges them with
all_gather_object together with (hostname, device ordinal), and every rank checks that all
peers share its host and that it can access every peer's device. The verdict is agreed by all
ranks before anything is opened, so either every rank maps every peer or no rank maps any
(`PeerMap.ok`, `.reason`); a half-mapped group cannot occur.
"""
from __future__ import annotations

import ctypes
import socket
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _lib


def _export(t: torch.Tensor):
    h = ctypes.create_string_buffer(_lib.IPC_HANDLE_BYTES)
    off = ctypes.c_int64()
    _lib.call("dl_ipc_handle", t.data_ptr(), h, ctypes.byref(off))
    return h.raw, off.value


class PeerMap:
    def __init__(self, tensors: Dict[str, torch.Tensor], group: Optional[dist.ProcessGroup],
                 device: torch.device):
        self.group = group
        self.n = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.device = torch.device(device)
        self.names = list(tensors)
        self._opened: List[int] = []
        self.ptrs: Dict[str, List[int]] = {k: [0] * self.n for k in self.names}
        self.ok, self.reason = True, ""
        for k, t in tensors.items():
            self.ptrs[k][self.rank] = t.data_ptr()
        if self.n == 1:
            return
        if self.n > 8:
            self.ok, self.reason = False, f"{self.n} peers (the kernel takes up to 8)"
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        mine = {"host": socket.gethostname(), "device": dev,
                "sizes": {k: t.numel() for k, t in tensors.items()}, "bufs": {}}
        try:
            mine["bufs"] = {k: _export(t) for k, t in tensors.items()}
        except _lib.DilocoHipError as e:
            self.ok, self.reason = False, f"export failed: {e}"
        everyone: List[dict] = [None] * self.n
        dist.all_gather_object(everyone, mine, group=group)
        if self.ok:
            try:
                self.ok, self.reason = self._check(everyone, mine)
            except _lib.DilocoHipError as e:  # a failed query is a "no" vote, never a raise
                self.ok, self.reason = False, f"peer query failed: {e}"
        votes: List[tuple] = [None] * self.n
        dist.all_gather_object(votes, (self.ok, self.reason), group=group)
        bad = [f"rank {q}: {r}" for q, (o, r) in enumerate(votes) if not o]
        if bad:
            self.ok, self.reason = False, "; ".join(bad)
            return
        err = ""
        try:
            for d in sorted({info["device"] for info in everyone} - {dev}):
                _lib.call("dl_enable_peer_access", int(d))
            for q, info in enumerate(everyone):
                if q == self.rank:
                    continue
                # tensors of one peer that live in the same allocation (e.g. θ and the wire
                # from one caching-allocator segment) share its IPC handle: open it once
                seen: Dict[bytes, int] = {}
                for k in self.names:
                    handle, off = info["bufs"][k]
                    if handle not in seen:
                        base = ctypes.c_void_p()
                        _lib.call("dl_ipc_open",
                                  ctypes.create_string_buffer(handle, len(handle)),
                                  ctypes.byref(base))
                        self._opened.append(base.value)
                        seen[handle] = base.value
                    self.ptrs[k][q] = seen[handle] + off
        except _lib.DilocoHipError as e:
            err = f"opening a peer's buffer failed: {e}"
        # second agreement: every rank mapped every peer, or every rank gives up together
        votes = [None] * self.n
        dist.all_gather_object(votes, err, group=group)
        bad = [f"rank {q}: {r}" for q, r in enumerate(votes) if r]
        if bad:
            self.close()
            self.ok, self.reason = False, "; ".join(bad)

    def _check(self, everyone, mine):
        for q, info in enumerate(everyone):
            if info["host"] != mine["host"]:
                return False, f"rank {q} is on {info['host']}, not {mine['host']}"
            if info["sizes"] != mine["sizes"]:
                return False, f"rank {q} has buffers {info['sizes']}, this rank {mine['sizes']}"
            if not info["bufs"]:
                return False, f"rank {q} exported nothing"
            can = ctypes.c_int32()
            _lib.call("dl_can_access_peer", mine["device"], info["device"], ctypes.byref(can))
            if not can.value:
                return False, f"device {mine['device']} cannot access device {info['device']}"
        return True, ""

    def table(self, name: str):
        return np.asarray(self.ptrs[name], dtype=np.uint64)

    def close(self) -> None:
        for b in self._opened:
            _lib.call("dl_ipc_close", ctypes.c_void_p(b))
        self._opened = []
