"""Pipeline point-to-point on the device: src/comm.py:16-69 without the host
bounce.

The reference's threads frame an activation with the Serializer on its device, copy it to the
host (`tensor.to("cpu")`, src/comm.py:38) and `dist.send` it over a gloo group; the receiver
posts an ANY-SOURCE `dist.recv` (src/comm.py:66) because SWARM's routing is stochastic -- the
sender picks a random rank of the next stage (src/comm.py:91). RCCL has no any-source
receive, so the device transport splits each message in two:

    header   8 B int64 over the reference's own gloo group, any-source: tells the receiver
             which rank sends next (the `src` the reference gets back from dist.recv)
    payload  the (2, *shape) fp32 frame built on the GPU by dl_serialize, sent with
             dist.send/recv over a DATA group: RCCL (xGMI) in production

A receiver handles headers in arrival order and posts the matching payload receive, so every
posted send meets its receive; forward and backward traffic of a stage boundary use separate
data groups (separate communicators and streams), so a rank's forward send never waits behind
its backward receive. Queue protocol, shapes, metadata and the (src, tensor, metadata) tuples
are the reference's.

Data groups with backend "gloo" stage the frame through host memory; that mode exists so the
threads can be exercised with several ranks on one GPU (RCCL refuses two ranks on one device).
"""
from __future__ import annotations

import os
import threading
import time
from queue import Queue
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from .serializer import Metadata, Serializer


def p2p_backend() -> str:
    """Payload backend of the device transport, read when the groups are made:
    DILOCO_P2P_BACKEND, "nccl" (RCCL) by default or "gloo" (host-staged, tests)."""
    return os.environ.get("DILOCO_P2P_BACKEND", "nccl")


def _staged(group) -> bool:
    return dist.get_backend(group) == "gloo"


class DeviceSendThread:
    """SendThread (src/comm.py:16-38) with device framing and a header/payload split."""

    TIMEOUT = 1e-4

    def __init__(self, shape: Tuple[int, ...], group, data_group, device: torch.device,
                 tag: int = 0, serialize: bool = True, start: bool = True, serializer=None,
                 **kwargs):
        self.group, self.data_group, self.tag, self.serialize = group, data_group, tag, serialize
        self.device = torch.device(device)
        self.logger = kwargs.get("logger")
        self.queue: Queue = Queue()
        self.shape = shape
        if serialize:
            self.serializer = serializer or Serializer(shape)
            self.shape = self.serializer.shape
        self.rank = dist.get_rank()
        self.error: Optional[BaseException] = None
        if start:
            threading.Thread(target=self._send_loop, daemon=True).start()

    def send(self, dst: int, tensor: torch.Tensor, metadata: Optional[Metadata]) -> None:
        from .comm import check_alive

        check_alive(self)
        self.queue.put((dst, tensor, metadata))

    def send_one(self, dst: int, tensor: torch.Tensor, metadata: Optional[Metadata]) -> None:
        frame = self.serializer.serialize(tensor, metadata) if self.serialize else tensor
        frame = frame.contiguous()
        dist.send(torch.tensor([self.rank], dtype=torch.int64), dst=dst, group=self.group,
                  tag=self.tag)
        if _staged(self.data_group):
            frame = frame.to("cpu")
        dist.send(frame, dst=dst, group=self.data_group, tag=self.tag)

    def _send_loop(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        while True:
            if self.queue.empty():
                time.sleep(self.TIMEOUT)
                continue
            dst, tensor, metadata = self.queue.get()
            try:
                self.send_one(dst, tensor, metadata)
            except BaseException as e:  # surfaced to the caller via .error, thread stops
                self.error = e
                raise


class DeviceRecvThread:
    """RecvThread (src/comm.py:40-69): any-source header, then the payload from that rank."""

    def __init__(self, shape: Tuple[int, ...], group, data_group, device: torch.device,
                 tag: int = 0, requires_grad: bool = True, dtype: torch.dtype = torch.float32,
                 serialize: bool = True, start: bool = True, serializer=None, **kwargs):
        self.group, self.data_group, self.tag = group, data_group, tag
        self.device = torch.device(device)
        self.requires_grad, self.dtype, self.serialize = requires_grad, dtype, serialize
        self.logger = kwargs.get("logger")
        self.queue: Queue = Queue()
        self.shape = shape
        if serialize:
            self.serializer = serializer or Serializer(shape)
            self.shape = self.serializer.shape
        self.error: Optional[BaseException] = None
        if start:
            threading.Thread(target=self._recv_loop, daemon=True).start()

    @property
    def can_receive(self) -> bool:
        return not self.queue.empty()

    def load(self, tensor: Optional[torch.Tensor], metadata: Optional[Metadata]) -> None:
        self.queue.put((-1, tensor, metadata))

    def receive(self):
        from .comm import receive_or_raise

        return receive_or_raise(self)

    def recv_one(self):
        hdr = torch.empty(1, dtype=torch.int64)
        src = dist.recv(hdr, group=self.group, tag=self.tag)
        if int(hdr.item()) != src:
            raise RuntimeError(f"p2p header from rank {src} names rank {int(hdr.item())}")
        if _staged(self.data_group):
            host = torch.empty(self.shape, dtype=self.dtype)
            dist.recv(host, src=src, group=self.data_group, tag=self.tag)
            buf = host.to(self.device)
        else:
            buf = torch.empty(self.shape, dtype=self.dtype, device=self.device)
            dist.recv(buf, src=src, group=self.data_group, tag=self.tag)
        if self.device.type == "cuda":
            # the consumer reads the tensor on its own stream: complete it here, in the thread
            torch.cuda.current_stream(self.device).synchronize()
        buf.requires_grad_(self.requires_grad)
        meta = None
        if self.serialize:
            buf, meta = self.serializer.deserialize(buf)
        return src, buf, meta

    def _recv_loop(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        while True:
            try:
                item = self.recv_one()
            except BaseException as e:
                from .comm import STOPPED

                self.error = e
                self.queue.put(STOPPED)  # a blocked receive() wakes up and raises
                raise
            self.queue.put(item)


def boundary_data_groups(world, backend: str = None) -> Dict[Tuple[int, int, str], object]:
    """One forward and one backward data group per stage boundary (s, s+1), over the same
    ranks as the reference's world.local_pg[(s, s+1)]. Collective: every rank calls it, in
    the same order (TrainingComm.__init__ runs on every rank)."""
    backend = backend or p2p_backend()
    groups = {}
    for s in range(world.num_stages - 1):
        ranks = sorted(world.stage2ranks[s] + world.stage2ranks[s + 1])
        for d in ("fwd", "bwd"):
            groups[(s, s + 1, d)] = dist.new_group(ranks, backend=backend)
    return groups
