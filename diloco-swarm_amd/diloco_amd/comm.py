"""Drop-in for src/comm.py: TrainingComm / InferenceComm with the DP sync on RCCL + HIP.

`TrainingComm(world, shape, logger)` keeps the reference's constructor and methods
(src/comm.py:71-149). What changes is `sync_gradients(model)` (src/comm.py:117-123):

  reference:  for p in model.parameters(): all_reduce(p.grad, SUM, gloo); p.grad /= n
  here:       one bucketed pass on the GPU over an RCCL group of the same ranks
              - host gradients (the DiLoCo outer model, src/train.py:265): the outer model's
                device mirror all-reduces its packed wire and divides in HBM
                (mirror.HostOuterMirror.all_reduce), then writes the averages back to .grad
              - device gradients (plain DP / SWARM, src/train.py:251): gradsync.GradSync
                (dl_gather -> RCCL -> dl_unpack_avg)
  Unchanged semantics: no-op for a single peer (no zero-fill either, src/comm.py:118-119),
  missing gradients become zeros, true division by the peer count, averages on every rank.

The pipeline point-to-point threads (src/comm.py:16-69) keep the reference's gloo transport
and queue protocol; their framing uses the HIP Serializer. They are outside the outer-step
path and carried for interface completeness.
"""
from __future__ import annotations

import os
import random
import threading
import time
from queue import Queue
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from .gradsync import GradSync
from .serializer import Metadata, Serializer


class ThreadStopped(RuntimeError):
    """A pipeline send/recv thread died; raised on the caller's side (the original exception
    is the __cause__) instead of leaving the caller blocked on a queue forever."""


STOPPED = object()  # queued by a dying receiver so that a blocked receive() wakes up


def check_alive(thread) -> None:
    if thread.error is not None:
        raise ThreadStopped(f"{type(thread).__name__} stopped: {thread.error!r}") from thread.error


def receive_or_raise(thread):
    """queue.get() that raises ThreadStopped once the receiving thread has died."""
    item = thread.queue.get()
    if item is STOPPED:
        thread.queue.put(STOPPED)  # every later receive() raises too
        check_alive(thread)
    return item


class SendThread:
    """Queue-fed sender (src/comm.py:16-38): optional framing, then dist.send from host memory.
    An exception in the thread (e.g. framing a tensor the Serializer rejects) stops it and is
    re-raised by the next send() call."""

    TIMEOUT = 1e-4

    def __init__(self, shape: Tuple[int, ...], group, tag: int = 0, serialize: bool = True,
                 start: bool = True, **kwargs):
        self.shape, self.group, self.tag, self.serialize = shape, group, tag, serialize
        self.logger = kwargs.get("logger")
        self.queue: Queue = Queue()
        self.error: Optional[BaseException] = None
        if serialize:
            self.serializer = Serializer(shape)
            self.shape = self.serializer.shape
        self.thread = threading.Thread(target=self._send_loop, daemon=True) if start else None
        if start:
            self.thread.start()

    def send(self, dst: int, tensor: torch.Tensor, metadata: Optional[Metadata]) -> None:
        check_alive(self)
        self.queue.put((dst, tensor, metadata))

    def _send_loop(self):
        try:
            while True:
                if self.queue.empty():
                    time.sleep(self.TIMEOUT)
                    continue
                dst, tensor, metadata = self.queue.get()
                if self.serialize:
                    tensor = self.serializer.serialize(tensor, metadata)
                dist.send(tensor.to("cpu"), dst=dst, group=self.group, tag=self.tag)
        except BaseException as e:
            self.error = e
            raise


class RecvThread:
    """Receiver thread (src/comm.py:40-69): dist.recv into host memory, optional unframing."""

    def __init__(self, shape: Tuple[int, ...], group, tag: int = 0, requires_grad: bool = True,
                 dtype: torch.dtype = torch.float32, serialize: bool = True, start: bool = True,
                 **kwargs):
        self.shape, self.group, self.tag = shape, group, tag
        self.requires_grad, self.dtype, self.serialize = requires_grad, dtype, serialize
        self.logger = kwargs.get("logger")
        self.queue: Queue = Queue()
        self.error: Optional[BaseException] = None
        if serialize:
            self.serializer = Serializer(shape)
            self.shape = self.serializer.shape
        self.thread = threading.Thread(target=self._recv_loop, daemon=True) if start else None
        if start:
            self.thread.start()

    @property
    def can_receive(self) -> bool:
        return not self.queue.empty()

    def load(self, tensor: Optional[torch.Tensor], metadata: Optional[Metadata]) -> None:
        self.queue.put((-1, tensor, metadata))

    def receive(self):
        return receive_or_raise(self)

    def _recv_loop(self):
        try:
            while True:
                buf = torch.empty(self.shape, dtype=self.dtype, requires_grad=self.requires_grad)
                src = dist.recv(buf, group=self.group, tag=self.tag)
                meta = None
                if self.serialize:
                    buf, meta = self.serializer.deserialize(buf)
                self.queue.put((src, buf, meta))
        except BaseException as e:
            self.error = e
            self.queue.put(STOPPED)  # can_receive turns true; receive() raises
            raise


# Collective backend of the DP group for device tensors: "nccl" = RCCL over xGMI (the
# product). "gloo" exists for multi-process tests that share one GPU (RCCL refuses two ranks
# on one device); the kernels are the same HIP kernels either way.
# None: DILOCO_DP_BACKEND as it is when the group is created ("nccl" if unset), like
# p2p.p2p_backend(); a value assigned here overrides it.
DP_BACKEND: Optional[str] = None


def dp_backend() -> str:
    return DP_BACKEND or os.environ.get("DILOCO_DP_BACKEND", "nccl")
# The DP average's exchange: "rccl" = RCCL's own order (the device-gradient GradSync's
# all_reduce; the outer model's exchange as get_outer_model chose it); "a2a" = all_to_all +
# rank-order average + all_gather (deterministic, bit-exact vs the oracle at any n) for the
# device gradients AND for the outer model's mirror (both placements)
DP_EXCHANGE = os.environ.get("DILOCO_DP_EXCHANGE", "rccl")


class DPSync:
    """The DP average of one stage's gradients (src/comm.py:117-123) on the GPU."""

    def __init__(self, world):
        self.world = world
        self._rccl_group = None
        self._grad_syncs: Dict[int, GradSync] = {}

    @property
    def num_peers(self) -> int:
        return len(self.world.stage2ranks[self.world.stage])

    def dp_group(self, device: torch.device):
        """The collective group of this stage's DP ranks on `device`'s transport.

        GPU: an RCCL group over world.stage2ranks[stage], created on first use by exactly the
        ranks that sync together (like the reference's curr_stage_group, src/world.py:39).
        CPU tensors use the reference's own gloo group."""
        if device.type != "cuda":
            return self.world.curr_stage_group
        if self._rccl_group is None:
            self._rccl_group = dist.new_group(self.world.stage2ranks[self.world.stage],
                                              backend=dp_backend(), use_local_synchronization=True)
        return self._rccl_group

    def sync_gradients(self, model: nn.Module) -> None:
        num_peers = self.num_peers
        if num_peers == 1:
            return
        m = getattr(model, "_diloco_mirror", None)  # utils._ATTR
        if m is not None:
            # an outer model whose steps run on the GPU (host placement after a device
            # compute_pseudo_gradient, or placement="device"): its packed mirror reduces
            # DILOCO_DP_EXCHANGE=a2a: the rank-order (deterministic) exchange here too
            m.all_reduce(self.dp_group(m.device), num_peers, ordered=DP_EXCHANGE == "a2a")
            return
        from .mirror import module_params
        from .utils import device_path

        params = module_params(model)
        if not params:
            return
        if not device_path(params[0]):
            # host tensors (the reference's --device cpu runs, or an outer model not yet
            # touched by a device step): the reference's loop on its gloo stage group
            group = self.world.curr_stage_group
            with torch.no_grad():
                for p in params:
                    if p.grad is None:
                        p.grad = torch.zeros_like(p)
                    dist.all_reduce(p.grad, op=dist.ReduceOp.SUM, group=group)
                    p.grad.div_(num_peers)
            return
        for p in params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        gs = self._grad_syncs.get(id(model))
        if gs is None or not gs.matches(params):
            gs = GradSync(params, self.dp_group(params[0].device), num_peers,
                          exchange=DP_EXCHANGE)
            self._grad_syncs[id(model)] = gs
        gs.sync()


_DP: Dict[int, DPSync] = {}


def dp_sync_gradients(world, model: nn.Module) -> None:
    """Module-level entry for a reference TrainingComm whose sync_gradients delegates here
    (INTEGRATION.md); one DPSync (and RCCL group) per World object."""
    d = _DP.get(id(world))
    if d is None or d.world is not world:
        d = _DP[id(world)] = DPSync(world)
    d.sync_gradients(model)


class TrainingComm:
    """src/comm.py:71-149. `transport` (default: DILOCO_P2P_TRANSPORT, else "host") selects the
    pipeline p2p threads: "host" = the reference's (frame, copy to host, gloo send/recv);
    "device" = p2p.DeviceSendThread / DeviceRecvThread (GPU framing, header over the same gloo
    group, payload over per-direction RCCL data groups) on `device`
    (default cuda:world.local_rank, the device src/train.py:368 trains on)."""

    def __init__(self, world, shape: Tuple[int, ...], logger, transport: Optional[str] = None,
                 device: Optional[torch.device] = None, serializer_factory=None):
        self.world, self.shape, self.logger = world, shape, logger
        kw = {"tag": 0, "serialize": True, "requires_grad": True, "logger": logger}
        self.transport = transport or os.environ.get("DILOCO_P2P_TRANSPORT", "host")
        if self.transport == "host":
            self.forward_send_thread = SendThread(shape, group=world.next_stage_group,
                                                  start=world.has_next_stage, **kw)
            self.backward_recv_thread = RecvThread(shape, group=world.next_stage_group,
                                                   start=world.has_next_stage, **kw)
            self.backward_send_thread = SendThread(shape, group=world.prev_stage_group,
                                                   start=world.has_prev_stage, **kw)
            self.forward_recv_thread = RecvThread(shape, group=world.prev_stage_group,
                                                  start=world.has_prev_stage, **kw)
        elif self.transport == "device":
            from .p2p import DeviceRecvThread, DeviceSendThread, boundary_data_groups

            if device is None:  # the reference's device: cuda:local_rank (src/utils.py:36-40,
                # src/train.py:368), not the current device, which it never sets
                device = torch.device("cuda", world.local_rank)
            if serializer_factory is not None:
                kw["serializer"] = serializer_factory(shape)
            dg = self.data_groups = boundary_data_groups(world)
            s = world.stage
            nxt = (s, s + 1)
            prv = (s - 1, s)
            self.forward_send_thread = DeviceSendThread(
                shape, world.next_stage_group, dg.get(nxt + ("fwd",)), device,
                start=world.has_next_stage, **kw)
            self.backward_recv_thread = DeviceRecvThread(
                shape, world.next_stage_group, dg.get(nxt + ("bwd",)), device,
                start=world.has_next_stage, **kw)
            self.backward_send_thread = DeviceSendThread(
                shape, world.prev_stage_group, dg.get(prv + ("bwd",)), device,
                start=world.has_prev_stage, **kw)
            self.forward_recv_thread = DeviceRecvThread(
                shape, world.prev_stage_group, dg.get(prv + ("fwd",)), device,
                start=world.has_prev_stage, **kw)
        else:
            raise ValueError(f"transport {self.transport!r}: 'host' or 'device'")
        self.dp = DPSync(world)

    # ---- pipeline p2p (unchanged protocol) ----------------------------------------------
    def send_forward(self, tensor: torch.Tensor, metadata: Metadata) -> None:
        if not self.world.has_next_stage:
            return
        dst = random.choice(self.world.stage2ranks[self.world.stage + 1])
        self.forward_send_thread.send(dst=dst, tensor=tensor, metadata=metadata)

    def send_backward(self, dst: int, tensor: torch.Tensor, metadata: Metadata) -> None:
        if not self.world.has_prev_stage:
            return
        self.backward_send_thread.send(dst=dst, tensor=tensor, metadata=metadata)

    def recv_forward(self):
        return self.forward_recv_thread.receive()

    def recv_backward(self):
        return self.backward_recv_thread.receive()

    def load_forward(self, metadata: Metadata) -> None:
        self.forward_recv_thread.load(tensor=None, metadata=metadata)

    # ---- the DP sync (outer-step hot path) ----------------------------------------------
    def sync_gradients(self, model: nn.Module) -> None:
        """src/comm.py:117-123 on RCCL + HIP (see DPSync)."""
        self.dp.sync_gradients(model)

    # ---- metrics aggregation (src/comm.py:125-149) ---------------------------------------
    def sync_outputs(self, outputs):
        peers = self.world.stage2ranks[self.world.stage]
        if len(peers) == 1:
            return outputs
        gathered: List = [None] * len(peers)
        dist.all_gather_object(gathered, outputs, group=self.world.curr_stage_group)

        def total(vals):
            return sum(v for v in vals if v not in (0, None))

        def mean(vals):
            kept = [v for v in vals if v not in (0, None)]
            return sum(kept) / len(kept) if kept else 0

        return type(outputs)(
            step=outputs.step,
            tokens=total([o.tokens for o in gathered]),
            num_micro_batches=total([o.num_micro_batches for o in gathered]),
            time=mean([o.time for o in gathered]),
            loss=mean([o.loss for o in gathered]),
            lr=mean([o.lr for o in gathered]),
            norm=mean([o.norm for o in gathered]),
            micro_step_time=mean([o.micro_step_time for o in gathered]),
        )


class InferenceComm:
    """Leader ring for sampling (src/comm.py:151-183); unframed p2p, unchanged protocol."""

    def __init__(self, world, shape: Tuple[int, ...], logger):
        self.world, self.shape, self.logger = world, shape, logger
        kw = {"tag": 1, "serialize": False, "requires_grad": False, "start": True,
              "logger": logger}
        if not world.is_leader:
            return
        if world.is_first_stage:
            self.send_thread = SendThread(shape, group=world.next_stage_group, **kw)
            self.recv_thread = RecvThread(shape[:-1], group=world.first_last_stage_group,
                                          dtype=torch.long, **kw)
        elif world.is_last_stage:
            self.send_thread = SendThread(shape[:-1], group=world.first_last_stage_group, **kw)
            self.recv_thread = RecvThread(shape, group=world.prev_stage_group, **kw)
        else:
            self.send_thread = SendThread(shape, group=world.next_stage_group, **kw)
            self.recv_thread = RecvThread(shape, group=world.prev_stage_group, **kw)
        self.receive_tensor_type = "hidden_states" if not world.is_first_stage else "input_ids"
        self.dst = (world.stage2leader[world.stage + 1] if not world.is_last_stage
                    else world.stage2leader[0])

    def receive(self):
        return self.receive_tensor_type, self.recv_thread.receive()[1]

    def send(self, tensor: torch.Tensor) -> None:
        if self.world.rank == self.dst:
            self.load(tensor)
            return
        self.send_thread.send(dst=self.dst, tensor=tensor, metadata=None)

    def load(self, tensor: torch.Tensor) -> None:
        self.recv_thread.load(tensor=tensor, metadata=None)
