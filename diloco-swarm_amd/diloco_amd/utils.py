"""Drop-in for the DiLoCo helpers of src/utils.py:203-226 and get_optimizer (src/utils.py:59-65).

Same names, arguments and host-visible results as the reference. Dispatch is on the inner
model's device, as the reference's `.to(param_outer.device)` / `.to(param_inner.device)`
copies are (src/utils.py:221,226): a GPU inner model runs the HIP path below; a CPU inner
model (the reference's --device cpu runs, tests/test_memorize.py:35-39) gets the reference's
per-tensor torch ops on the host. The GPU path has no CPU fallback: without libdiloco_hip.so
it raises. On the GPU:

  get_outer_model(inner)            deepcopy(inner).to("cpu")              src/utils.py:213-216
  compute_pseudo_gradient(in, out)  out.grad = out - in   (dl_delta_pack)   src/utils.py:218-221
  sync_inner_model(out, in)         in = out              (dl_scatter)      src/utils.py:223-226
  get_optimizer(model, cfg)         AdamW | SGD (outer: OuterSGD, HIP)      src/utils.py:59-65

Placement of the outer model (`get_outer_model(..., placement=)`, default from the
DILOCO_OUTER_PLACEMENT environment variable, "host" if unset):

  "host"    the reference's placement: a CPU module whose parameters, gradients and momentum
            buffers hold exactly the reference's values whenever they are read. Write-back
            (`get_outer_model(..., write_back=)`, default from DILOCO_HOST_WRITEBACK):
              "lazy" (default)  the outer step runs on an HBM twin of the outer model
                        (mirror.LazyHostOuterMirror around a DeviceOuterMirror: the same
                        kernels and exchange as "device" below, no PCIe traffic per step);
                        the CPU tensors are views of pinned arenas refreshed from HBM when
                        something reads them (mirror.HostParameter / HostTensor), and host
                        writes are uploaded before the next call;
              "sync"    the host tensors are authoritative: every call ends with them
                        updated, one pinned DMA per arena (mirror.HostOuterMirror);
              "deferred"  as "sync", the step's write-back issued by sync_inner_model in one
                        batch of DMAs and not waited for (flush_outer_model / state_dict()
                        wait for it).
  "device"  SURVEY §8f row 2: the outer module lives on the inner model's GPU, its parameters,
            .grad and momentum buffers are views of packed HBM arenas
            (mirror.DeviceOuterMirror); host copies are made by torch on demand (`.cpu()`).

For "device" and "host"/"lazy": fused (`get_outer_model(..., fused=)`, DILOCO_OUTER_FUSED, on
if unset) runs the four calls as one HBM pass at one peer (dl_delta_pack_sgd) and as
pack -> exchange -> one SGD pass at N > 1, with .grad completing the deferred work when read
and sync_inner_model a verified no-op after the step; wire (DILOCO_OUTER_WIRE, "f32";
"bf16": BASELINE config #5's codec on the DP exchange); exchange (DILOCO_OUTER_EXCHANGE;
"replicated", the host placement's default: all_reduce -> the SGD pass on every rank, so
.grad and the momentum are local on every rank as in the reference; "sharded", the device
placement's default: reduce_scatter -> SGD on this rank's 1/n -> all_gather of θ, SURVEY §8e;
"a2a": the sharded form with a rank-order sum, bit-exact at every n; DILOCO_DP_EXCHANGE=a2a
selects it too). Under the sharded forms a read of .grad or of the momentum buffers at N > 1
gathers them from the peers: a collective over the DP group that every rank must make; a read
its peers do not make raises RuntimeError after DILOCO_COLLECTIVE_READ_TIMEOUT seconds
(mirror.collective_read) instead of hanging.
"""
from __future__ import annotations

import copy
import os

import torch
import torch.nn as nn
from torch.optim import SGD, AdamW, Optimizer

from .kernels import default_kernels
from .mirror import (DEFAULT_EXCHANGE, OUTER_EXCHANGES, OUTER_WIRES, WRITE_BACKS,
                     DeviceOuterMirror, HostOuterMirror, LazyHostOuterMirror, module_params)
from .optim import OuterSGD
from .plan import DEFAULT_BUCKET_CAP_ELEMS

_ATTR = "_diloco_mirror"
_OUTER = "_diloco_outer"
_PLACEMENT = "_diloco_placement"
_WRITE_BACK = "_diloco_write_back"
_FUSED = "_diloco_fused"
_WIRE = "_diloco_wire"
_EXCHANGE = "_diloco_exchange"
_PENDING = "_diloco_pending_device"  # placement="device" built before the inner model moved
PLACEMENTS = ("host", "device")
_TRUE = ("1", "true", "on", "yes")
_FALSE = ("0", "false", "off", "no")


def env_flag(name: str, default: bool) -> bool:
    """A boolean knob from the environment: 1/0, true/false, on/off, yes/no (any case);
    anything else raises instead of silently meaning "on"."""
    v = os.environ.get(name)
    if v is None or v.strip() == "":
        return default
    v = v.strip().lower()
    if v in _TRUE:
        return True
    if v in _FALSE:
        return False
    raise ValueError(f"{name}={os.environ[name]!r}: one of {_TRUE + _FALSE}")


def device_path(t: torch.Tensor) -> bool:
    """True when tensors on t's device take the HIP path: device tensors always; host tensors
    only under a test backend that declares it computes on host tensors
    (tests/oracle_kernels.py: accepts_host_tensors, installed with set_default_kernels)."""
    return t.device.type != "cpu" or getattr(default_kernels(), "accepts_host_tensors", False)


def has_mirror(outer_model: nn.Module) -> bool:
    return getattr(outer_model, _ATTR, None) is not None


def outer_mirror(outer_model: nn.Module, device=None):
    """The device mirror of an outer model (created on first use): HostOuterMirror for the
    reference's host placement, DeviceOuterMirror for placement="device"."""
    m = getattr(outer_model, _ATTR, None)
    if m is None:
        k = default_kernels()
        if getattr(outer_model, _PLACEMENT, "host") == "device":
            p = next(outer_model.parameters(), None)
            if p is None:
                raise ValueError("outer model has no parameters")
            keep = getattr(outer_model, _PENDING, False)
            dev = p.device
            if keep:  # the device is the inner model's, named now by the caller
                if device is None:
                    raise RuntimeError("the device outer model gets its device from the inner "
                                       "model's first compute_pseudo_gradient on the GPU")
                # its CPU parameters go straight into the HBM arena, tensor by tensor
                # (DeviceOuterMirror keep_params): no whole-model device copy first
                dev = torch.device(device)
                object.__setattr__(outer_model, _PENDING, False)
            cap = int(os.environ.get("DILOCO_OUTER_BUCKET_ELEMS", DEFAULT_BUCKET_CAP_ELEMS))
            m = DeviceOuterMirror(outer_model, dev, kernels=k, bucket_cap_elems=cap,
                                  fused=getattr(outer_model, _FUSED, False),
                                  wire=getattr(outer_model, _WIRE, "f32"),
                                  exchange=getattr(outer_model, _EXCHANGE,
                                                   DEFAULT_EXCHANGE["device"]),
                                  keep_params=keep)
            object.__setattr__(outer_model, _ATTR, m)
            return m
        if device is None:
            device = getattr(k, "default_device", None)
            if device is None:
                if not torch.cuda.is_available():
                    raise RuntimeError("the DiLoCo outer step runs on the GPU; no HIP device")
                device = torch.device("cuda", torch.cuda.current_device())
        wb = getattr(outer_model, _WRITE_BACK, "lazy")
        if wb == "lazy":
            cap = int(os.environ.get("DILOCO_OUTER_BUCKET_ELEMS", DEFAULT_BUCKET_CAP_ELEMS))
            m = LazyHostOuterMirror(outer_model, torch.device(device), kernels=k,
                                    bucket_cap_elems=cap,
                                    fused=getattr(outer_model, _FUSED, True),
                                    wire=getattr(outer_model, _WIRE, "f32"),
                                    exchange=getattr(outer_model, _EXCHANGE,
                                                     DEFAULT_EXCHANGE["host"]))
        else:
            m = HostOuterMirror(outer_model, torch.device(device), kernels=k, write_back=wb)
        object.__setattr__(outer_model, _ATTR, m)  # not a submodule / not in state_dict
    return m


def _inner_device(inner_model: nn.Module) -> torch.device:
    p = next(inner_model.parameters(), None)
    if p is None:
        raise ValueError("inner model has no parameters")
    return p.device


def get_outer_model(inner_model: nn.Module, placement: str = None,
                    write_back: str = None, fused: bool = None, wire: str = None,
                    exchange: str = None) -> nn.Module:
    """Initializes the outer model from the inner model (src/utils.py:213-216).

    placement "host" (the reference's, default) or "device" (in HBM: on the inner model's GPU;
    built while the inner model is on the CPU, it stays there until the first
    compute_pseudo_gradient names the device); write_back "lazy" (default: the host outer
    model stepped on an HBM twin), "sync" or "deferred" for the host placement; fused
    (default on), wire ("f32" default, "bf16": BASELINE config #5's codec; "int8") and
    exchange ("replicated" for the host placement and "sharded" for placement="device" by
    default, or "a2a") for placement="device" and for the lazy host write-back (see the module
    docstring)."""
    if placement is None:
        placement = os.environ.get("DILOCO_OUTER_PLACEMENT", "host")
    if placement not in PLACEMENTS:
        raise ValueError(f"placement {placement!r}: one of {PLACEMENTS}")
    if write_back is None:
        write_back = os.environ.get("DILOCO_HOST_WRITEBACK", "lazy")
    if write_back not in WRITE_BACKS:
        raise ValueError(f"write_back {write_back!r}: one of {WRITE_BACKS}")
    if fused is None:
        fused = env_flag("DILOCO_OUTER_FUSED", True)
    if wire is None:
        wire = os.environ.get("DILOCO_OUTER_WIRE", "f32")
    if wire not in OUTER_WIRES:
        raise ValueError(f"wire {wire!r}: one of {OUTER_WIRES}")
    if exchange is None:
        exchange = os.environ.get("DILOCO_OUTER_EXCHANGE") or DEFAULT_EXCHANGE[placement]
    if exchange not in OUTER_EXCHANGES:
        raise ValueError(f"exchange {exchange!r}: one of {OUTER_EXCHANGES}")
    lazy = placement == "device" or write_back == "lazy"  # the outer step runs on an HBM copy
    if wire != "f32" and not lazy:
        raise ValueError("the bf16 outer wire needs placement='device' or write_back='lazy' "
                         "(write_back 'sync' / 'deferred' keep the host tensors authoritative)")
    outer_model = copy.deepcopy(inner_model)
    has_params = next(inner_model.parameters(), None) is not None
    if placement == "host":
        outer_model = outer_model.to("cpu")
    elif has_params:  # the inner model's GPU. The reference builds the outer model before it
        # moves the inner one to cuda:local_rank (src/train.py:382, :163, :368 with
        # src/utils.py:36-40) and never sets the current device: a CPU inner model leaves the
        # outer one on the CPU until the first compute_pseudo_gradient names the device
        # (outer_mirror; until then the four calls are the reference's host loops)
        dev = _inner_device(inner_model)
        if dev.type == "cpu" and device_path(next(inner_model.parameters())):
            # a test backend that computes on host tensors (tests/oracle_kernels.py)
            outer_model = outer_model.to(default_kernels().default_device)
        elif dev.type == "cpu":
            object.__setattr__(outer_model, _PENDING, True)
        else:
            outer_model = outer_model.to(dev)
    object.__setattr__(outer_model, _OUTER, True)  # get_optimizer: SGD here is the outer SGD
    object.__setattr__(outer_model, _PLACEMENT, placement)
    object.__setattr__(outer_model, _WRITE_BACK, write_back)
    object.__setattr__(outer_model, _FUSED, bool(fused) and lazy)
    object.__setattr__(outer_model, _WIRE, wire)
    object.__setattr__(outer_model, _EXCHANGE, exchange)
    if placement == "device" and has_params and not getattr(outer_model, _PENDING, False):
        # lay the parameters out in the packed HBM arena now (fused: as OuterParameters);
        # a model without parameters keeps none: the four calls are the reference's empty loops
        outer_mirror(outer_model)
    elif write_back == "lazy" and has_params and device_path(next(inner_model.parameters())):
        # the inner model is on its GPU already: the HBM twin now (the reference builds the
        # outer model before moving the inner one, src/train.py:382; then the first
        # compute_pseudo_gradient creates it)
        outer_mirror(outer_model, _inner_device(inner_model))
    elif write_back == "deferred":
        # a checkpoint of the outer model waits for the write-back in flight
        outer_model.register_state_dict_pre_hook(lambda mod, prefix, keep_vars:
                                                  flush_outer_model(mod))
    return outer_model


def flush_outer_model(outer_model: nn.Module) -> None:
    """Make the host tensors of an outer model (parameters, .grad, momentum buffers) current:
    waits for a deferred write-back (a no-op for write_back="sync" and placement="device")."""
    m = getattr(outer_model, _ATTR, None)
    if m is not None:
        m.flush()


def _host_path(inner_model: nn.Module, outer_model: nn.Module) -> bool:
    """The reference's host semantics apply: a CPU inner model (or one without parameters,
    for which the reference's loops run zero times) and no device mirror."""
    p = next(inner_model.parameters(), None)
    return (p is None or not device_path(p)) and not has_mirror(outer_model)


def compute_pseudo_gradient(inner_model: nn.Module, outer_model: nn.Module) -> None:
    """outer.grad = outer - inner for every parameter (src/utils.py:218-221)."""
    m = getattr(outer_model, _ATTR, None)
    if m is not None:  # every call after the first: straight to the mirror
        m.pseudo_gradient(module_params(inner_model))
        return
    if _host_path(inner_model, outer_model):
        with torch.no_grad():
            for po, pi in zip(outer_model.parameters(), inner_model.parameters()):
                po.grad = torch.sub(po.data, pi.data.to(po.device))  # a fresh tensor
        return
    dev = _inner_device(inner_model)
    m = outer_mirror(outer_model, dev if dev.type != "cpu" else None)
    m.pseudo_gradient(module_params(inner_model))


def sync_inner_model(outer_model: nn.Module, inner_model: nn.Module) -> None:
    """inner = outer for every parameter (src/utils.py:223-226)."""
    m = getattr(outer_model, _ATTR, None)
    if m is not None:
        m.copy_to_inner(module_params(inner_model))
        return
    if _host_path(inner_model, outer_model):
        with torch.no_grad():
            for po, pi in zip(outer_model.parameters(), inner_model.parameters()):
                pi.data.copy_(po.data.to(pi.device))
        return
    dev = _inner_device(inner_model)
    m = outer_mirror(outer_model, dev if dev.type != "cpu" else None)
    m.copy_to_inner(module_params(inner_model))


def get_optimizer(model: nn.Module, optimizer_config) -> Optimizer:
    """src/utils.py:59-65. SGD on the outer model (from get_outer_model) -> OuterSGD."""
    if optimizer_config.type == "AdamW":
        return AdamW(model.parameters(), lr=optimizer_config.lr,
                     weight_decay=optimizer_config.weight_decay, betas=optimizer_config.betas)
    elif optimizer_config.type == "SGD":
        if getattr(model, _OUTER, False):
            return OuterSGD(model, lr=optimizer_config.lr, momentum=optimizer_config.momentum,
                            nesterov=optimizer_config.nesterov)
        return SGD(model.parameters(), lr=optimizer_config.lr, momentum=optimizer_config.momentum,
                   nesterov=optimizer_config.nesterov)
    else:
        raise ValueError(f"Invalid optimizer type: {optimizer_config.type}")
