"""Drop-in for the DiLoCo helpers of src/utils.py:203-226 and get_optimizer (src/utils.py:59-65).

Same names, arguments and host-visible results as the reference; the work runs on the GPU:

  get_outer_model(inner)            deepcopy(inner).to("cpu")              src/utils.py:213-216
  compute_pseudo_gradient(in, out)  out.grad = out - in   (dl_delta_pack)   src/utils.py:218-221
  sync_inner_model(out, in)         in = out              (dl_scatter)      src/utils.py:223-226
  get_optimizer(model, cfg)         AdamW | SGD (outer: OuterSGD, HIP)      src/utils.py:59-65

The outer model stays a CPU module whose parameters, gradients and momentum buffers hold
exactly the reference's values; a device mirror (mirror.HostOuterMirror) is attached to it on
first use and keeps the packed copies in HBM coherent with the host tensors.
"""
from __future__ import annotations

import copy

import torch
import torch.nn as nn
from torch.optim import SGD, AdamW, Optimizer

from .kernels import default_kernels
from .mirror import HostOuterMirror
from .optim import OuterSGD

_ATTR = "_diloco_mirror"
_OUTER = "_diloco_outer"


def outer_mirror(outer_model: nn.Module, device=None) -> HostOuterMirror:
    """The device mirror of a host outer model (created on first use)."""
    m = getattr(outer_model, _ATTR, None)
    if m is None:
        k = default_kernels()
        if device is None:
            device = getattr(k, "default_device", None)
            if device is None:
                if not torch.cuda.is_available():
                    raise RuntimeError("the DiLoCo outer step runs on the GPU; no HIP device")
                device = torch.device("cuda", torch.cuda.current_device())
        m = HostOuterMirror(outer_model, torch.device(device), kernels=k)
        object.__setattr__(outer_model, _ATTR, m)  # not a submodule / not in state_dict
    return m


def _inner_device(inner_model: nn.Module) -> torch.device:
    p = next(inner_model.parameters(), None)
    if p is None:
        raise ValueError("inner model has no parameters")
    return p.device


def get_outer_model(inner_model: nn.Module) -> nn.Module:
    """Initializes the outer model from the inner model (src/utils.py:213-216)."""
    outer_model = copy.deepcopy(inner_model)
    outer_model = outer_model.to("cpu")
    object.__setattr__(outer_model, _OUTER, True)  # get_optimizer: SGD here is the outer SGD
    return outer_model


def compute_pseudo_gradient(inner_model: nn.Module, outer_model: nn.Module) -> None:
    """outer.grad = outer - inner for every parameter (src/utils.py:218-221)."""
    dev = _inner_device(inner_model)
    m = outer_mirror(outer_model, dev if dev.type != "cpu" else None)
    m.pseudo_gradient(list(inner_model.parameters()))


def sync_inner_model(outer_model: nn.Module, inner_model: nn.Module) -> None:
    """inner = outer for every parameter (src/utils.py:223-226)."""
    dev = _inner_device(inner_model)
    m = outer_mirror(outer_model, dev if dev.type != "cpu" else None)
    m.copy_to_inner(list(inner_model.parameters()))


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
