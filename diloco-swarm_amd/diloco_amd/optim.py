"""The outer optimizer: torch.optim.SGD's interface, the HIP fused update underneath.

`get_optimizer(outer_model, cfg)` with cfg.type == "SGD" (src/utils.py:62-63; the DiLoCo
runs use Nesterov, configs/optimizer/nesterov.toml, lr 0.7 at experiments/experiment1.sh:65)
returns an `OuterSGD`. It IS a torch.optim.SGD (param_groups, state_dict, LR schedulers work
unchanged) whose step() runs `_single_tensor_sgd`'s arithmetic for the whole tree in one
dl_unpack_sgd launch on the device mirror of the outer model (mirror.HostOuterMirror), then
writes θ and the momentum buffers back to the host tensors the optimizer owns.
"""
from __future__ import annotations

import torch
from torch.optim import SGD

from .mirror import HostOuterMirror


class OuterSGD(SGD):
    def __init__(self, model: torch.nn.Module, lr: float, momentum: float = 0.0,
                 nesterov: bool = False):
        super().__init__(model.parameters(), lr=lr, momentum=momentum, nesterov=nesterov)
        self._model = model

    def _mirror(self) -> HostOuterMirror:
        from .utils import outer_mirror  # local import: utils builds on this module

        return outer_mirror(self._model)

    def state_dict(self):
        """torch.optim.SGD.state_dict, after a deferred write-back of the momentum landed."""
        from .utils import flush_outer_model

        flush_outer_model(self._model)
        return super().state_dict()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if len(self.param_groups) != 1:
            raise NotImplementedError("OuterSGD: one parameter group (as get_optimizer builds)")
        g = self.param_groups[0]
        if g["weight_decay"] != 0 or g["dampening"] != 0 or g["maximize"]:
            raise NotImplementedError(
                "OuterSGD implements SGD as src/utils.py:63 builds it: weight_decay=0, "
                "dampening=0, maximize=False")
        if g["nesterov"] and g["momentum"] == 0:
            raise ValueError("Nesterov momentum requires a momentum")
        from .utils import device_path, has_mirror

        if not has_mirror(self._model) and not device_path(g["params"][0]):
            # host tensors never stepped on the GPU (the reference's --device cpu runs):
            # torch.optim.SGD itself, as src/utils.py:62-63 builds it
            super().step()
            return loss
        mirror = self._mirror()
        params = g["params"]
        if len(params) != len(mirror.params) or any(a is not b for a, b in zip(params, mirror.params)):
            raise RuntimeError("OuterSGD parameters differ from its model's parameters()")
        momentum = float(g["momentum"])
        host_bufs = [self.state[p].get("momentum_buffer") for p in params]
        lr = g["lr"]
        if isinstance(lr, torch.Tensor):
            lr = float(lr.item())
        bufs = mirror.sgd_step(float(lr), momentum, bool(g["nesterov"]), host_bufs)
        if momentum != 0:
            for p, b in zip(params, bufs):
                self.state[p]["momentum_buffer"] = b
        return loss
