"""The outer optimizer: torch.optim.SGD's interface, the HIP fused update underneath.

`get_optimizer(outer_model, cfg)` with cfg.type == "SGD" (src/utils.py:62-63; the DiLoCo
runs use Nesterov, configs/optimizer/nesterov.toml, lr 0.7 at experiments/experiment1.sh:65)
returns an `OuterSGD`. It IS a torch.optim.SGD (param_groups, state_dict, LR schedulers work
unchanged) whose step() runs `_single_tensor_sgd`'s arithmetic for the whole tree in one
dl_unpack_sgd launch on the device mirror of the outer model (mirror.HostOuterMirror), then
writes θ and the momentum buffers back to the host tensors the optimizer owns; on the device
outer model (mirror.DeviceOuterMirror) its state's momentum buffers are views of the packed
HBM momentum (mirror.MomentumBuffer).
"""
from __future__ import annotations

import inspect
from operator import is_, methodcaller

import torch
from torch.optim import SGD

from .mirror import HostOuterMirror

_MOMENTUM_BUFFER = methodcaller("get", "momentum_buffer")


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
        """One outer SGD step (src/train.py:267). torch.optim.Optimizer wraps it as it wraps
        every optimizer's step (its profiler annotation, the global and per-optimizer pre /
        post hooks), so hooks and LR schedulers see an ordinary SGD."""
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
        mirror = getattr(self._model, "_diloco_mirror", None)  # utils._ATTR
        if mirror is None:
            from .utils import device_path
        if mirror is None and not device_path(g["params"][0]):
            # host tensors never stepped on the GPU (the reference's --device cpu runs):
            # torch.optim.SGD's own step body, as src/utils.py:62-63 builds it -- unwrapped,
            # since this call already runs inside the hook wrapper (no_grad is ours)
            inspect.unwrap(SGD.step)(self)
            return loss
        if mirror is None:
            mirror = self._mirror()
        params = g["params"]
        if len(params) != len(mirror.params) or not all(map(is_, params, mirror.params)):
            raise RuntimeError("OuterSGD parameters differ from its model's parameters()")
        momentum = float(g["momentum"])
        # self.state is keyed by tensor (a Python __hash__ per lookup): when it holds exactly
        # the parameters in order -- every step after the first -- walk its values instead
        st = self.state
        same = len(st) == len(params) and all(map(is_, st.keys(), params))
        if same:
            host_bufs = list(map(_MOMENTUM_BUFFER, st.values()))
        else:
            host_bufs = [st[p].get("momentum_buffer") for p in params]
        lr = g["lr"]
        if isinstance(lr, torch.Tensor):
            lr = float(lr.item())
        bufs = mirror.sgd_step(float(lr), momentum, bool(g["nesterov"]), host_bufs)
        if momentum != 0:
            if same and all(map(is_, host_bufs, bufs)):
                pass  # the state already holds these buffers (every step after the first)
            elif same:
                for v, b in zip(st.values(), bufs):
                    v["momentum_buffer"] = b
            else:
                for p, b in zip(params, bufs):
                    st[p]["momentum_buffer"] = b
        return loss
