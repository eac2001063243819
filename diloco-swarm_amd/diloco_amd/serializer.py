"""Activation framing for SWARM point-to-point sends (src/serializer.py).

Same interface and wire format as the reference: `Serializer(shape).shape == (2, *shape)`;
`serialize(t, (a, b))` returns a (2, *t.shape) tensor on t's device whose plane 0 carries a, b
as floats at flat indices 0 and 1 (the rest of plane 0 is unspecified: the reference leaves
it uninitialised, src/serializer.py:12) and whose plane 1 is t promoted with fp32 (torch.cat's
promotion of the fp32 metadata plane with the payload: fp32/bf16/fp16 -> fp32, fp64 -> fp64);
`deserialize` returns (payload view, (int(a), int(b))).

Dispatch is on the payload's device, as the reference frames on `tensor.device`
(src/serializer.py:12):
  GPU  one HIP kernel (dl_serialize: 2 metadata writes + a converting copy; dl_serialize_f64
       for fp64 payloads, whose frame is fp64 as torch.cat makes it) instead of torch.empty +
       two indexed writes + reshape + cat. The frame keeps the payload's autograd graph, as
       torch.cat's does: a payload that requires grad is framed through an autograd.Function
       whose backward hands plane 1's gradient back in the payload's dtype. Without
       libdiloco_hip.so this raises (no fallback for device tensors).
  CPU  the same frame built with torch ops in host memory (the reference's --device cpu runs,
       tests/test_memorize.py:35-39).
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import _lib

Metadata = Tuple[int, int]  # (root, local_micro_step)

_SRC = {torch.float32: _lib.DL_F32, torch.bfloat16: _lib.DL_BF16, torch.float16: _lib.DL_F16}


def _frame_device(tensor: torch.Tensor, m0: float, m1: float) -> torch.Tensor:
    """dl_serialize(_f64) of a device payload into a new (2, *shape) frame."""
    src = tensor.detach().contiguous()
    s = torch.cuda.current_stream(tensor.device).cuda_stream
    if tensor.dtype == torch.float64:
        out = torch.empty((2, *tensor.shape), dtype=torch.float64, device=tensor.device)
        _lib.call("dl_serialize_f64", src.data_ptr(), src.numel(), m0, m1, out.data_ptr(), s)
        return out
    if tensor.dtype not in _SRC:
        raise TypeError(f"serialize: payload dtype {tensor.dtype} (fp32/bf16/fp16/fp64)")
    out = torch.empty((2, *tensor.shape), dtype=torch.float32, device=tensor.device)
    _lib.call("dl_serialize", src.data_ptr(), _SRC[tensor.dtype], src.numel(), m0, m1,
              out.data_ptr(), s)
    return out


class _Frame(torch.autograd.Function):
    """The HIP frame with torch.cat's backward: d(frame)/d(payload) is plane 1, cast back."""

    @staticmethod
    def forward(ctx, tensor, m0, m1):
        ctx.dtype = tensor.dtype
        return _frame_device(tensor, m0, m1)

    @staticmethod
    def backward(ctx, grad):
        return grad[1].to(ctx.dtype), None, None


class Serializer:
    def __init__(self, shape: Tuple[int, ...]):
        self.shape = (2, *shape)

    def serialize(self, tensor: torch.Tensor, metadata: Metadata) -> torch.Tensor:
        n = tensor.numel()
        if n < 2:  # the reference fails on metadata_tensor[1] for the same inputs
            raise IndexError(f"index {n} is out of bounds for dimension 0 with size {n}")
        if tensor.device.type != "cuda":
            return self._frame_host(tensor, metadata)
        m0, m1 = float(metadata[0]), float(metadata[1])
        if tensor.requires_grad and torch.is_grad_enabled():
            return _Frame.apply(tensor, m0, m1)
        return _frame_device(tensor, m0, m1)

    @staticmethod
    def _frame_host(tensor: torch.Tensor, metadata: Metadata) -> torch.Tensor:
        """The frame in host memory: payload copied into plane 1 (with torch.cat's dtype
        promotion and autograd), the two metadata floats written into plane 0."""
        dtype = torch.promote_types(torch.float32, tensor.dtype)
        meta = torch.empty(tensor.shape, dtype=torch.float32, device=tensor.device)
        flat = meta.view(-1)  # the metadata values are fp32 first, as in the reference
        flat[0] = float(metadata[0])
        flat[1] = float(metadata[1])
        return torch.stack([meta.to(dtype), tensor.to(dtype)])

    def deserialize(self, serialized: torch.Tensor) -> Tuple[torch.Tensor, Metadata]:
        meta = serialized[0].flatten()[:2].tolist()  # one device->host read for both values
        return serialized[1:].squeeze(0), (int(meta[0]), int(meta[1]))
