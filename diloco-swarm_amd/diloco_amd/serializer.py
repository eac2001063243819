"""Activation framing for SWARM point-to-point sends (src/serializer.py), on the GPU.

Same interface and wire format as the reference: `Serializer(shape).shape == (2, *shape)`;
`serialize(t, (a, b))` returns a (2, *t.shape) fp32 tensor whose plane 0 carries a, b as
floats at flat indices 0 and 1 (the rest of plane 0 is unspecified: the reference leaves it
uninitialised, src/serializer.py:12) and whose plane 1 is t promoted to fp32 (torch.cat's
promotion of an fp32 metadata plane with an fp32/bf16/fp16 payload); `deserialize` returns
(payload view, (int(a), int(b))).

serialize is one HIP kernel (dl_serialize: 2 metadata writes + a converting copy) instead of
torch.empty + two indexed writes + reshape + cat. It frames device tensors only.
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import _lib

Metadata = Tuple[int, int]  # (root, local_micro_step)

_SRC = {torch.float32: _lib.DL_F32, torch.bfloat16: _lib.DL_BF16, torch.float16: _lib.DL_F16}


class Serializer:
    def __init__(self, shape: Tuple[int, ...]):
        self.shape = (2, *shape)

    def serialize(self, tensor: torch.Tensor, metadata: Metadata) -> torch.Tensor:
        if tensor.device.type != "cuda":
            raise ValueError("diloco_amd.Serializer frames device tensors (HIP kernel); got "
                             f"{tensor.device}")
        if tensor.dtype not in _SRC:
            raise TypeError(f"serialize: payload dtype {tensor.dtype} (fp32/bf16/fp16)")
        n = tensor.numel()
        if n < 2:  # the reference fails on metadata_tensor[1] for the same inputs
            raise IndexError(f"index {n} is out of bounds for dimension 0 with size {n}")
        src = tensor.detach().contiguous()
        out = torch.empty((2, *tensor.shape), dtype=torch.float32, device=tensor.device)
        _lib.call("dl_serialize", src.data_ptr(), _SRC[tensor.dtype], n, float(metadata[0]),
                  float(metadata[1]), out.data_ptr(),
                  torch.cuda.current_stream(tensor.device).cuda_stream)
        return out

    def deserialize(self, serialized: torch.Tensor) -> Tuple[torch.Tensor, Metadata]:
        meta = serialized[0].flatten()[:2].tolist()  # one device->host read for both values
        return serialized[1:].squeeze(0), (int(meta[0]), int(meta[1]))
