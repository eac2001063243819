"""Packed layout of a parameter tree and the device handle that walks it.

The reference has no layout: it loops over `model.parameters()` one tensor at a time
(src/comm.py:120-123, src/utils.py:220,225). The build packs the tree, in that order, into one
flat buffer: segment i starts at seg_off[i] (a multiple of ALIGN_ELEMS = 64 elements, 256 B),
and buckets are greedy runs of whole segments whose padded size stays <= the cap. The rule is
frozen (oracle/diloco_oracle.c:or_plan_tables, tests/golden/plan_tables.json).
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence, Tuple

import numpy as np

from . import _lib

SLOT_INNER = 0   # inner model parameters (device)
SLOT_GRAD = 1    # per-tensor gradients (device)
SLOT_AUX = 2
SLOT_AUX2 = 3

DEFAULT_BUCKET_CAP_ELEMS = 64 << 20  # 256 MiB of fp32 per bucket


def plan_tables(numels: Sequence[int], cap_elems: int = DEFAULT_BUCKET_CAP_ELEMS,
                align_elems: int = _lib.ALIGN_ELEMS,
                bucket_align_elems: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """(seg_off[n+1], bkt_bounds[n_bkt+1]) from the C planner (host only, no GPU needed).
    bucket_align_elems (0 = align_elems): every bucket starts at a multiple of it, so a bucket
    splits into equal aligned shards for a reduce-scatter (ALIGN_ELEMS * peers)."""
    n = len(numels)
    num = np.ascontiguousarray(np.asarray(numels, dtype=np.int64))
    seg = np.zeros(n + 1, dtype=np.int64)
    bnd = np.zeros(n + 1, dtype=np.int64)
    nb = ctypes.c_int32(0)
    p64 = ctypes.POINTER(ctypes.c_int64)
    _lib.call(
        "dl_plan_tables_ex",
        num.ctypes.data_as(p64) if n else None, n, int(cap_elems), int(align_elems),
        int(bucket_align_elems or align_elems),
        seg.ctypes.data_as(p64), bnd.ctypes.data_as(p64), ctypes.byref(nb),
    )
    return seg, bnd[: nb.value + 1].copy()


class PackedTree:
    """Device handle (dl_tree_t) for one parameter tree on the current HIP device."""

    def __init__(self, numels: Sequence[int], cap_elems: int = DEFAULT_BUCKET_CAP_ELEMS,
                 bucket_align_elems: int = _lib.ALIGN_ELEMS):
        self.numels = [int(n) for n in numels]
        self.bucket_align = int(bucket_align_elems)
        n = len(self.numels)
        num = np.asarray(self.numels, dtype=np.int64)
        h = ctypes.c_void_p()
        _lib.call(
            "dl_tree_create_ex",
            num.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)) if n else None, n,
            int(cap_elems), self.bucket_align, ctypes.byref(h),
        )
        self._h = h
        tot, ns, nb, nc = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _lib.call("dl_tree_query", h, ctypes.byref(tot), ctypes.byref(ns), ctypes.byref(nb),
                  ctypes.byref(nc))
        self.total, self.n_seg, self.n_buckets, self.n_chunks = tot.value, ns.value, nb.value, nc.value
        seg = np.zeros(n + 1, dtype=np.int64)
        _lib.call("dl_tree_seg_off", h, seg.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
        self.seg_off = seg
        self.bucket_ranges: List[Tuple[int, int]] = []
        self.bucket_chunks: List[Tuple[int, int]] = []
        for b in range(self.n_buckets):
            lo, hi = ctypes.c_int64(), ctypes.c_int64()
            _lib.call("dl_tree_bucket_range", h, b, ctypes.byref(lo), ctypes.byref(hi))
            self.bucket_ranges.append((lo.value, hi.value))
            c0, c1 = ctypes.c_int32(), ctypes.c_int32()
            _lib.call("dl_tree_bucket_chunks", h, b, ctypes.byref(c0), ctypes.byref(c1))
            self.bucket_chunks.append((c0.value, c1.value))
        self._bound = [None] * _lib.MAX_SLOTS

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("PackedTree used after close()")
        return self._h

    def bind(self, slot: int, tensors, stream, key=None) -> None:
        """Upload the device addresses of `tensors` (fp32, contiguous) into `slot`.

        No-op when the addresses are unchanged since the last bind of this slot. key: the
        tuple of the tensors' addresses when the caller has it already.
        """
        if key is None:
            key = tuple([t.data_ptr() for t in tensors])
        if self._bound[slot] == key:  # fast path: same storage as last time (every outer step)
            return
        ptrs = []
        for i, t in enumerate(tensors):
            if t.dtype.itemsize != 4 or not t.is_floating_point():
                raise TypeError(f"tensor {i}: dtype {t.dtype}, the outer step is fp32")
            if not t.is_cuda or not t.is_contiguous():
                raise ValueError(f"tensor {i}: must be a contiguous device tensor")
            if t.numel() != self.numels[i]:
                raise ValueError(f"tensor {i}: numel {t.numel()} != planned {self.numels[i]}")
            ptrs.append(t.data_ptr())
        if len(ptrs) != self.n_seg:
            raise ValueError(f"{len(ptrs)} tensors for a {self.n_seg}-tensor tree")
        arr = np.asarray(ptrs, dtype=np.uint64)
        _lib.call("dl_tree_bind", self.handle, slot,
                  arr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)) if ptrs else None,
                  len(ptrs), stream)
        self._bound[slot] = key

    def tune(self, max_blocks: int = 0, flags: int = _lib.TUNE_AUTO) -> None:
        """Launch shape of the walker kernels (speed only; results are identical)."""
        _lib.call("dl_tree_tune", self.handle, int(max_blocks), int(flags))

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            try:
                _lib.call("dl_tree_destroy", self._h)
            finally:
                self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
