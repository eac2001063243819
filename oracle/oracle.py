"""Python face of the CPU oracle (TEST INFRASTRUCTURE -- checker only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It wraps oracle/liboracle.so (the C restatement of the reference's outer step, see
diloco_oracle.c for the file:line map) and composes the per-tensor reference sequence of
src/train.py:261-269 over a whole tree:

    delta_r  = outer - inner_r                      src/utils.py:221
    avg      = (Σ_r delta_r) / n   (n == 1: delta)   src/comm.py:117-123
    θ, buf   = SGD-Nesterov(θ, buf, avg)             src/train.py:267 (torch _single_tensor_sgd)
    inner    = θ                                     src/utils.py:226
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

_F = ctypes.POINTER(ctypes.c_float)
_I64 = ctypes.POINTER(ctypes.c_int64)
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        lib.or_plan_tables.argtypes = [_I64, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, _I64,
                                       _I64, ctypes.POINTER(ctypes.c_int32)]
        lib.or_plan_tables.restype = ctypes.c_int
        lib.or_plan_tables_ex.argtypes = [_I64, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                                          ctypes.c_int64, _I64, _I64,
                                          ctypes.POINTER(ctypes.c_int32)]
        lib.or_plan_tables_ex.restype = ctypes.c_int
        lib.or_delta.argtypes = [_F, _F, _F, ctypes.c_int64]
        lib.or_sum_avg.argtypes = [ctypes.POINTER(_F), ctypes.c_int32, _F, ctypes.c_int64]
        lib.or_sgd.argtypes = [_F, _F, _F, ctypes.c_int64, ctypes.c_float, ctypes.c_float,
                               ctypes.c_int32, ctypes.c_int32]
        lib.or_copy.argtypes = [_F, _F, ctypes.c_int64]
        lib.or_bf16_round.argtypes = [_F, _F, ctypes.c_int64]
        lib.or_fill_synth.argtypes = [_F, ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint64,
                                      ctypes.c_float, ctypes.c_float, _F]
        _U8 = ctypes.POINTER(ctypes.c_uint8)
        lib.or_delta_q8.argtypes = [_F, _F, ctypes.c_int64, _U8]
        lib.or_q8_deq.argtypes = [_U8, ctypes.c_int64, _F]
        lib.or_q8_reduce.argtypes = [_U8, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _U8]
        for f in ("or_delta", "or_sum_avg", "or_sgd", "or_copy", "or_bf16_round", "or_fill_synth",
                  "or_delta_q8", "or_q8_deq", "or_q8_reduce"):
            getattr(lib, f).restype = None
        _lib = lib
    return _lib


def _fp(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(_F)


# ---- planner ------------------------------------------------------------------------------
def plan_tables(numels: Sequence[int], cap: int, align: int = 64,
                bucket_align: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    lib = load()
    n = len(numels)
    num = np.asarray(numels, dtype=np.int64)
    seg = np.zeros(n + 1, dtype=np.int64)
    bnd = np.zeros(n + 1, dtype=np.int64)
    nb = ctypes.c_int32()
    rc = lib.or_plan_tables_ex(num.ctypes.data_as(_I64), n, cap, align, bucket_align or align,
                               seg.ctypes.data_as(_I64), bnd.ctypes.data_as(_I64),
                               ctypes.byref(nb))
    if rc:
        raise ValueError("or_plan_tables: bad arguments")
    return seg, bnd[: nb.value + 1].copy()


def plan_tables_py(numels: Sequence[int], cap: int, align: int = 64, bucket_align: int = 0):
    """Pure-Python statement of the same rule (cross-checks the C oracle)."""
    ba = bucket_align or align
    up = lambda x, a: -(-x // a) * a  # noqa: E731
    if not numels:
        return [0], [0]
    seg, bounds, nxt, begin = [], [0], 0, 0
    for i, n in enumerate(numels):
        at = nxt
        if cap > 0 and i > bounds[-1] and up(at + n, align) - begin > cap:
            at = begin = up(nxt, ba)
            bounds.append(i)
        seg.append(at)
        nxt = up(at + n, align)
    seg.append(up(nxt, ba))
    bounds.append(len(numels))
    return seg, bounds


# ---- elementwise steps ---------------------------------------------------------------------
def delta(outer: np.ndarray, inner: np.ndarray) -> np.ndarray:
    out = np.empty_like(outer)
    load().or_delta(_fp(outer), _fp(inner), _fp(out), outer.size)
    return out


def sum_avg(grads: Sequence[np.ndarray]) -> np.ndarray:
    n = len(grads)
    arr = (_F * n)(*[_fp(g) for g in grads])
    out = np.empty_like(grads[0])
    load().or_sum_avg(arr, n, _fp(out), out.size)
    return out


def sgd(theta: np.ndarray, buf: Optional[np.ndarray], g: np.ndarray, lr: float, momentum: float,
        nesterov: bool, first: bool) -> None:
    """In place on theta (and buf)."""
    if buf is None:
        buf = np.empty_like(theta)
    load().or_sgd(_fp(theta), _fp(buf), _fp(g), theta.size, lr, momentum, int(nesterov),
                  int(first))


def bf16_round(x: np.ndarray) -> np.ndarray:
    out = np.empty_like(x)
    load().or_bf16_round(_fp(x), _fp(out), x.size)
    return out


def fill_synth(n: int, seed: int, stream: int, base: float, scale: float, add=None) -> np.ndarray:
    out = np.empty(n, dtype=np.float32)
    load().or_fill_synth(_fp(out), n, seed, stream, base, scale,
                         _fp(add) if add is not None else None)
    return out


# ---- int8 wire codec ------------------------------------------------------------------------
Q8_SLOT, Q8_HDR, CHUNK = 4160, 64, 4096


def _u8(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def chunks_of(numel: int):
    """(offset, length) of each DL_CHUNK_ELEMS chunk of one tensor, in order."""
    return [(o, min(CHUNK, numel - o)) for o in range(0, numel, CHUNK)]


def delta_q8(outer: np.ndarray, inner: np.ndarray) -> np.ndarray:
    """Slots (one per chunk) of quantise(outer - inner) for one tensor."""
    ch = chunks_of(outer.size)
    slots = np.zeros(len(ch) * Q8_SLOT, dtype=np.uint8)
    for k, (o, n) in enumerate(ch):
        load().or_delta_q8(_fp(np.ascontiguousarray(outer[o:o + n])),
                           _fp(np.ascontiguousarray(inner[o:o + n])), n,
                           _u8(slots[k * Q8_SLOT:(k + 1) * Q8_SLOT]))
    return slots


def q8_reduce(recv: np.ndarray, n: int, m: int, divisor: int) -> np.ndarray:
    out = np.zeros(m * Q8_SLOT, dtype=np.uint8)
    load().or_q8_reduce(_u8(np.ascontiguousarray(recv)), n, m, divisor, _u8(out))
    return out


def q8_deq(slots: np.ndarray, numel: int) -> np.ndarray:
    out = np.empty(numel, dtype=np.float32)
    for k, (o, n) in enumerate(chunks_of(numel)):
        buf = np.empty(n, dtype=np.float32)
        load().or_q8_deq(_u8(np.ascontiguousarray(slots[k * Q8_SLOT:(k + 1) * Q8_SLOT])), n,
                         _fp(buf))
        out[o:o + n] = buf
    return out


def q8_average(deltas_by_rank, numels, bucket_chunks):
    """The int8 exchange of one outer step, restated: per-tensor deltas of every rank ->
    per-tensor averaged, dequantised g (what every rank applies). bucket_chunks: list of
    chunk counts per bucket (chunks in tree order)."""
    n = len(deltas_by_rank)
    slots = [np.concatenate([delta_q8_from(d[t]) for t in range(len(numels))])
             for d in deltas_by_rank]
    avg_slots, c = [], 0
    for nch in bucket_chunks:
        m = -(-nch // n)
        per = []
        for r in range(n):
            s = np.zeros(n * m * Q8_SLOT, dtype=np.uint8)
            s[:nch * Q8_SLOT] = slots[r][c * Q8_SLOT:(c + nch) * Q8_SLOT]
            per.append(s)
        gathered = []
        for p in range(n):  # all_to_all: peer p gets slots [p*m, (p+1)*m) from every rank
            recv = np.concatenate([per[r][p * m * Q8_SLOT:(p + 1) * m * Q8_SLOT] for r in range(n)])
            gathered.append(q8_reduce(recv, n, m, n))
        avg_slots.append(np.concatenate(gathered)[:nch * Q8_SLOT])  # all_gather, drop padding
        c += nch
    flat = np.concatenate(avg_slots)
    out, c = [], 0
    for t, numel in enumerate(numels):
        k = len(chunks_of(numel))
        out.append(q8_deq(flat[c * Q8_SLOT:(c + k) * Q8_SLOT], numel))
        c += k
    return out


def delta_q8_from(delta: np.ndarray) -> np.ndarray:
    """Slots of quantise(delta) for one tensor (delta = outer - inner already formed)."""
    return delta_q8(delta, np.zeros_like(delta))


# ---- one outer step over a tree ----------------------------------------------------------
class OuterState:
    """Host state of the reference's outer optimizer for one tree (list of flat fp32 arrays)."""

    def __init__(self, theta: Sequence[np.ndarray], lr=0.7, momentum=0.9, nesterov=True):
        self.theta = [np.array(t, dtype=np.float32, copy=True).reshape(-1) for t in theta]
        self.buf: List[Optional[np.ndarray]] = [None] * len(self.theta)
        self.lr, self.momentum, self.nesterov = lr, momentum, nesterov
        self.steps = 0

    def step(self, inners_by_rank: Sequence[Sequence[np.ndarray]], wire: str = "f32"):
        """Run a2..a5 for every rank's inner tree; returns (deltas_by_rank, avg)."""
        n = len(inners_by_rank)
        deltas = [[delta(self.theta[t], inner[t].reshape(-1)) for t in range(len(self.theta))]
                  for inner in inners_by_rank]
        if wire == "bf16":
            deltas = [[bf16_round(d) for d in dr] for dr in deltas]
        avg = [sum_avg([deltas[r][t] for r in range(n)]) for t in range(len(self.theta))]
        first = self.steps == 0
        for t in range(len(self.theta)):
            if self.momentum != 0 and self.buf[t] is None:
                self.buf[t] = np.empty_like(self.theta[t])
            sgd(self.theta[t], self.buf[t], avg[t], self.lr, self.momentum, self.nesterov, first)
        self.steps += 1
        return deltas, avg
