"""ctypes binding of libdiloco_hip.so (C-ABI declared in include/diloco_hip.h).

The product path has no fallback: if the library is missing or fails to load, every entry
point raises. Build it with `make -C diloco-swarm_amd/csrc` (or `__graft_entry__.build()`).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "DILOCO_HIP_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libdiloco_hip.so")
)

# constants mirrored from include/diloco_hip.h
ABI_VERSION = 2
ALIGN_ELEMS = 64
CHUNK_ELEMS = 4096
ALL_BUCKETS = -1
MAX_SLOTS = 4
Q8_SLOT_BYTES = 4160
IPC_HANDLE_BYTES = 64
DL_F32, DL_BF16, DL_F16, DL_U8 = 0, 1, 2, 3
TUNE_NT_LOADS, TUNE_NT_STORES, TUNE_WT_STORES, TUNE_PAIRS = 1, 2, 8, 16
TUNE_AUTO = -1
COPY_WIDE, COPY_READ, COPY_WRITE = 8, 16, 32


def COPY_STREAMS(s: int) -> int:
    """DL_COPY_STREAMS(s): the read / write probe over s equal streams (1..4)."""
    return ((s - 1) & 3) << 8


_i32, _i64, _u64, _f32 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float
_vp = ctypes.c_void_p
_pi64 = ctypes.POINTER(ctypes.c_int64)
_pi32 = ctypes.POINTER(ctypes.c_int32)
_pu64 = ctypes.POINTER(ctypes.c_uint64)

# name -> (restype, argtypes); must list every DL_API function of include/diloco_hip.h
SIGNATURES = {
    "dl_plan_tables": (ctypes.c_int, [_pi64, _i32, _i64, _i32, _pi64, _pi64, _pi32]),
    "dl_plan_tables_ex": (ctypes.c_int, [_pi64, _i32, _i64, _i32, _i64, _pi64, _pi64, _pi32]),
    "dl_tree_create": (ctypes.c_int, [_pi64, _i32, _i64, ctypes.POINTER(_vp)]),
    "dl_tree_create_ex": (ctypes.c_int, [_pi64, _i32, _i64, _i64, ctypes.POINTER(_vp)]),
    "dl_tree_destroy": (ctypes.c_int, [_vp]),
    "dl_tree_query": (ctypes.c_int, [_vp, _pi64, _pi32, _pi32, _pi32]),
    "dl_tree_bucket_range": (ctypes.c_int, [_vp, _i32, _pi64, _pi64]),
    "dl_tree_seg_off": (ctypes.c_int, [_vp, _pi64]),
    "dl_tree_bucket_chunks": (ctypes.c_int, [_vp, _i32, _pi32, _pi32]),
    "dl_tree_bind": (ctypes.c_int, [_vp, _i32, _pu64, _i32, _vp]),
    "dl_tree_tune": (ctypes.c_int, [_vp, _i32, _i32]),
    "dl_tuning_build": (ctypes.c_int, []),
    "dl_delta_pack": (ctypes.c_int, [_vp, _i32, _i32, _vp, _vp, _i32, _vp]),
    "dl_unpack_avg": (ctypes.c_int, [_vp, _i32, _vp, _i32, _i32, _i32, _vp, _vp]),
    "dl_unpack_sgd": (
        ctypes.c_int,
        [_vp, _i32, _vp, _i32, _i32, _vp, _vp, _f32, _f32, _i32, _i32, _i32, _vp],
    ),
    "dl_delta_sgd": (ctypes.c_int, [_vp, _i32, _i32, _vp, _vp, _f32, _f32, _i32, _i32, _vp]),
    "dl_delta_pack_sgd": (
        ctypes.c_int, [_vp, _i32, _i32, _vp, _vp, _i32, _vp, _f32, _f32, _i32, _i32, _vp],
    ),
    "dl_pack_sgd_tiled": (
        ctypes.c_int,
        [_vp, _i32, _i32, _vp, _vp, _i32, _vp, _f32, _f32, _i32, _i32, _i32, _vp],
    ),
    "dl_shard_sgd": (
        ctypes.c_int, [_vp, _i32, _i32, _vp, _vp, _i64, _f32, _f32, _i32, _i32, _vp],
    ),
    "dl_shard_reduce_sgd": (
        ctypes.c_int, [_vp, _i32, _i32, _i64, _vp, _vp, _f32, _f32, _i32, _i32, _vp],
    ),
    "dl_shard_reduce_avg": (ctypes.c_int, [_vp, _i32, _i32, _i64, _vp, _vp]),
    "dl_delta_q8": (ctypes.c_int, [_vp, _i32, _i32, _vp, _vp, _vp]),
    "dl_q8_reduce": (ctypes.c_int, [_vp, _i32, _i32, _i32, _vp, _vp]),
    "dl_unpack_sgd_q8": (
        ctypes.c_int, [_vp, _i32, _vp, _vp, _vp, _f32, _f32, _i32, _i32, _i32, _vp],
    ),
    "dl_gather": (ctypes.c_int, [_vp, _i32, _i32, _vp, _i32, _vp]),
    "dl_scatter": (ctypes.c_int, [_vp, _i32, _vp, _i32, _vp]),
    "dl_serialize": (ctypes.c_int, [_vp, _i32, _i64, _f32, _f32, _vp, _vp]),
    "dl_serialize_f64": (ctypes.c_int, [_vp, _i64, _f32, _f32, _vp, _vp]),
    "dl_fill_synth": (ctypes.c_int, [_vp, _i64, _u64, _u64, _f32, _f32, _vp, _vp]),
    "dl_spin": (ctypes.c_int, [_u64, _vp]),
    "dl_rccl_load": (ctypes.c_int, [ctypes.c_char_p]),
    "dl_rccl_version": (ctypes.c_int, [_pi32]),
    "dl_comm_unique_id": (ctypes.c_int, [_vp]),
    "dl_comm_init": (ctypes.c_int, [ctypes.POINTER(_vp), _i32, _vp, _i32]),
    "dl_comm_destroy": (ctypes.c_int, [_vp]),
    "dl_allreduce": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp]),
    "dl_reduce_scatter": (ctypes.c_int, [_vp, _vp, _i64, _i32, _vp, _vp]),
    "dl_all_gather": (ctypes.c_int, [_vp, _vp, _i64, _i32, _vp, _vp]),
    "dl_ipc_handle": (ctypes.c_int, [_vp, _vp, _pi64]),
    "dl_ipc_open": (ctypes.c_int, [_vp, ctypes.POINTER(_vp)]),
    "dl_ipc_close": (ctypes.c_int, [_vp]),
    "dl_can_access_peer": (ctypes.c_int, [_i32, _i32, _pi32]),
    "dl_enable_peer_access": (ctypes.c_int, [_i32]),
    "dl_sys_fence": (ctypes.c_int, [_vp]),
    "dl_sys_fence_census": (ctypes.c_int, [_vp, _i32, _pi32, _vp]),
    "dl_send": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _vp]),
    "dl_recv": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _vp]),
    "dl_group_start": (ctypes.c_int, []),
    "dl_group_end": (ctypes.c_int, []),
    "dl_copy": (ctypes.c_int, [_vp, _vp, _i64, _i32, _vp]),
    "dl_peer_gather": (ctypes.c_int, [_pu64, _i32, _i64, _vp, _vp]),
    "dl_xgmi_reduce_sgd": (
        ctypes.c_int,
        [_pu64, _pu64, _i32, _i32, _i64, _i64, _vp, _f32, _f32, _i32, _i32, _vp],
    ),
    "dl_xgmi_delta_sgd": (
        ctypes.c_int,
        [_pu64, _pu64, _i32, _i32, _i64, _i64, _vp, _f32, _f32, _i32, _i32, _vp],
    ),
    "dl_last_error": (ctypes.c_char_p, []),
    "dl_abi_version": (ctypes.c_int, []),
}


class DilocoHipError(RuntimeError):
    """A libdiloco_hip call failed; `code` is the DL_E_* (<0) or hipError_t (>0) value."""

    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


_lock = threading.Lock()
_lib = None


def load() -> ctypes.CDLL:
    """Load and type the library once; raise loudly if it is absent (no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libdiloco_hip.so not found at {LIB_PATH}; build it with "
                "`make -C diloco-swarm_amd/csrc` (hipcc --offload-arch=gfx950). "
                "There is no CPU fallback for the DiLoCo outer-step path."
            )
        # PyTorch-ROCm bundles its own HIP runtime (torch/lib/libamdhip64.so, soname
        # libamdhip64.so.7). Import torch first so our NEEDED libamdhip64.so.7 binds to that
        # already-loaded runtime: one HIP runtime per process, shared streams and pointers.
        import torch  # noqa: F401

        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.dl_abi_version() != ABI_VERSION:
            raise ImportError(
                f"libdiloco_hip ABI {lib.dl_abi_version()} != expected {ABI_VERSION}; rebuild"
            )
        _lib = lib
        return lib


def call(name: str, *args) -> None:
    """Invoke a status-returning entry point, raising DilocoHipError on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.dl_last_error()
        raise DilocoHipError(name, rc, msg.decode(errors="replace") if msg else "")


def lib_path() -> str:
    return LIB_PATH
