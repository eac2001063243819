"""The C-ABI library loads without a GPU, exports every symbol include/diloco_hip.h declares,
its host-only planner matches the frozen tables, and GPU entry points fail loudly here."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO, load_json
from diloco_amd import _lib
from diloco_amd.plan import plan_tables
from diloco_amd.trees import get_tree

HEADER = os.path.join(REPO, "include", "diloco_hip.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"DL_API\s+[\w\s\*]+?\b(dl_\w+)\s*\(", src)))


def test_header_declares_the_abi():
    syms = declared_symbols()
    assert "dl_delta_pack" in syms and "dl_unpack_sgd" in syms and len(syms) >= 17


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    assert sorted(_lib.SIGNATURES) == declared_symbols()
    assert lib.dl_abi_version() == _lib.ABI_VERSION


def test_product_library_is_not_the_tuning_build():
    """The shipped libdiloco_hip.so instantiates the AUTO policies only."""
    assert _lib.load().dl_tuning_build() == 0


def test_header_constants_match_python_mirror():
    src = open(HEADER).read()
    consts = dict(re.findall(r"#define (DL_\w+) \(?(-?\d+)\)?", src))
    assert int(consts["DL_TUNE_AUTO"]) == _lib.TUNE_AUTO
    assert (int(consts["DL_TUNE_NT_LOADS"]), int(consts["DL_TUNE_NT_STORES"]),
            int(consts["DL_TUNE_WT_STORES"]), int(consts["DL_TUNE_PAIRS"])) == (
        _lib.TUNE_NT_LOADS, _lib.TUNE_NT_STORES, _lib.TUNE_WT_STORES, _lib.TUNE_PAIRS)
    assert "DL_TUNE_REVERSE" not in consts and "dl_tree_slot" not in src
    assert (int(consts["DL_COPY_WIDE"]), int(consts["DL_COPY_READ"]),
            int(consts["DL_COPY_WRITE"])) == (_lib.COPY_WIDE, _lib.COPY_READ, _lib.COPY_WRITE)
    assert int(consts["DL_ALIGN_ELEMS"]) == _lib.ALIGN_ELEMS
    assert int(consts["DL_CHUNK_ELEMS"]) == _lib.CHUNK_ELEMS
    assert int(consts["DL_MAX_SLOTS"]) == _lib.MAX_SLOTS
    assert int(consts["DL_ABI_VERSION"]) == _lib.ABI_VERSION


def test_c_planner_matches_frozen_tables():
    ref = load_json("plan_tables.json")
    for name in ("micro", "tiny", "t125", "t1.3b"):
        numels = get_tree(name).numels()
        for p in ref[name]["plans"]:
            seg, bnd = plan_tables(numels, p["cap"], p["align"])
            assert seg.tolist() == p["seg_off"], name
            assert bnd.tolist() == p["bkt_bounds"], name
    for e in ref["edge"]:
        seg, bnd = plan_tables(e["numels"], e["cap"], e["align"])
        assert seg.tolist() == e["seg_off"] and bnd.tolist() == e["bkt_bounds"], e


def test_planner_properties_t13b():
    numels = get_tree("t1.3b").numels()
    seg, bnd = plan_tables(numels, 64 << 20)
    assert (seg % 64 == 0).all() and (np.diff(seg) >= np.asarray(numels)).all()
    assert (np.diff(seg) - np.asarray(numels) < 64).all()
    assert bnd[0] == 0 and bnd[-1] == len(numels) and (np.diff(bnd) > 0).all()
    for b in range(len(bnd) - 1):
        size = seg[bnd[b + 1]] - seg[bnd[b]]
        assert size <= 64 << 20 or bnd[b + 1] - bnd[b] == 1


def test_planner_rejects_bad_arguments():
    with pytest.raises(_lib.DilocoHipError):
        plan_tables([1, -2, 3])
    with pytest.raises(_lib.DilocoHipError):
        plan_tables([1], 0, 0)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure mode")
def test_device_entry_points_fail_loudly_without_gpu():
    from diloco_amd.plan import PackedTree

    with pytest.raises(_lib.DilocoHipError) as e:
        PackedTree([10, 20])
    assert "hip" in str(e.value).lower()
    # kernel launches with no device: an error code, never a silent no-op
    with pytest.raises(_lib.DilocoHipError):
        _lib.call("dl_sys_fence", None)
    with pytest.raises(_lib.DilocoHipError):
        _lib.call("dl_shard_sgd", 16, _lib.DL_F32, 1, 32, 48, 4, 0.7, 0.9, 1, 0, None)
    with pytest.raises(_lib.DilocoHipError):
        _lib.call("dl_shard_reduce_sgd", 16, _lib.DL_F32, 2, 4, 32, 48, 0.7, 0.9, 1, 0, None)
    with pytest.raises(_lib.DilocoHipError):
        _lib.call("dl_shard_reduce_avg", 16, _lib.DL_BF16, 3, 8, 32, None)


def test_ordered_reduce_argument_checks():
    """dl_shard_reduce_sgd / _avg reject bad shapes before touching a device."""
    for args, msg in [((16, _lib.DL_F32, 2, 6, 32, 48, 0.7, 0.9, 1, 0, None), "multiple of 4"),
                      ((16, _lib.DL_F32, 0, 8, 32, 48, 0.7, 0.9, 1, 0, None), "n_slices"),
                      ((16, 7, 2, 8, 32, 48, 0.7, 0.9, 1, 0, None), "wire dtype"),
                      ((16, _lib.DL_F32, 2, 8, 36, 48, 0.7, 0.9, 1, 0, None), "aligned"),
                      ((16, _lib.DL_F32, 2, 8, 32, 48, 0.7, 0.0, 1, 0, None), "Nesterov")]:
        with pytest.raises(_lib.DilocoHipError, match=msg):
            _lib.call("dl_shard_reduce_sgd", *args)
    with pytest.raises(_lib.DilocoHipError, match="multiple of 4"):
        _lib.call("dl_shard_reduce_avg", 16, _lib.DL_F32, 2, 5, 32, None)
    _lib.call("dl_shard_reduce_avg", 16, _lib.DL_F32, 2, 0, 32, None)  # empty: no error


def test_missing_library_is_an_import_error(tmp_path, monkeypatch):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(ImportError, match="no CPU fallback"):
        _lib.load()


def test_planner_fuzz_against_oracle_rule():
    """Random trees and caps: the C planner == the oracle's C rule == the Python statement."""
    from hypothesis import given, settings
    from hypothesis import strategies as st

    from oracle import oracle

    @settings(max_examples=300, deadline=None)
    @given(st.lists(st.integers(0, 300_000), max_size=60), st.integers(-1, 400_000),
           st.sampled_from([1, 4, 64, 256]))
    def check(numels, cap, align):
        seg, bnd = plan_tables(numels, cap, align)
        oseg, obnd = oracle.plan_tables(numels, cap, align)
        pseg, pbnd = oracle.plan_tables_py(numels, cap, align)
        assert seg.tolist() == oseg.tolist() == list(pseg)
        assert bnd.tolist() == obnd.tolist() == list(pbnd)

    check()


def test_bucket_aligned_planner_fuzz_and_properties():
    """dl_plan_tables_ex (the sharded step's layout): C planner == oracle C == Python rule; every
    bucket starts at a multiple of bucket_align so it splits into n equal aligned shards; tensors
    never overlap; bucket_align == align reproduces dl_plan_tables exactly."""
    from hypothesis import given, settings
    from hypothesis import strategies as st

    from oracle import oracle

    @settings(max_examples=300, deadline=None)
    @given(st.lists(st.integers(0, 300_000), max_size=60), st.integers(-1, 400_000),
           st.sampled_from([1, 2, 3, 4, 7, 8]))
    def check(numels, cap, peers):
        ba = 64 * peers
        seg, bnd = plan_tables(numels, cap, 64, ba)
        oseg, obnd = oracle.plan_tables(numels, cap, 64, ba)
        pseg, pbnd = oracle.plan_tables_py(numels, cap, 64, ba)
        assert seg.tolist() == oseg.tolist() == list(pseg)
        assert bnd.tolist() == obnd.tolist() == list(pbnd)
        n = len(numels)
        for i in range(n):
            assert seg[i] % 64 == 0 and seg[i] + numels[i] <= seg[i + 1]
        assert seg[n] % ba == 0
        for b in range(len(bnd) - 1):
            lo, hi = seg[bnd[b]], seg[bnd[b + 1]]
            assert lo % ba == 0 and (hi - lo) % ba == 0
        s1, b1 = plan_tables(numels, cap, 64, 64)
        s0, b0 = plan_tables(numels, cap, 64)
        assert s1.tolist() == s0.tolist() and b1.tolist() == b0.tolist()

    check()
    with pytest.raises(_lib.DilocoHipError):
        plan_tables([1, 2], 0, 64, 96)  # not a multiple of align


def test_rccl_entry_points_resolve_and_fail_loudly():
    """The C-ABI's RCCL layer loads RCCL at run time (no GPU needed for that) and reports a bad
    library path or a null communicator as an error, never a crash."""
    from diloco_amd import rccl

    with pytest.raises(_lib.DilocoHipError, match="cannot open"):
        rccl.load("/nonexistent/librccl.so")
    rccl.load(None)
    assert rccl.version() >= 20000  # NCCL_VERSION_CODE of RCCL 2.x
    with pytest.raises(_lib.DilocoHipError, match="null communicator"):
        _lib.call("dl_allreduce", None, 0, _lib.DL_F32, None, None)
    with pytest.raises(_lib.DilocoHipError, match="unsupported dtype"):
        _lib.call("dl_all_gather", None, None, 0, 7, 1, None)
