"""Maximum sizes: a tree whose packed space runs past 2^31 elements (8.6 GB per fp32 buffer).

Offsets beyond the 32-bit range are where an index type narrowed anywhere on the path would
show. The tree is [5, 2^31 + 12295, 4099] elements: the middle tensor is larger than the
bucket cap (its own bucket, SURVEY §8c5 "maximum sizes") and 16-B aligned (vector path); the
last one is an unaligned view (the scalar path) whose packed offset lies beyond 2^31. Two outer
steps of the one-replica fused step that keeps the pseudo-gradient (the bench headline's
kernel, dl_delta_pack_sgd), of the tiled two-kernel step with the bf16 wire and of the int8
codec's step, plus the per-step DP gradient sync's gather / unpack round trip, compared bit-exact
against the C oracle on windows at the start, across the 2^31 boundary, at the end of the big
tensor and over both small tensors (the step is elementwise, so a window's oracle is the
oracle of the whole tensor restricted to it). About 45 GB of HBM at the peak."""
import numpy as np
import pytest
import torch

from diloco_amd.outer import OuterSync
from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
BIG = (1 << 31) + 12295
HALF_W = 1 << 15


def _windows(n):
    """(lo, hi) windows of a tensor of n elements covering the places an overflow would hit;
    every lo is a multiple of the 4096-element chunk (the int8 codec scales per chunk)."""
    if n <= 4 * HALF_W:
        return [(0, n)]
    b = 1 << 31
    return [(0, 2 * HALF_W), (b - HALF_W, min(n, b + HALF_W)),
            ((n - 2 * HALF_W) // 4096 * 4096, n)]


def _params():
    g = torch.Generator(device=DEV)
    g.manual_seed(7)
    t0 = torch.randn(5, device=DEV, generator=g) * 0.02
    t1 = torch.randn(BIG, device=DEV, generator=g) * 0.02
    base = torch.randn(4099 + 1, device=DEV, generator=g) * 0.02
    t2 = base[1:]  # 4-B offset: not 16-B aligned
    assert t2.data_ptr() % 16 != 0 and t1.data_ptr() % 16 == 0
    return [t0, t1, t2]


def _perturb(params, step):
    """inner = θ + 1e-3·N(0,1), in place (the stand-in for H inner steps)."""
    g = torch.Generator(device=DEV)
    g.manual_seed(1000 + step)
    for p in params:
        p.add_(torch.randn(p.shape, device=DEV, generator=g), alpha=1e-3)


def _win(t, lo, hi):
    return t.detach().reshape(-1)[lo:hi].cpu().numpy().copy()


def _q8_step(st, inner):
    """The oracle's one-replica int8 step on one chunk-aligned window (state updated)."""
    d = oracle.delta(st.theta[0], inner)
    nch = len(oracle.chunks_of(d.size))
    g = oracle.q8_average([[d]], [d.size], [nch])[0]
    first = st.steps == 0
    if st.buf[0] is None:
        st.buf[0] = np.empty_like(st.theta[0])
    oracle.sgd(st.theta[0], st.buf[0], g, st.lr, st.momentum, st.nesterov, first)
    st.steps += 1
    return d


@pytest.mark.parametrize("variant", ["fused_keep_wire", "two_kernel_bf16", "int8"])
def test_packed_offsets_beyond_2_31(variant):
    free, _total = torch.cuda.mem_get_info()
    if free < 60 << 30:
        pytest.skip(f"needs ~45 GB of free HBM, {free >> 30} GiB free")
    params = _params()
    if variant == "fused_keep_wire":
        e = OuterSync(params, world_size=1, fuse_single=True, keep_wire=True)
        wire = "f32"
    elif variant == "two_kernel_bf16":
        e = OuterSync(params, world_size=1, fuse_single=False, wire_dtype=torch.bfloat16)
        wire = "bf16"
    else:  # one bucket per launch: the int8 exchange works bucket by bucket
        e = OuterSync(params, world_size=1, wire_dtype=torch.int8)
        wire = "int8"
    assert e.tree.total > (1 << 31) and int(e.tree.seg_off[2]) > (1 << 31)
    assert e.tree.n_buckets >= 2  # the big tensor exceeds the cap: a bucket of its own
    wins = [_windows(p.numel()) for p in params]
    # the oracle state on every window, θ_0 = the inner params before the first step
    states = [[oracle.OuterState([_win(p, lo, hi)]) for lo, hi in ws]
              for p, ws in zip(params, wins)]
    for step in (1, 2):
        _perturb(params, step)
        inner = [[_win(p, lo, hi) for lo, hi in ws] for p, ws in zip(params, wins)]
        e.step()
        torch.cuda.synchronize()
        theta = e.unpacked(e.theta)
        mom = e.unpacked(e.mom)
        wire_t = e.unpacked(e.wire.float()) if e.wire is not None else None
        for i, ws in enumerate(wins):
            for k, (lo, hi) in enumerate(ws):
                st = states[i][k]
                if wire == "int8":
                    _q8_step(st, inner[i][k])
                else:
                    deltas, _avg = st.step([[inner[i][k]]], wire=wire)
                where = f"step {step} tensor {i} [{lo}, {hi})"
                got = _win(theta[i], lo, hi)
                assert got.tobytes() == st.theta[0].tobytes(), where
                assert _win(params[i], lo, hi).tobytes() == got.tobytes(), where + " inner"
                assert _win(mom[i], lo, hi).tobytes() == st.buf[0].tobytes(), where + " mom"
                if variant == "fused_keep_wire":
                    assert _win(wire_t[i], lo, hi).tobytes() == deltas[0][0].tobytes(), where
    e.close()
    del e, params
    torch.cuda.empty_cache()


def test_gradsync_round_trip_beyond_2_31():
    """GradSync (dl_gather -> identity exchange -> dl_unpack_avg) at one replica over the same
    tree: every gradient comes back bit-identical (x / 1 is exact), windows checked."""
    from diloco_amd.gradsync import GradSync

    free, _total = torch.cuda.mem_get_info()
    if free < 60 << 30:
        pytest.skip(f"needs ~30 GB of free HBM, {free >> 30} GiB free")
    params = [torch.nn.Parameter(p) for p in _params()]
    for p in params:
        p.grad = torch.randn_like(p)
    wins = [_windows(p.numel()) for p in params]
    want = [[_win(p.grad, lo, hi) for lo, hi in ws] for p, ws in zip(params, wins)]
    gs = GradSync(params, None, 1)
    assert gs.tree.total > (1 << 31)
    gs.sync()
    torch.cuda.synchronize()
    for i, ws in enumerate(wins):
        for k, (lo, hi) in enumerate(ws):
            assert _win(params[i].grad, lo, hi).tobytes() == want[i][k].tobytes(), (i, lo)
            # and the packed wire holds them at their packed offsets
            o = int(gs.tree.seg_off[i])
            assert _win(gs.wire, o + lo, o + hi).tobytes() == want[i][k].tobytes(), (i, lo)
    gs.close()
    del gs, params
    torch.cuda.empty_cache()


class _Cfg:
    def __init__(self, **kw):
        self.__dict__.update(kw)


@pytest.mark.parametrize("placement", ["device", None])
def test_dropin_calls_beyond_2_31(placement):
    """The reference's four calls (src/train.py:263-269) over the same tree: get_outer_model on
    the device placement and on the default lazy host one (pinned host arenas of 8.6 GB each,
    one DMA per read), get_optimizer's OuterSGD, one peer. Two outer steps; θ, .grad, the
    momentum (opt.state) and the inner params bit-exact against the C oracle on the windows."""
    from diloco_amd.comm import TrainingComm
    from diloco_amd.utils import (compute_pseudo_gradient, get_optimizer, get_outer_model,
                                  sync_inner_model)
    from diloco_amd.world import World
    import tempfile
    import torch.distributed as dist

    free, _total = torch.cuda.mem_get_info()
    if free < 80 << 30:
        pytest.skip(f"needs ~50 GB of free HBM, {free >> 30} GiB free")
    if not dist.is_initialized():
        dist.init_process_group("gloo", init_method="file://" + tempfile.mktemp(prefix="dl_pg_"),
                                rank=0, world_size=1)
    inner = torch.nn.Module()
    inner.ps = torch.nn.ParameterList([torch.nn.Parameter(p) for p in _params()])
    outer = get_outer_model(inner, placement)
    opt = get_optimizer(outer, _Cfg(type="SGD", lr=0.7, momentum=0.9, nesterov=True))
    comm = TrainingComm(World.from_default_group(1), (1, 1, 8), None)
    params = list(inner.parameters())
    wins = [_windows(p.numel()) for p in params]
    states = [[oracle.OuterState([_win(p, lo, hi)]) for lo, hi in ws]
              for p, ws in zip(params, wins)]
    for step in (1, 2):
        with torch.no_grad():
            _perturb(params, step)
        inner_w = [[_win(p, lo, hi) for lo, hi in ws] for p, ws in zip(params, wins)]
        compute_pseudo_gradient(inner, outer)
        comm.sync_gradients(outer)
        opt.step()
        sync_inner_model(outer, inner)
        torch.cuda.synchronize()
        ops = list(outer.parameters())
        for i, ws in enumerate(wins):
            for k, (lo, hi) in enumerate(ws):
                st = states[i][k]
                deltas, avg = st.step([[inner_w[i][k]]])
                where = f"{placement} step {step} tensor {i} [{lo}, {hi})"
                got = _win(ops[i].detach(), lo, hi)
                assert got.tobytes() == st.theta[0].tobytes(), where
                assert _win(params[i].detach(), lo, hi).tobytes() == got.tobytes(), where
                assert _win(ops[i].grad, lo, hi).tobytes() == avg[0].tobytes(), where + " grad"
                buf = opt.state[ops[i]]["momentum_buffer"]
                assert _win(buf, lo, hi).tobytes() == st.buf[0].tobytes(), where + " mom"
    outer._diloco_mirror.close()
    del outer, opt, inner, params
    torch.cuda.empty_cache()
