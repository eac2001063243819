"""Runtime properties of the HIP path on the GPU: the cross-GPU fence reaches every XCD, pointer
tables rebind asynchronously and in stream order, and the outer step is unaffected by other
threads' default-stream traffic (the reference's p2p threads call
.to("cpu") concurrently with the outer step, src/comm.py:28,38)."""
import ctypes
import threading

import numpy as np
import pytest
import torch

from conftest import load_npz
from diloco_amd import _lib, synth
from diloco_amd.plan import SLOT_GRAD, PackedTree
from diloco_amd.trees import get_tree

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_sys_fence_reaches_every_xcd():
    """dl_sys_fence launches one workgroup per CU (multiProcessorCount) and every XCD of the
    MI355X (8) runs at least one of them, so the L2 write-back + invalidate that orders the
    direct exchange's IPC traffic happens on every XCD (dl_xgmi.hip)."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for _ in range(3):
        ids = torch.full((cus,), 0xFFFF, dtype=torch.int32, device=DEV)
        grid = ctypes.c_int32()
        _lib.call("dl_sys_fence_census", ids.data_ptr(), cus, ctypes.byref(grid),
                  torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert grid.value == cus
        got = ids.cpu().numpy()
        assert (got < 8).all(), "every workgroup recorded its XCD"
        counts = np.bincount(got, minlength=8)
        assert (counts > 0).all() and counts.size == 8, counts.tolist()
    with pytest.raises(_lib.DilocoHipError, match="entries"):
        _lib.call("dl_sys_fence_census", ids.data_ptr(), cus - 1, ctypes.byref(grid),
                  torch.cuda.current_stream().cuda_stream)


def test_rebinding_is_stream_ordered_without_host_sync():
    """Ten pointer sets bound back to back on one stream (more than the 4-slot staging ring),
    each followed by a gather of its tensors, no host synchronisation in between: every
    gather packs exactly the tensors bound just before it."""
    numels = [1, 3, 5000, 64, 4097, 70000, 0, 12345]
    tree = PackedTree(numels, 6000)
    s = torch.cuda.current_stream().cuda_stream
    sets, packed = [], []
    for k in range(10):
        ts = [torch.full((n,), float(k * 100 + i), device=DEV) for i, n in enumerate(numels)]
        out = torch.empty(tree.total, device=DEV)
        tree.bind(SLOT_GRAD, ts, s)
        _lib.call("dl_gather", tree.handle, _lib.ALL_BUCKETS, SLOT_GRAD, out.data_ptr(),
                  _lib.DL_F32, s)
        sets.append(ts)
        packed.append(out)
    torch.cuda.synchronize()
    for k, (ts, out) in enumerate(zip(sets, packed)):
        for i, n in enumerate(numels):
            o = int(tree.seg_off[i])
            assert torch.equal(out[o:o + n], ts[i]), (k, i)
    tree.close()


def test_gradsync_after_zero_grad_set_to_none():
    """The plain-DP sync (src/train.py:249-251) after torch reallocates every .grad
    (zero_grad(set_to_none=True), src/train.py:164): each step rebinds and averages the new
    tensors (identity at one peer), in place."""
    from diloco_amd.gradsync import GradSync

    params = [torch.nn.Parameter(torch.zeros(n, device=DEV)) for n in (1, 3, 5000, 64, 4097)]
    gs = GradSync(params, None, 1, bucket_cap_elems=4096)
    for step in range(5):
        for p in params:
            p.grad = None
        for i, p in enumerate(params):
            p.grad = torch.full_like(p, float(step * 10 + i))
        gs.sync()
        torch.cuda.synchronize()
        for i, p in enumerate(params):
            assert torch.equal(p.grad, torch.full_like(p, float(step * 10 + i)))
    gs.close()


class _DefaultStreamTraffic:
    """A daemon thread copying a (32, 1024, 768) activation to the host on the default stream,
    in a loop, as the reference's SendThread does (src/comm.py:38)."""

    def __init__(self):
        self.act = torch.randn(32, 1024, 768, device=DEV)
        self.stop = threading.Event()
        self.copies = 0
        self.error = None
        self.t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        try:
            torch.cuda.set_device(0)
            while not self.stop.is_set():
                host = self.act.to("cpu")
                assert host.shape == self.act.shape
                self.copies += 1
        except BaseException as e:  # reported by the test
            self.error = e

    def __enter__(self):
        import time

        self.t.start()
        t0 = time.time()  # the traffic is running before the outer step starts
        while self.copies == 0 and self.error is None and time.time() - t0 < 30:
            time.sleep(0.001)
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.t.join(timeout=60)
        return False


@pytest.mark.parametrize("fuse,side_stream", [(True, None), (True, True), (False, None),
                                              (False, False)])
def test_outer_step_under_concurrent_default_stream_traffic(fuse, side_stream):
    from diloco_amd.outer import OuterSync

    spec = get_tree("micro")
    g = load_npz("micro_n1.npz")
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, DEV), shapes)]
    e = OuterSync(params, world_size=1, fuse_single=fuse, side_stream=side_stream)
    # auto policy: the one-kernel fused step on the caller's stream, the two-kernel step on
    # the engine's side stream
    assert (e.stream is None) == (side_stream is False or (side_stream is None and fuse))
    with _DefaultStreamTraffic() as traffic:
        for s in (1, 2):
            th = [t.reshape(-1) for t in e.unpacked(e.theta)]
            synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in params])
            e.step()
            torch.cuda.current_stream().synchronize()
            got = np.concatenate([p.reshape(-1).cpu().numpy() for p in params])
            assert got.tobytes() == g[f"theta_s{s}"].tobytes(), s
    assert traffic.error is None and traffic.copies > 0
    e.close()


@pytest.mark.parametrize("placement,write_back", [("host", "sync"), ("host", "deferred"),
                                                  ("device", "sync")])
def test_dropin_sequence_under_concurrent_default_stream_traffic(placement, write_back):
    """The reference's four calls (src/train.py:263-269) through the drop-in, while another
    thread keeps copying an activation to the host on the default stream: bit-exact vs the
    reference's own outputs (micro_n1.npz)."""
    import tempfile

    import torch.distributed as dist

    from test_dropin_gpu import _outer_steps

    if not dist.is_initialized():
        f = tempfile.mktemp(prefix="dl_pg_")
        dist.init_process_group("gloo", init_method=f"file://{f}", rank=0, world_size=1)
    g = load_npz("micro_n1.npz")
    with _DefaultStreamTraffic() as traffic:
        rec = _outer_steps(0, 1, placement=placement, write_back=write_back)
    assert traffic.error is None and traffic.copies > 0
    for s in (1, 2):
        assert rec[f"delta_s{s}"].tobytes() == g[f"delta_s{s}_r0"].tobytes()
        assert rec[f"theta_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()
        assert rec[f"buf_s{s}"].tobytes() == g[f"buf_s{s}"].tobytes()
        assert rec[f"inner_s{s}"].tobytes() == g[f"theta_s{s}"].tobytes()


@pytest.mark.parametrize("flags", [0, 1, 8, 9])
def test_copy_kernel_copies_exactly(flags):
    """dl_copy (the bench's copy-ceiling kernel and its cache scrub) in every variant: exact
    bytes, partial last workgroup, nothing written past the end."""
    for n16 in (1, 1023, 1024, 2049, 1 << 18):
        src = torch.arange(4 * n16, dtype=torch.float32, device=DEV)
        dst = torch.full((4 * n16 + 64,), -1.0, device=DEV)
        _lib.call("dl_copy", src.data_ptr(), dst.data_ptr(), 16 * n16, flags,
                  torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(dst[:4 * n16], src), (flags, n16)
        assert bool((dst[4 * n16:] == -1.0).all()), (flags, n16)
    with pytest.raises(_lib.DilocoHipError, match="multiple of 16"):
        _lib.call("dl_copy", src.data_ptr(), dst.data_ptr(), 20, flags, None)


@pytest.mark.parametrize("nt", [0, 1])
@pytest.mark.parametrize("streams", [1, 2, 3, 4])
def test_copy_kernel_read_and_write_probes(nt, streams):
    """The read-only and write-only probes of dl_copy over 1-4 streams (bench.py's mix
    ceiling): DL_COPY_READ writes nothing (dst may be NULL); DL_COPY_WRITE sets each 32-bit
    word of dst[0:bytes) to its index and nothing past the end (src may be NULL)."""
    st = torch.cuda.current_stream().cuda_stream
    f = nt | _lib.COPY_STREAMS(streams)
    for per16 in (1, 1023, 1024, 2049, 1 << 16):
        n16 = per16 * streams
        src = torch.arange(4 * n16, dtype=torch.float32, device=DEV)
        dst = torch.full((4 * n16 + 64,), -1.0, device=DEV)
        _lib.call("dl_copy", src.data_ptr(), dst.data_ptr(), 16 * n16, f | _lib.COPY_READ, st)
        _lib.call("dl_copy", src.data_ptr(), None, 16 * n16, f | _lib.COPY_READ, st)
        torch.cuda.synchronize()
        assert bool((dst == -1.0).all()), (nt, streams, per16)
        _lib.call("dl_copy", None, dst.data_ptr(), 16 * n16, f | _lib.COPY_WRITE, st)
        torch.cuda.synchronize()
        idx = torch.arange(4 * n16, dtype=torch.int32, device=DEV)
        assert torch.equal(dst[:4 * n16].view(torch.int32), idx), (nt, streams, per16)
        assert bool((dst[4 * n16:] == -1.0).all()), (nt, streams, per16)
    with pytest.raises(_lib.DilocoHipError, match="together"):
        _lib.call("dl_copy", src.data_ptr(), dst.data_ptr(), 16 * streams,
                  f | _lib.COPY_READ | _lib.COPY_WRITE, None)
    if streams > 1:
        with pytest.raises(_lib.DilocoHipError, match="streams"):
            _lib.call("dl_copy", src.data_ptr(), None, 16 * streams + 16, f | _lib.COPY_READ,
                      None)
        with pytest.raises(_lib.DilocoHipError, match="needs a probe"):
            _lib.call("dl_copy", src.data_ptr(), dst.data_ptr(), 16 * streams, f, None)


def test_outer_step_called_on_the_engines_own_stream():
    """A caller already running on the engine's stream (e.g. a loop that does all its outer
    work under `torch.cuda.stream(engine.stream)`) skips the stream joins; results stay
    bit-exact against the reference (micro_n1.npz)."""
    from diloco_amd.outer import OuterSync

    spec = get_tree("micro")
    g = load_npz("micro_n1.npz")
    shapes = [s for _, s in spec.params()]
    params = [t.view(s) for t, s in zip(synth.outer_tree_device(spec, DEV), shapes)]
    e = OuterSync(params, world_size=1, fuse_single=True, keep_wire=True, side_stream=True)
    assert e.stream is not None
    with torch.cuda.stream(e.stream):
        for s in (1, 2):
            th = [t.reshape(-1) for t in e.unpacked(e.theta)]
            synth.inner_tree_device(th, s, 0, out=[p.view(-1) for p in params])
            e.step()
    torch.cuda.synchronize()
    got = np.concatenate([p.reshape(-1).cpu().numpy() for p in params])
    assert got.tobytes() == g["theta_s2"].tobytes()
    e.close()


def test_dl_spin_holds_the_stream_for_its_duration():
    """dl_spin, the slow producer of the ordering tests: a kernel after it on the same stream
    starts only once the requested time has passed on the device clock (events around it),
    and the host is not held (the call returns at once)."""
    import time

    s = torch.cuda.current_stream()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t = time.perf_counter()
    _lib.call("dl_spin", 150_000_000, s.cuda_stream)  # 150 ms
    issued = time.perf_counter() - t
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1)
    assert 140.0 <= ms <= 400.0, ms
    assert issued < 0.05
    with pytest.raises(_lib.DilocoHipError, match="10 s"):
        _lib.call("dl_spin", 11_000_000_000, s.cuda_stream)
