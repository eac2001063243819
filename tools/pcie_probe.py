#!/usr/bin/env python3
"""PCIe rates of the host placement's transfers: one packed T125-size arena
(498 MB) device -> pinned host and back, as the HostOuterMirror issues them (torch copy_,
i.e. the SDMA engines), split over 2 / 4 streams, three arenas at once (the deferred
write-back's batch), and written / read by a kernel (dl_copy over the pinned buffer's
device address: shader stores / loads across PCIe instead of the DMA engines). Diagnostic."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "diloco-swarm_amd"))

import torch  # noqa: E402

from diloco_amd import _lib  # noqa: E402

N = 124475904  # T125 params
REPS = 5


def timed(fn, streams):
    cur = torch.cuda.current_stream()
    best = 1e9
    for _ in range(REPS + 1):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        for s in streams:
            s.wait_stream(cur)
        fn()
        for s in streams:
            cur.wait_stream(s)
        e1.record(cur)
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


def main():
    lib = _lib.load()
    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.device("cuda", 0)
    d = [torch.randn(N, device=dev) for _ in range(3)]
    h = [torch.empty(N, pin_memory=True) for _ in range(3)]
    nbytes = 4 * N
    ss = [torch.cuda.Stream() for _ in range(4)]
    out = {}

    def split(dst, src, k):
        c = N // k
        for i in range(k):
            with torch.cuda.stream(ss[i]):
                hi = N if i == k - 1 else (i + 1) * c
                dst[i * c:hi].copy_(src[i * c:hi], non_blocking=True)

    for k in (1, 2, 4):
        ms = timed(lambda: split(h[0], d[0], k), ss[:k])
        out[f"d2h_copy_{k}stream"] = nbytes / ms / 1e6
        ms = timed(lambda: split(d[0], h[0], k), ss[:k])
        out[f"h2d_copy_{k}stream"] = nbytes / ms / 1e6

    def three():
        for i in range(3):
            with torch.cuda.stream(ss[i]):
                h[i].copy_(d[i], non_blocking=True)
    ms = timed(three, ss[:3])
    out["d2h_three_arenas_3streams"] = 3 * nbytes / ms / 1e6

    dptr = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(dptr), ctypes.c_void_p(h[0].data_ptr()), 0)
    if rc == 0 and dptr.value:
        s = torch.cuda.current_stream().cuda_stream
        for name, flags in (("plain", 0), ("nt", 1)):
            ms = timed(lambda: _lib.call("dl_copy", d[0].data_ptr(), dptr.value, nbytes, flags, s), [])
            out[f"d2h_kernel_{name}"] = nbytes / ms / 1e6
            ok = torch.equal(h[0], d[0].cpu())
            out[f"d2h_kernel_{name}_ok"] = bool(ok)
            ms = timed(lambda: _lib.call("dl_copy", dptr.value, d[1].data_ptr(), nbytes, flags, s), [])
            out[f"h2d_kernel_{name}"] = nbytes / ms / 1e6
    else:
        out["kernel_variants"] = f"hipHostGetDevicePointer rc={rc}"
    for k, v in out.items():
        print(f"{k:32s} {v:.2f}" if isinstance(v, float) else f"{k:32s} {v}")


if __name__ == "__main__":
    main()
