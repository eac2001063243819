"""Checker backend for CPU tests: the engines' kernel interface implemented with the oracle.

TEST INFRASTRUCTURE. Installed only by tests (diloco_amd.kernels.set_default_kernels) so the
engines' orchestration -- buckets, pipelining over a real gloo process group, /n, optimizer
state, host coherence -- runs on CPU tensors at world_size 2 and 4. Every elementwise step is
the C oracle (oracle/diloco_oracle.c); the packed layout comes from the product's host-only
planner (dl_plan_tables), whose tables are pinned separately.
"""
import numpy as np
import torch

from diloco_amd.plan import plan_tables
from oracle import oracle


class CpuTree:
    def __init__(self, numels, cap, bucket_align=64):
        self.numels = [int(n) for n in numels]
        self.bucket_align = bucket_align
        seg, bnd = plan_tables(self.numels, cap, bucket_align_elems=bucket_align)
        self.seg_off = seg
        self.bounds = bnd
        self.total = int(seg[-1])
        self.n_seg = len(self.numels)
        self.n_buckets = len(bnd) - 1
        self.n_chunks = 0
        self.bucket_ranges = [(int(seg[bnd[b]]), int(seg[bnd[b + 1]])) for b in range(self.n_buckets)]
        self.slots = {}
        # chunk table in tree order: (seg, offset in tensor, length, packed offset)
        self.chunks, self.bucket_chunks = [], []
        for b in range(self.n_buckets):
            c0 = len(self.chunks)
            for i in range(int(bnd[b]), int(bnd[b + 1])):
                for o, n in oracle.chunks_of(self.numels[i]):
                    self.chunks.append((i, o, n, int(seg[i]) + o))
            self.bucket_chunks.append((c0, len(self.chunks)))

    def segs(self, bucket):
        if bucket == -1:
            return range(self.n_seg)
        return range(int(self.bounds[bucket]), int(self.bounds[bucket + 1]))

    def close(self):
        pass


def _np(t):
    return t.detach().numpy()


class OracleKernels:
    name = "oracle"
    default_device = torch.device("cpu")
    # the engines treat host tensors as "device" tensors under this backend, so the mirror /
    # engine orchestration runs on CPU (diloco_amd.utils.device_path)
    accepts_host_tensors = True

    def check_device(self, device):
        assert device.type == "cpu"

    def tree(self, numels, device, cap_elems=64 << 20, bucket_align=64):
        return CpuTree(numels, cap_elems, bucket_align)

    def bind(self, tree, slot, tensors, device, key=None):
        tree.slots[slot] = [t.detach().reshape(-1) for t in tensors]

    def _seg(self, tree, packed, i):
        o = int(tree.seg_off[i])
        return _np(packed)[o:o + tree.numels[i]]

    def _rd(self, tree, packed, i):
        """Segment i of a packed fp32 or bf16 buffer, as a fresh fp32 array."""
        if packed.dtype == torch.bfloat16:
            o = int(tree.seg_off[i])
            return packed[o:o + tree.numels[i]].float().numpy().copy()
        return self._seg(tree, packed, i).copy()

    def _wr(self, tree, packed, i, x):
        """Store fp32 values into segment i (a bf16 buffer: rounded to nearest even, as the
        kernels' v_cvt_pk_bf16_f32; oracle.bf16_round, exact in bf16 afterwards)."""
        if packed.dtype == torch.bfloat16:
            o = int(tree.seg_off[i])
            packed[o:o + tree.numels[i]] = torch.from_numpy(
                oracle.bf16_round(np.ascontiguousarray(x, dtype=np.float32))).to(torch.bfloat16)
        else:
            self._seg(tree, packed, i)[:] = x

    def delta_pack(self, tree, bucket, inner_slot, theta, wire):
        for i in tree.segs(bucket):
            d = oracle.delta(np.ascontiguousarray(self._seg(tree, theta, i)),
                             _np(tree.slots[inner_slot][i]).copy())
            self._wr(tree, wire, i, d)

    def unpack_sgd(self, tree, bucket, wire, divisor, theta, mom, lr, momentum, nesterov, first,
                   inner_slot):
        for i in tree.segs(bucket):
            g = self._rd(tree, wire, i)
            if divisor != 1:
                g = (g / np.float32(divisor)).astype(np.float32)
            th = self._seg(tree, theta, i).copy()
            b = self._seg(tree, mom, i).copy() if mom is not None else None
            oracle.sgd(th, b, g, lr, momentum, nesterov, first)
            self._seg(tree, theta, i)[:] = th
            if mom is not None:
                self._seg(tree, mom, i)[:] = b
            if inner_slot >= 0:
                _np(tree.slots[inner_slot][i])[:] = th

    def pack_sgd_tiled(self, tree, bucket, inner_slot, theta, wire, mom, lr, momentum,
                       nesterov, first, tile_chunks):
        # tiling only changes the launch order of elementwise work: the two whole-range steps
        self.delta_pack(tree, bucket, inner_slot, theta, wire)
        self.unpack_sgd(tree, bucket, wire, 1, theta, mom, lr, momentum, nesterov, first,
                        inner_slot)

    def delta_pack_sgd(self, tree, bucket, inner_slot, theta, wire, mom, lr, momentum,
                       nesterov, first):
        # one pass on the device; restated as the pair it is bit-identical to
        self.delta_pack(tree, bucket, inner_slot, theta, wire)
        self.unpack_sgd(tree, bucket, wire, 1, theta, mom, lr, momentum, nesterov, first,
                        inner_slot)

    def delta_sgd(self, tree, bucket, inner_slot, theta, mom, lr, momentum, nesterov, first):
        for i in tree.segs(bucket):
            th = self._seg(tree, theta, i).copy()
            inner = _np(tree.slots[inner_slot][i])
            g = oracle.delta(th, inner.copy())
            b = self._seg(tree, mom, i).copy() if mom is not None else None
            oracle.sgd(th, b, g, lr, momentum, nesterov, first)
            self._seg(tree, theta, i)[:] = th
            if mom is not None:
                self._seg(tree, mom, i)[:] = b
            inner[:] = th

    def shard_sgd(self, wire, divisor, theta, mom, lr, momentum, nesterov, first):
        g = _np(wire).astype(np.float32)
        if divisor != 1:
            g = (g / np.float32(divisor)).astype(np.float32)
        th = _np(theta).copy()
        b = _np(mom).copy() if mom is not None else None
        oracle.sgd(th, b, np.ascontiguousarray(g), lr, momentum, nesterov, first)
        _np(theta)[:] = th
        if mom is not None:
            _np(mom)[:] = b

    def shard_reduce_sgd(self, slices, n_slices, theta, mom, lr, momentum, nesterov, first):
        """Σ over the n slices in rank order, /n (oracle/or_sum_avg), then the shard's SGD."""
        assert slices.dtype == torch.float32
        L, s = theta.numel(), _np(slices)
        g = oracle.sum_avg([np.ascontiguousarray(s[q * L:(q + 1) * L]) for q in range(n_slices)])
        th = _np(theta).copy()
        b = _np(mom).copy() if mom is not None else None
        oracle.sgd(th, b, g, lr, momentum, nesterov, first)
        _np(theta)[:] = th
        if mom is not None:
            _np(mom)[:] = b

    def shard_reduce_avg(self, slices, n_slices, out):
        assert slices.dtype == torch.float32
        L, s = out.numel(), _np(slices)
        _np(out)[:] = oracle.sum_avg([np.ascontiguousarray(s[q * L:(q + 1) * L])
                                      for q in range(n_slices)])

    def _chunk_range(self, tree, bucket):
        return (0, len(tree.chunks)) if bucket == -1 else tree.bucket_chunks[bucket]

    def sys_fence(self, device=None):
        pass  # host memory: nothing to order

    def delta_q8(self, tree, bucket, inner_slot, theta, slots):
        c0, c1 = self._chunk_range(tree, bucket)
        th, q = _np(theta), _np(slots)
        for c in range(c0, c1):
            seg, o, n, po = tree.chunks[c]
            inner = _np(tree.slots[inner_slot][seg])[o:o + n]
            j = (c - c0) * oracle.Q8_SLOT
            oracle.load().or_delta_q8(oracle._fp(np.ascontiguousarray(th[po:po + n])),
                                      oracle._fp(np.ascontiguousarray(inner)), n,
                                      oracle._u8(q[j:j + oracle.Q8_SLOT]))

    def q8_reduce(self, recv, n_peers, n_slots, divisor, out):
        res = oracle.q8_reduce(_np(recv).copy(), n_peers, n_slots, divisor)
        _np(out)[:res.size] = res

    def unpack_sgd_q8(self, tree, bucket, slots, theta, mom, lr, momentum, nesterov, first,
                      inner_slot):
        c0, c1 = self._chunk_range(tree, bucket)
        q = _np(slots)
        for c in range(c0, c1):
            seg, o, n, po = tree.chunks[c]
            j = (c - c0) * oracle.Q8_SLOT
            g = np.empty(n, dtype=np.float32)
            oracle.load().or_q8_deq(oracle._u8(q[j:j + oracle.Q8_SLOT]), n, oracle._fp(g))
            th = _np(theta)[po:po + n].copy()
            b = _np(mom)[po:po + n].copy() if mom is not None else None
            oracle.sgd(th, b, g, lr, momentum, nesterov, first)
            _np(theta)[po:po + n] = th
            if mom is not None:
                _np(mom)[po:po + n] = b
            if inner_slot >= 0:
                _np(tree.slots[inner_slot][seg])[o:o + n] = th

    def unpack_avg(self, tree, bucket, wire, divisor, dst_slot, dst_packed=None):
        for i in tree.segs(bucket):
            g = self._rd(tree, wire, i)
            if divisor != 1:
                g = (g / np.float32(divisor)).astype(np.float32)
            if dst_slot >= 0:
                _np(tree.slots[dst_slot][i])[:] = g
            else:
                self._seg(tree, dst_packed, i)[:] = g

    def gather(self, tree, bucket, src_slot, packed):
        for i in tree.segs(bucket):
            self._wr(tree, packed, i, _np(tree.slots[src_slot][i]))

    def scatter(self, tree, bucket, packed, dst_slot):
        for i in tree.segs(bucket):
            _np(tree.slots[dst_slot][i])[:] = self._seg(tree, packed, i)
