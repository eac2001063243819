"""IEEE special values through the HIP outer step, against the reference's own torch CPU ops
(src/utils.py:221 torch.sub, src/comm.py:122-123 sum and true division, torch.optim.SGD with
Nesterov as src/utils.py:59-65 builds it, src/utils.py:226 copy), bit for bit.

NaN, ±Inf, ±0, subnormals (the library is built with denormals kept), ±FLT_MAX (whose
difference overflows to Inf) and values whose delta is subnormal are planted at the start of a
chunk, in the < 4-element vector tail, in a tensor with 4-B-aligned storage (the scalar path)
and across a chunk boundary, then two outer steps run through every fp32 path: the one-pass
kernels with and without the kept wire, the two-kernel pair, the emulated two-replica exchange
(Σ then /2) and the sharded step's dl_shard_sgd; and the bf16 wire, whose rounding of the
special values is torch's `.to(torch.bfloat16)`. NaNs compare by position (payloads are not
part of the contract), every other value by its bytes, signed zeros included."""
import numpy as np
import pytest
import torch

from diloco_amd.outer import OuterSync

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
NUMELS = [4096 + 7, 5, 33, 4096 * 2 + 3]
MISALIGNED = 2  # tensor index living at a 4-B offset: the scalar path
F = np.float32
MAXF = float(np.finfo(F).max)
SPECIAL_THETA = [np.nan, np.inf, -np.inf, 0.0, -0.0, 1e-40, -1e-40, MAXF, -MAXF, 1.0, 1e-30,
                 5e-39, -0.0, 2.0, np.inf, 1e-38]
SPECIAL_INNER = [1.0, 1.0, np.inf, -0.0, 0.0, 2e-40, 1e-40, -MAXF, MAXF, np.nan, 1e-30,
                 -5e-39, -0.0, 2.0 + 2 ** -22, -np.inf, 1.1e-38]


def _plant(rng, numel, values):
    x = (rng.standard_normal(numel) * 0.02).astype(F)
    v = np.asarray(values, dtype=F)
    spots = [0, max(0, numel - len(v)), max(0, min(4096 - len(v) // 2, numel - len(v)))]
    for s in spots:  # chunk start, the tail, across the first chunk boundary
        k = min(len(v), numel - s)
        x[s:s + k] = v[:k]
    return x


def _host_tree(seed, values):
    rng = np.random.default_rng(seed)
    return [_plant(rng, n, values) for n in NUMELS]


def _device(host):
    base = torch.zeros(sum(NUMELS) + 64, device=DEV)
    out, at = [], 0
    for i, h in enumerate(host):
        at += 1 if i == MISALIGNED else (-at) % 4  # 16-B aligned except one tensor
        p = base[at:at + h.size]
        p.copy_(torch.from_numpy(h))
        out.append(p)
        at += h.size
    return base, out


def _same(got, ref, what):
    got, ref = np.asarray(got, dtype=F), np.asarray(ref, dtype=F)
    assert np.array_equal(np.isnan(got), np.isnan(ref)), what + ": NaN positions"
    m = ~np.isnan(ref)
    assert got[m].tobytes() == ref[m].tobytes(), what


class _TorchReference:
    """The reference's per-tensor sequence on CPU torch tensors for n replicas."""

    def __init__(self, theta0, wire_bf16=False):
        self.theta = [torch.from_numpy(t.copy()) for t in theta0]
        self.params = [torch.nn.Parameter(t) for t in self.theta]
        self.opt = torch.optim.SGD(self.params, lr=0.7, momentum=0.9, nesterov=True)
        self.wire_bf16 = wire_bf16

    def step(self, inners):
        n = len(inners)
        deltas = []
        with torch.no_grad():
            for i, p in enumerate(self.params):
                ds = [torch.sub(p.data, torch.from_numpy(inn[i])) for inn in inners]
                if self.wire_bf16:
                    ds = [d.to(torch.bfloat16).to(torch.float32) for d in ds]
                deltas.append(ds[0].clone())
                g = ds[0].clone()
                for d in ds[1:]:
                    g += d
                if n > 1:
                    g.div_(n)
                p.grad = g
        self.opt.step()
        return deltas

    def theta_np(self):
        return [p.data.numpy() for p in self.params]

    def mom_np(self):
        return [self.opt.state[p]["momentum_buffer"].numpy() for p in self.params]


@pytest.mark.parametrize("variant", ["fused_keep_wire", "fused", "two_kernel", "replicas_2",
                                     "sharded", "bf16_wire"])
def test_special_values_match_torch(variant):
    theta0 = _host_tree(5, SPECIAL_THETA)
    n = 2 if variant == "replicas_2" else 1
    ref = _TorchReference(theta0, wire_bf16=variant == "bf16_wire")
    kw = dict(world_size=n, bucket_cap_elems=4096)
    kw.update({"fused_keep_wire": dict(fuse_single=True, keep_wire=True),
               "fused": dict(fuse_single=True),
               "two_kernel": dict(fuse_single=False, tile_chunks=0),
               "replicas_2": dict(shard=False),
               "sharded": dict(shard=True),
               "bf16_wire": dict(fuse_single=False, tile_chunks=0,
                                 wire_dtype=torch.bfloat16)}[variant])
    bases, replicas, engines = [], [], []
    for _ in range(n):
        b, ps = _device(theta0)
        bases.append(b)
        replicas.append(ps)
        engines.append(OuterSync(ps, **kw))
    assert replicas[0][MISALIGNED].data_ptr() % 16 != 0
    for step in (1, 2):
        th_now = ref.theta_np()
        inners = []
        for r in range(n):
            pert = _host_tree(100 * step + r, SPECIAL_INNER)
            with np.errstate(invalid="ignore", over="ignore"):  # inf - inf etc. are intended
                inner = [(t + p * F(1e-3)).astype(F) if step == 2 else p
                         for t, p in zip(th_now, pert)]
            inners.append(inner)
            for dst, x in zip(replicas[r], inner):
                dst.copy_(torch.from_numpy(x))
        deltas = ref.step(inners)
        if n == 1:
            engines[0].step()
        else:
            for e in engines:
                e.pseudo_gradient()
            total = engines[0].wire.clone()
            for e in engines[1:]:
                total += e.wire
            for e in engines:
                e.wire.copy_(total)
                e.apply()
                e.steps_done += 1
        torch.cuda.synchronize()
        for r, (e, ps) in enumerate(zip(engines, replicas)):
            th = e.unpacked(e.theta)
            mom = e.unpacked(e.momentum_full())
            for i in range(len(NUMELS)):
                where = f"{variant} step {step} replica {r} tensor {i}"
                _same(th[i].cpu().numpy(), ref.theta_np()[i], where + " theta")
                _same(mom[i].cpu().numpy(), ref.mom_np()[i], where + " momentum")
                _same(ps[i].cpu().numpy(), ref.theta_np()[i], where + " inner")
                if variant in ("fused_keep_wire", "two_kernel"):  # the wire = outer.grad
                    _same(e.unpacked(e.wire)[i].cpu().numpy(), deltas[i].numpy(),
                          where + " wire")
    for e in engines:
        e.close()


def test_special_values_int8_wire_match_oracle():
    """The int8 codec has no reference counterpart: its special-value semantics are the
    oracle's C restatement (oracle/diloco_oracle.c or_delta_q8 / or_q8_reduce / or_q8_deq:
    amax by fmaxf, so NaN is ignored by the scale and quantises to -127; an Inf amax gives
    an Inf scale), matched bit for bit (NaN positions) over two steps."""
    from oracle import oracle

    theta0 = _host_tree(5, SPECIAL_THETA)
    b, ps = _device(theta0)
    e = OuterSync(ps, world_size=1, bucket_cap_elems=4096, wire_dtype=torch.int8)
    st = oracle.OuterState(theta0)
    for step in (1, 2):
        pert = _host_tree(100 * step, SPECIAL_INNER)
        with np.errstate(invalid="ignore", over="ignore"):
            inner = [(t + p * F(1e-3)).astype(F) if step == 2 else p
                     for t, p in zip(st.theta, pert)]
        for dst, x in zip(ps, inner):
            dst.copy_(torch.from_numpy(x))
        deltas = [oracle.delta(st.theta[t], inner[t]) for t in range(len(NUMELS))]
        g = oracle.q8_average([deltas], NUMELS, [c1 - c0 for c0, c1 in e.tree.bucket_chunks])
        for t in range(len(NUMELS)):
            if st.buf[t] is None:
                st.buf[t] = np.empty_like(st.theta[t])
            oracle.sgd(st.theta[t], st.buf[t], g[t], st.lr, st.momentum, st.nesterov, step == 1)
        st.steps += 1
        e.step()
        torch.cuda.synchronize()
        th, mom = e.unpacked(e.theta), e.unpacked(e.mom)
        for t in range(len(NUMELS)):
            where = f"int8 step {step} tensor {t}"
            _same(th[t].cpu().numpy(), st.theta[t], where + " theta")
            _same(mom[t].cpu().numpy(), st.buf[t], where + " momentum")
            _same(ps[t].cpu().numpy(), st.theta[t], where + " inner")
    e.close()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_serializer_widens_every_16_bit_pattern_like_torch(dtype):
    """dl_serialize's payload conversion (src/serializer.py:12-13: torch.cat promotes a bf16 /
    fp16 payload to the fp32 metadata plane's dtype) over ALL 65,536 bit patterns -- NaNs,
    infinities, signed zeros, subnormals -- against torch's own .to(torch.float32)."""
    from diloco_amd.serializer import Serializer

    bits = torch.arange(-32768, 32768, dtype=torch.int32).to(torch.int16)
    x = bits.view(dtype).reshape(256, 256)
    framed = Serializer((256, 256)).serialize(x.to(DEV), (7, 11))
    torch.cuda.synchronize()
    got = framed[1].cpu().numpy()
    ref = x.to(torch.float32).numpy()
    _same(got.reshape(-1), ref.reshape(-1), f"{dtype} payload")
    assert framed[0].reshape(-1)[:2].tolist() == [7.0, 11.0]
