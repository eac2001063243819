// HIP kernels for the DiLoCo outer step on gfx950 (MI355X, CDNA4).
//
// Every hot-path kernel is one "segment walker": a workgroup of 256 lanes (4 waves) takes one
// 16 KiB chunk of one tensor from the chunk table (a wave-uniform scalar load), issues all of
// its 16-B loads for the chunk up front (4 float4 per lane per stream), then computes and
// stores. There are no MFMA and no LDS: the work is elementwise and HBM-bound (DESIGN.md
// "Kernels"), so what matters is full-width coalesced access and enough bytes in flight.
// Default launch: one workgroup per chunk (T125: 30,458 workgroups, ~119 per CU) with
// non-temporal loads -- the fastest shape measured (tools/hbm_bench.hip).
//
// Numerics follow the reference exactly (compiled with -ffp-contract=off and correctly
// rounded fp32 division):
//   delta      : outer - inner                         (src/utils.py:221)
//   average    : sum / n, IEEE true division            (src/comm.py:123)
//   SGD        : torch _single_tensor_sgd as used with nesterov, dampening 0, wd 0
//                buf = buf*m + g (two roundings: mul_ then add_)
//                u   = fma(buf, m, g)   (grad.add(buf, alpha=m): CPU fmadd)
//                θ   = fma(u, -lr, θ)   (param.add_(grad, alpha=-lr))
//   copy-back  : inner = θ                              (src/utils.py:226)
#include "dl_device.h"

namespace dl {
namespace {

// a2: wire = outer - inner
template <typename W>
struct DeltaPack {
  int inner_slot;
  const float* outer;
  W* wire;
  template <bool NTL, int NTS>
  __device__ __forceinline__ void run(const Chunk& ck, int c, void* const* caddr, int nchunk, int tid) const {
    const float* in = slot_ptr<const float>(caddr, nchunk, inner_slot, c);
    const float* th = outer + ck.poff;
    W* w = wire + ck.poff;
    if (aligned16(in)) {
      const int nv = ck.len >> 2;
      float4 a[kUnroll], b[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) {
          a[u] = ldf4<NTL>(th, v);
          b[u] = ldf4<NTL>(in, v);
        }
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) WireIO<W>::template st4<NTS>(w, v, sub4(a[u], b[u]));
      }
      const int i = (nv << 2) + tid;
      if (i < ck.len) WireIO<W>::st1(w, i, th[i] - in[i]);
    } else {
      for (int i = tid; i < ck.len; i += kThreads) WireIO<W>::st1(w, i, th[i] - in[i]);
    }
  }
};

#ifdef DL_TUNING
// Two chunks per workgroup, every load of both issued before the first store: 8 float4 per
// lane per input stream in flight instead of 4 (were the 2-read / 1-write
// kernels latency-bound at 4?). Measured cold and interleaved (profiles/r03_pairs_ab.txt): 2-4 %
// SLOWER than one chunk per workgroup for dl_delta_pack and dl_gather on T125 and T1.3B, with
// SQ_WAIT_ANY up (0.61 -> 0.72) and the DRAM read-credit stalls unchanged (0.058): the reads
// are limited by the memory controller, not by loads in flight. Tuning build only
// (DL_TUNE_PAIRS). A misaligned tensor takes the one-chunk body for both chunks.
template <typename W>
struct DeltaPackPair {
  DeltaPack<W> one;
  template <bool NTL, int NTS>
  __device__ __forceinline__ void run(const Chunk& ck, int c, void* const* caddr, int nchunk, int tid) const {
    one.template run<NTL, NTS>(ck, c, caddr, nchunk, tid);
  }
  template <bool NTL, int NTS>
  __device__ __forceinline__ void run2(const Chunk& k0, int c0, const Chunk& k1, int c1,
                                       void* const* caddr, int nchunk, int tid) const {
    const float* in0 = slot_ptr<const float>(caddr, nchunk, one.inner_slot, c0);
    const float* in1 = slot_ptr<const float>(caddr, nchunk, one.inner_slot, c1);
    if (!aligned16(in0) || !aligned16(in1)) {
      run<NTL, NTS>(k0, c0, caddr, nchunk, tid);
      run<NTL, NTS>(k1, c1, caddr, nchunk, tid);
      return;
    }
    const float* th0 = one.outer + k0.poff;
    const float* th1 = one.outer + k1.poff;
    const int nv0 = k0.len >> 2, nv1 = k1.len >> 2;
    float4 a0[kUnroll], b0[kUnroll], a1[kUnroll], b1[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int v = u * kThreads + tid;
      if (v < nv0) {
        a0[u] = ldf4<NTL>(th0, v);
        b0[u] = ldf4<NTL>(in0, v);
      }
      if (v < nv1) {
        a1[u] = ldf4<NTL>(th1, v);
        b1[u] = ldf4<NTL>(in1, v);
      }
    }
    W* w0 = one.wire + k0.poff;
    W* w1 = one.wire + k1.poff;
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int v = u * kThreads + tid;
      if (v < nv0) WireIO<W>::template st4<NTS>(w0, v, sub4(a0[u], b0[u]));
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int v = u * kThreads + tid;
      if (v < nv1) WireIO<W>::template st4<NTS>(w1, v, sub4(a1[u], b1[u]));
    }
    const int i0 = (nv0 << 2) + tid, i1 = (nv1 << 2) + tid;
    if (i0 < k0.len) WireIO<W>::st1(w0, i0, th0[i0] - in0[i0]);
    if (i1 < k1.len) WireIO<W>::st1(w1, i1, th1[i1] - in1[i1]);
  }
};

#endif  // DL_TUNING

// a3 unpack: dst = wire / d
template <typename W, bool DIV>
struct UnpackAvg {
  const W* wire;
  int dst_slot;
  float* dst_packed;
  float d;
  template <bool NTL, int NTS>
  __device__ __forceinline__ void run(const Chunk& ck, int c, void* const* caddr, int nchunk, int tid) const {
    float* dst = dst_slot >= 0 ? slot_ptr<float>(caddr, nchunk, dst_slot, c) : dst_packed + ck.poff;
    const W* w = wire + ck.poff;
    if (aligned16(dst)) {
      const int nv = ck.len >> 2;
      float4 x[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) x[u] = WireIO<W>::template ld4<NTL>(w, v);
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) stf4<NTS>(dst, v, DIV ? div4(x[u], d) : x[u]);
      }
      const int i = (nv << 2) + tid;
      if (i < ck.len) {
        const float g = WireIO<W>::ld1(w, i);
        dst[i] = DIV ? g / d : g;
      }
    } else {
      for (int i = tid; i < ck.len; i += kThreads) {
        const float g = WireIO<W>::ld1(w, i);
        dst[i] = DIV ? g / d : g;
      }
    }
  }
};

template <typename W, bool DIV, int MODE>
struct UnpackSgd {
  const W* wire;
  float* outer;
  float* mom;
  float d;
  SgdArgs a;
  int inner_slot;
  template <bool NTL, int NTS>
  __device__ __forceinline__ void run(const Chunk& ck, int c, void* const* caddr, int nchunk, int tid) const {
    float* in = inner_slot >= 0 ? slot_ptr<float>(caddr, nchunk, inner_slot, c) : nullptr;
    const W* w = wire + ck.poff;
    float* th = outer + ck.poff;
    float* mb = mom + ck.poff;
    if (in == nullptr || aligned16(in)) {
      const int nv = ck.len >> 2;
      float4 g[kUnroll], t[kUnroll], m[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) {
          g[u] = WireIO<W>::template ld4<NTL>(w, v);
          t[u] = ldf4<NTL>(th, v);
          if (MODE == 2) m[u] = ldf4<NTL>(mb, v);
        }
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const float4 gg = DIV ? div4(g[u], d) : g[u];
        sgd1<MODE>(gg.x, m[u].x, t[u].x, a);
        sgd1<MODE>(gg.y, m[u].y, t[u].y, a);
        sgd1<MODE>(gg.z, m[u].z, t[u].z, a);
        sgd1<MODE>(gg.w, m[u].w, t[u].w, a);
      }
      store_rows<NTS>(th, t, nv, tid);
      if (MODE != 0) store_rows<NTS>(mb, m, nv, tid);
      if (in) store_rows<NTS>(in, t, nv, tid);
      const int i = (nv << 2) + tid;
      if (i < ck.len) {
        float gg = WireIO<W>::ld1(w, i);
        if (DIV) gg = gg / d;
        float b = (MODE == 2) ? mb[i] : 0.f, t1 = th[i];
        sgd1<MODE>(gg, b, t1, a);
        th[i] = t1;
        if (MODE != 0) mb[i] = b;
        if (in) in[i] = t1;
      }
    } else {
      for (int i = tid; i < ck.len; i += kThreads) {
        float gg = WireIO<W>::ld1(w, i);
        if (DIV) gg = gg / d;
        float b = (MODE == 2) ? mb[i] : 0.f, t1 = th[i];
        sgd1<MODE>(gg, b, t1, a);
        th[i] = t1;
        if (MODE != 0) mb[i] = b;
        in[i] = t1;
      }
    }
  }
};

// a2+a4+a5 at ONE peer (src/comm.py:118-119: no all-reduce, no division): the delta never
// leaves registers. g = θ - inner; SGD; θ and inner <- θ'. 24 B/param (20 first step)
// instead of 12 + 24 for delta_pack + unpack_sgd; results are bit-identical to that pair.
template <int MODE>
struct DeltaSgd {
  float* outer;
  float* mom;
  SgdArgs a;
  int inner_slot;
  template <bool NTL, int NTS>
  __device__ __forceinline__ void run(const Chunk& ck, int c, void* const* caddr, int nchunk, int tid) const {
    float* in = slot_ptr<float>(caddr, nchunk, inner_slot, c);
    float* th = outer + ck.poff;
    float* mb = mom + ck.poff;
    if (aligned16(in)) {
      const int nv = ck.len >> 2;
      float4 x[kUnroll], t[kUnroll], m[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) {
          t[u] = ldf4<NTL>(th, v);
          x[u] = ldf4<NTL>(in, v);
          if (MODE == 2) m[u] = ldf4<NTL>(mb, v);
        }
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const float4 g = sub4(t[u], x[u]);
        sgd1<MODE>(g.x, m[u].x, t[u].x, a);
        sgd1<MODE>(g.y, m[u].y, t[u].y, a);
        sgd1<MODE>(g.z, m[u].z, t[u].z, a);
        sgd1<MODE>(g.w, m[u].w, t[u].w, a);
      }
      store_rows<NTS>(th, t, nv, tid);
      if (MODE != 0) store_rows<NTS>(mb, m, nv, tid);
      store_rows<NTS>(in, t, nv, tid);
      const int i = (nv << 2) + tid;
      if (i < ck.len) {
        const float g = th[i] - in[i];
        float b = (MODE == 2) ? mb[i] : 0.f, t1 = th[i];
        sgd1<MODE>(g, b, t1, a);
        th[i] = t1;
        if (MODE != 0) mb[i] = b;
        in[i] = t1;
      }
    } else {
      for (int i = tid; i < ck.len; i += kThreads) {
        const float g = th[i] - in[i];
        float b = (MODE == 2) ? mb[i] : 0.f, t1 = th[i];
        sgd1<MODE>(g, b, t1, a);
        th[i] = t1;
        if (MODE != 0) mb[i] = b;
        in[i] = t1;
      }
    }
  }
};

// a2+a3+a4+a5 at ONE peer with the pseudo-gradient kept: dl_delta_sgd that also stores the
// packed wire (outer.grad of src/utils.py:221, the reference's observable .grad after the
// step). g = θ - inner; wire = W(g); the SGD consumes the value on the wire (a bf16 wire
// rounds it first, as dl_unpack_sgd would read it back); θ, buf, inner <- new values.
// 28 B/param (fp32 wire; 24 on the first step) instead of 12 + 24 for dl_delta_pack +
// dl_unpack_sgd: the wire and θ are not read back. Bit-identical to that pair.
template <typename W, int MODE>
struct DeltaPackSgd {
  float* outer;
  W* wire;
  float* mom;
  SgdArgs a;
  int inner_slot;
  static __device__ __forceinline__ float on_wire(float g) {
    if constexpr (sizeof(W) == 2) return bf2f(f2bf(g));
    else return g;
  }
  template <bool NTL, int NTS>
  __device__ __forceinline__ void run(const Chunk& ck, int c, void* const* caddr, int nchunk, int tid) const {
    float* in = slot_ptr<float>(caddr, nchunk, inner_slot, c);
    float* th = outer + ck.poff;
    float* mb = mom + ck.poff;
    W* w = wire + ck.poff;
    if (aligned16(in)) {
      const int nv = ck.len >> 2;
      float4 x[kUnroll], t[kUnroll], m[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) {
          t[u] = ldf4<NTL>(th, v);
          x[u] = ldf4<NTL>(in, v);
          if (MODE == 2) m[u] = ldf4<NTL>(mb, v);
        }
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) x[u] = sub4(t[u], x[u]);  // the pseudo-gradient
      // Store order of the four output streams (DL_DPS_ORDER, tools/store_order_ab.py; the
      // product build is 0): 0 = the SGD arithmetic, then wire, θ, momentum, inner, each
      // stream's rows back to back; 1 = the wire rows issued before the SGD arithmetic;
      // 2 = row by row across the four streams; 3 = inner, momentum, θ, wire.
#if DL_DPS_ORDER == 1
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) WireIO<W>::template st4<DL_DPS_WIRE_NTS(NTS)>(w, v, x[u]);
      }
#endif
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const float4 g = make_float4(on_wire(x[u].x), on_wire(x[u].y), on_wire(x[u].z),
                                     on_wire(x[u].w));
        sgd1<MODE>(g.x, m[u].x, t[u].x, a);
        sgd1<MODE>(g.y, m[u].y, t[u].y, a);
        sgd1<MODE>(g.z, m[u].z, t[u].z, a);
        sgd1<MODE>(g.w, m[u].w, t[u].w, a);
      }
#if DL_DPS_ORDER == 2
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) {
          WireIO<W>::template st4<DL_DPS_WIRE_NTS(NTS)>(w, v, x[u]);
          stf4<NTS>(th, v, t[u]);
          if (MODE != 0) stf4<NTS>(mb, v, m[u]);
          stf4<NTS>(in, v, t[u]);
        }
      }
#elif DL_DPS_ORDER == 3
      store_rows<NTS>(in, t, nv, tid);
      if (MODE != 0) store_rows<NTS>(mb, m, nv, tid);
      store_rows<NTS>(th, t, nv, tid);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) WireIO<W>::template st4<DL_DPS_WIRE_NTS(NTS)>(w, v, x[u]);
      }
#else
#if DL_DPS_ORDER == 0
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) WireIO<W>::template st4<DL_DPS_WIRE_NTS(NTS)>(w, v, x[u]);
      }
#endif
      store_rows<NTS>(th, t, nv, tid);
      if (MODE != 0) store_rows<NTS>(mb, m, nv, tid);
      store_rows<NTS>(in, t, nv, tid);
#endif
      const int i = (nv << 2) + tid;
      if (i < ck.len) {
        const float g0 = th[i] - in[i];
        WireIO<W>::st1(w, i, g0);
        const float g = on_wire(g0);
        float b = (MODE == 2) ? mb[i] : 0.f, t1 = th[i];
        sgd1<MODE>(g, b, t1, a);
        th[i] = t1;
        if (MODE != 0) mb[i] = b;
        in[i] = t1;
      }
    } else {
      for (int i = tid; i < ck.len; i += kThreads) {
        const float g0 = th[i] - in[i];
        WireIO<W>::st1(w, i, g0);
        const float g = on_wire(g0);
        float b = (MODE == 2) ? mb[i] : 0.f, t1 = th[i];
        sgd1<MODE>(g, b, t1, a);
        th[i] = t1;
        if (MODE != 0) mb[i] = b;
        in[i] = t1;
      }
    }
  }
};

// per-tensor fp32 -> packed W
template <typename W>
struct Gather {
  int src_slot;
  W* packed;
  template <bool NTL, int NTS>
  __device__ __forceinline__ void run(const Chunk& ck, int c, void* const* caddr, int nchunk, int tid) const {
    const float* src = slot_ptr<const float>(caddr, nchunk, src_slot, c);
    W* p = packed + ck.poff;
    if (aligned16(src)) {
      const int nv = ck.len >> 2;
      float4 x[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) x[u] = ldf4<NTL>(src, v);
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) WireIO<W>::template st4<NTS>(p, v, x[u]);
      }
      const int i = (nv << 2) + tid;
      if (i < ck.len) WireIO<W>::st1(p, i, src[i]);
    } else {
      for (int i = tid; i < ck.len; i += kThreads) WireIO<W>::st1(p, i, src[i]);
    }
  }
};

#ifdef DL_TUNING
template <typename W>
struct GatherPair {
  Gather<W> one;
  template <bool NTL, int NTS>
  __device__ __forceinline__ void run(const Chunk& ck, int c, void* const* caddr, int nchunk, int tid) const {
    one.template run<NTL, NTS>(ck, c, caddr, nchunk, tid);
  }
  template <bool NTL, int NTS>
  __device__ __forceinline__ void run2(const Chunk& k0, int c0, const Chunk& k1, int c1,
                                       void* const* caddr, int nchunk, int tid) const {
    const float* s0 = slot_ptr<const float>(caddr, nchunk, one.src_slot, c0);
    const float* s1 = slot_ptr<const float>(caddr, nchunk, one.src_slot, c1);
    if (!aligned16(s0) || !aligned16(s1)) {
      run<NTL, NTS>(k0, c0, caddr, nchunk, tid);
      run<NTL, NTS>(k1, c1, caddr, nchunk, tid);
      return;
    }
    const int nv0 = k0.len >> 2, nv1 = k1.len >> 2;
    float4 x0[kUnroll], x1[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int v = u * kThreads + tid;
      if (v < nv0) x0[u] = ldf4<NTL>(s0, v);
      if (v < nv1) x1[u] = ldf4<NTL>(s1, v);
    }
    W* p0 = one.packed + k0.poff;
    W* p1 = one.packed + k1.poff;
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int v = u * kThreads + tid;
      if (v < nv0) WireIO<W>::template st4<NTS>(p0, v, x0[u]);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int v = u * kThreads + tid;
      if (v < nv1) WireIO<W>::template st4<NTS>(p1, v, x1[u]);
    }
    const int i0 = (nv0 << 2) + tid, i1 = (nv1 << 2) + tid;
    if (i0 < k0.len) WireIO<W>::st1(p0, i0, s0[i0]);
    if (i1 < k1.len) WireIO<W>::st1(p1, i1, s1[i1]);
  }
};

#endif  // DL_TUNING

// packed fp32 -> per-tensor fp32
struct Scatter {
  const float* packed;
  int dst_slot;
  template <bool NTL, int NTS>
  __device__ __forceinline__ void run(const Chunk& ck, int c, void* const* caddr, int nchunk, int tid) const {
    float* dst = slot_ptr<float>(caddr, nchunk, dst_slot, c);
    const float* p = packed + ck.poff;
    if (aligned16(dst)) {
      const int nv = ck.len >> 2;
      float4 x[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) x[u] = ldf4<NTL>(p, v);
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) stf4<NTS>(dst, v, x[u]);
      }
      const int i = (nv << 2) + tid;
      if (i < ck.len) dst[i] = p[i];
    } else {
      for (int i = tid; i < ck.len; i += kThreads) dst[i] = p[i];
    }
  }
};

// ---- serializer and synthetic fill -----------------------------------------------------------
template <typename S>
__device__ __forceinline__ float to_f32(const S* p, int64_t i);
template <>
__device__ __forceinline__ float to_f32<float>(const float* p, int64_t i) {
  return p[i];
}
template <>
__device__ __forceinline__ float to_f32<uint16_t>(const uint16_t* p, int64_t i) {
  return bf2f(p[i]);
}
struct half_bits {
  uint16_t b;
};
template <>
__device__ __forceinline__ float to_f32<half_bits>(const half_bits* p, int64_t i) {
  return h2f(p[i].b);
}

template <typename S>
__global__ void __launch_bounds__(kThreads)
    k_serialize(const S* __restrict__ src, int64_t numel, float m0, float m1,
                float* __restrict__ out) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    out[0] = m0;
    out[1] = m1;
  }
  float* dst = out + numel;
  const int64_t stride = int64_t(gridDim.x) * kThreads;
  for (int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x; i < numel; i += stride)
    dst[i] = to_f32<S>(src, i);
}

__global__ void __launch_bounds__(kThreads)
    k_serialize_f32x4(const float4* __restrict__ src, int64_t nv, float m0, float m1,
                      float4* __restrict__ dst, float* __restrict__ out) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    out[0] = m0;
    out[1] = m1;
  }
  const int64_t stride = int64_t(gridDim.x) * kThreads;
  for (int64_t v = int64_t(blockIdx.x) * kThreads + threadIdx.x; v < nv; v += stride)
    dst[v] = src[v];
}

__global__ void __launch_bounds__(kThreads)
    k_serialize_f64(const double* __restrict__ src, int64_t numel, float m0, float m1,
                    double* __restrict__ out) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    out[0] = double(m0);
    out[1] = double(m1);
  }
  double* dst = out + numel;
  const int64_t stride = int64_t(gridDim.x) * kThreads;
  for (int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x; i < numel; i += stride)
    dst[i] = src[i];
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void __launch_bounds__(kThreads)
    k_fill_synth(float* __restrict__ dst, int64_t n, uint64_t key0, float base, float scale,
                 const float* __restrict__ add) {
  const int64_t stride = int64_t(gridDim.x) * kThreads;
  for (int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x; i < n; i += stride) {
    const uint64_t z = splitmix64(key0 + uint64_t(i));
    const float u = float(int32_t(z >> 40) - 8388608) * 1.1920928955078125e-07f;
    float x = base + u * scale;
    if (add) x = x + add[i];
    dst[i] = x;
  }
}

// dl_tree_bind's table expansion: the address of every chunk inside its bound tensor
__global__ void __launch_bounds__(kThreads)
    k_resolve_chunks(const Chunk* __restrict__ chunks, const int64_t* __restrict__ loff,
                     const uint64_t* __restrict__ segptr, int32_t nch, uint64_t* __restrict__ out) {
  for (int32_t c = int32_t(blockIdx.x) * kThreads + int32_t(threadIdx.x); c < nch;
       c += int32_t(gridDim.x) * kThreads)
    out[c] = segptr[chunks[c].seg] + uint64_t(loff[c]) * sizeof(float);
}

// Calibration copy (bench.py's same-run copy ceiling): U float4 loads per lane issued before
// the stores, one workgroup per U*1024 float4. U = 4 is the walker's access shape; U = 8 (twice
// the bytes in flight) is the fastest flat copy measured (tools/mem_ceiling.hip copy<8>).
template <bool NT, int U>
__global__ void __launch_bounds__(kThreads)
    k_copy(const float* __restrict__ src, float* __restrict__ dst, int64_t n16) {
  const int64_t base = int64_t(blockIdx.x) * (kThreads * U);
  float4 x[U];
  const float* s = src + base * 4;
  float* d = dst + base * 4;
  const int64_t rem = n16 - base;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int v = u * kThreads + int(threadIdx.x);
    if (v < rem) x[u] = ldf4<NT>(s, v);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int v = u * kThreads + int(threadIdx.x);
    if (v < rem) stf4<NT>(d, v, x[u]);
  }
}

// Read and write probes (bench.py's mix ceiling, tools/rw_mix.hip): the buffer is S equal
// streams and workgroup t touches tile t (4 float4 per lane) of every stream, as a walker
// kernel with S input (or output) buffers does. The read probe's store is guarded by `sink`,
// which the host passes as 0: the loads stay live and nothing is written. The write probe sets
// every 32-bit word to its index.
template <bool NT, int S>
__global__ void __launch_bounds__(kThreads)
    k_probe_read(const float* __restrict__ src, int64_t per16, int32_t sink, float* __restrict__ out) {
  const int64_t base = int64_t(blockIdx.x) * (kThreads * kUnroll);
  const int64_t rem = per16 - base;
  float4 x[S][kUnroll];
#pragma unroll
  for (int k = 0; k < S; ++k)
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int v = u * kThreads + int(threadIdx.x);
      if (v < rem) x[k][u] = ldf4<NT>(src + (k * per16 + base) * 4, v);
    }
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < S; ++k)
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int v = u * kThreads + int(threadIdx.x);
      if (v < rem) acc += x[k][u].x + x[k][u].y + x[k][u].z + x[k][u].w;
    }
  if (sink) out[threadIdx.x] = acc;
}

template <bool NT, int S>
__global__ void __launch_bounds__(kThreads)
    k_probe_write(float* __restrict__ dst, int64_t per16) {
  const int64_t base = int64_t(blockIdx.x) * (kThreads * kUnroll);
  const int64_t rem = per16 - base;
#pragma unroll
  for (int k = 0; k < S; ++k)
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int v = u * kThreads + int(threadIdx.x);
      const uint32_t w = uint32_t(k * per16 + base + v) * 4u;
      if (v < rem)
        stf4<NT>(dst + (k * per16 + base) * 4, v,
                 make_float4(__uint_as_float(w), __uint_as_float(w + 1), __uint_as_float(w + 2),
                             __uint_as_float(w + 3)));
    }
}

}  // namespace

// ---- launchers -------------------------------------------------------------------------------
hipError_t launch_resolve_chunks(const Chunk* chunks, const int64_t* loff, const uint64_t* segptr,
                                 int32_t nch, void** out, hipStream_t s) {
  if (nch <= 0) return hipSuccess;
  int32_t grid = (nch + kThreads - 1) / kThreads;
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(k_resolve_chunks, dim3(grid), dim3(kThreads), 0, s, chunks, loff, segptr,
                     nch, reinterpret_cast<uint64_t*>(out));
  return hipGetLastError();
}

template <bool NT, int U>
static hipError_t copy_u(const void* src, void* dst, int64_t n16, hipStream_t s) {
  const int64_t per = kThreads * U;
  const int64_t grid = (n16 + per - 1) / per;
  if (grid > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_copy<NT, U>), dim3(uint32_t(grid)), dim3(kThreads), 0, s,
                     static_cast<const float*>(src), static_cast<float*>(dst), n16);
  return hipGetLastError();
}

hipError_t launch_copy(const void* src, void* dst, int64_t n16, bool nt, bool wide,
                       hipStream_t s) {
  if (n16 <= 0) return hipSuccess;
  if (wide) return nt ? copy_u<true, 8>(src, dst, n16, s) : copy_u<false, 8>(src, dst, n16, s);
  return nt ? copy_u<true, 4>(src, dst, n16, s) : copy_u<false, 4>(src, dst, n16, s);
}

template <bool NT, int S>
static hipError_t probe_s(bool write, const void* src, void* dst, int64_t per16, hipStream_t s) {
  const int64_t per = kThreads * kUnroll;
  const int64_t grid = (per16 + per - 1) / per;
  if (grid > INT32_MAX) return hipErrorInvalidValue;
  if (write)
    hipLaunchKernelGGL((k_probe_write<NT, S>), dim3(uint32_t(grid)), dim3(kThreads), 0, s,
                       static_cast<float*>(dst), per16);
  else
    hipLaunchKernelGGL((k_probe_read<NT, S>), dim3(uint32_t(grid)), dim3(kThreads), 0, s,
                       static_cast<const float*>(src), per16, 0, static_cast<float*>(dst));
  return hipGetLastError();
}

template <bool NT>
static hipError_t probe_nt(bool write, int streams, const void* src, void* dst, int64_t per16,
                           hipStream_t s) {
  switch (streams) {
    case 1: return probe_s<NT, 1>(write, src, dst, per16, s);
    case 2: return probe_s<NT, 2>(write, src, dst, per16, s);
    case 3: return probe_s<NT, 3>(write, src, dst, per16, s);
    default: return probe_s<NT, 4>(write, src, dst, per16, s);
  }
}

hipError_t launch_probe(bool write, int streams, const void* src, void* dst, int64_t per16,
                        bool nt, hipStream_t s) {
  if (per16 <= 0) return hipSuccess;
  return nt ? probe_nt<true>(write, streams, src, dst, per16, s)
            : probe_nt<false>(write, streams, src, dst, per16, s);
}

hipError_t launch_delta_pack(const Launch& L, int inner_slot, const float* outer, void* wire,
                             int wire_dtype) {
#ifdef DL_TUNING
  if (wire_dtype == DL_BF16) {
    const DeltaPack<bf16_t> one{inner_slot, outer, static_cast<bf16_t*>(wire)};
    return L.pairs ? run_pairs(L, DeltaPackPair<bf16_t>{one}) : run(L, one);
  }
  const DeltaPack<float> one{inner_slot, outer, static_cast<float*>(wire)};
  return L.pairs ? run_pairs(L, DeltaPackPair<float>{one}) : run(L, one);
#else
  if (wire_dtype == DL_BF16)
    return run(L, DeltaPack<bf16_t>{inner_slot, outer, static_cast<bf16_t*>(wire)});
  return run(L, DeltaPack<float>{inner_slot, outer, static_cast<float*>(wire)});
#endif
}

template <typename W>
static hipError_t unpack_avg_t(const Launch& L, const W* w, int divisor, int dst_slot,
                               float* dst_packed) {
  const float d = float(divisor);
  if (divisor == 1) return run(L, UnpackAvg<W, false>{w, dst_slot, dst_packed, d});
  return run(L, UnpackAvg<W, true>{w, dst_slot, dst_packed, d});
}

hipError_t launch_unpack_avg(const Launch& L, const void* wire, int wire_dtype, int divisor,
                             int dst_slot, float* dst_packed) {
  if (wire_dtype == DL_BF16)
    return unpack_avg_t(L, static_cast<const bf16_t*>(wire), divisor, dst_slot, dst_packed);
  return unpack_avg_t(L, static_cast<const float*>(wire), divisor, dst_slot, dst_packed);
}

template <typename W, bool DIV>
static hipError_t unpack_sgd_mode(const Launch& L, const W* w, float d, float* outer, float* mom,
                                  SgdArgs a, int inner_slot) {
  if (a.momentum == 0.f) return run(L, UnpackSgd<W, DIV, 0>{w, outer, mom, d, a, inner_slot});
  if (a.first) return run(L, UnpackSgd<W, DIV, 1>{w, outer, mom, d, a, inner_slot});
  return run(L, UnpackSgd<W, DIV, 2>{w, outer, mom, d, a, inner_slot});
}

template <typename W>
static hipError_t unpack_sgd_t(const Launch& L, const W* w, int divisor, float* outer, float* mom,
                               SgdArgs a, int inner_slot) {
  const float d = float(divisor);
  if (divisor == 1) return unpack_sgd_mode<W, false>(L, w, d, outer, mom, a, inner_slot);
  return unpack_sgd_mode<W, true>(L, w, d, outer, mom, a, inner_slot);
}

hipError_t launch_unpack_sgd(const Launch& L, const void* wire, int wire_dtype, int divisor,
                             float* outer, float* mom, SgdArgs a, int inner_slot) {
  if (wire_dtype == DL_BF16)
    return unpack_sgd_t(L, static_cast<const bf16_t*>(wire), divisor, outer, mom, a, inner_slot);
  return unpack_sgd_t(L, static_cast<const float*>(wire), divisor, outer, mom, a, inner_slot);
}

// Sharded outer step: after the reduce-scatter each peer owns a contiguous 1/n of
// every bucket; the same UnpackSgd body runs over it as flat 4096-element chunks (no tree, no
// inner copy: θ is all-gathered and scattered to the inner params afterwards).
template <class Body>
__global__ void __launch_bounds__(kThreads) k_flat(int64_t n, Body body) {
  for (int64_t base = int64_t(blockIdx.x) * DL_CHUNK_ELEMS; base < n;
       base += int64_t(gridDim.x) * DL_CHUNK_ELEMS) {
    Chunk ck;
    ck.poff = base;
    ck.len = int32_t(n - base < DL_CHUNK_ELEMS ? n - base : DL_CHUNK_ELEMS);
    ck.seg = 0;
    body.template run<true, true>(ck, 0, nullptr, 0, int(threadIdx.x));  // NT loads + stores
  }
}

template <class Body>
static hipError_t run_flat(int64_t n, const Body& body, hipStream_t s) {
  const int32_t grid = int32_t((n + DL_CHUNK_ELEMS - 1) / DL_CHUNK_ELEMS);
  hipLaunchKernelGGL(k_flat<Body>, dim3(grid), dim3(kThreads), 0, s, n, body);
  return hipGetLastError();
}

template <typename W, bool DIV>
static hipError_t shard_sgd_mode(const W* w, float d, float* outer, float* mom, int64_t n,
                                 SgdArgs a, hipStream_t s) {
  if (a.momentum == 0.f) return run_flat(n, UnpackSgd<W, DIV, 0>{w, outer, mom, d, a, -1}, s);
  if (a.first) return run_flat(n, UnpackSgd<W, DIV, 1>{w, outer, mom, d, a, -1}, s);
  return run_flat(n, UnpackSgd<W, DIV, 2>{w, outer, mom, d, a, -1}, s);
}

template <typename W>
static hipError_t shard_sgd_t(const W* w, int divisor, float* outer, float* mom, int64_t n,
                              SgdArgs a, hipStream_t s) {
  const float d = float(divisor);
  if (divisor == 1) return shard_sgd_mode<W, false>(w, d, outer, mom, n, a, s);
  return shard_sgd_mode<W, true>(w, d, outer, mom, n, a, s);
}

hipError_t launch_shard_sgd(const void* wire, int wire_dtype, int divisor, float* outer, float* mom,
                            int64_t n, SgdArgs a, hipStream_t s) {
  if (wire_dtype == DL_BF16)
    return shard_sgd_t(static_cast<const bf16_t*>(wire), divisor, outer, mom, n, a, s);
  return shard_sgd_t(static_cast<const float*>(wire), divisor, outer, mom, n, a, s);
}

// a3 + a4 after an all_to_all (OuterSync(exchange="a2a"), the deterministic alternative to a
// SUM reduce-scatter): `slices` holds n equal slices of `len` elements of wire type W, slice q
// being rank q's copy of this peer's shard. g = ((s_0 + s_1) + ... + s_{n-1}) / n in fp32, in
// rank order -- the order of oracle/or_sum_avg and dl_xgmi_reduce_sgd, identical on every
// rank whatever the transport -- then dl_shard_sgd's SGD on this peer's θ and momentum shards.
// Reads n·sizeof(W) + 8 B, writes 8 B per shard element. N = 0: n read at run time (n > 8).
// MODE 3 (dl_shard_reduce_avg, the ordered DP gradient sync): no SGD -- `th` receives g.
// float4 rows per lane: 4 (the walker's 16 KiB per stream and workgroup) while the slices'
// registers allow it, 2 beyond two slices (N = 8: 16 slice float4 + θ, m per lane)
template <int N>
constexpr int slice_rows() { return N >= 1 && N <= 2 ? 4 : 2; }
template <int N, typename W, int MODE>
__global__ void __launch_bounds__(kThreads)
    k_slices_sgd(const W* __restrict__ slices, int32_t n, int64_t len, float* __restrict__ th,
                 float* __restrict__ mom, SgdArgs a) {
  constexpr int kSU = slice_rows<N>();
  constexpr int64_t kSliceStep = kThreads * kSU * 4;
  const int nn = N > 0 ? N : n;
  for (int64_t base = int64_t(blockIdx.x) * kSliceStep; base < len;
       base += int64_t(gridDim.x) * kSliceStep) {
    const int32_t nv = int32_t((len - base) / 4 < kThreads * kSU ? (len - base) / 4 : kThreads * kSU);
    float* t0 = th + base;
    float* m0 = mom + base;
    float4 g[kSU], t[kSU], m[kSU];
    if constexpr (N > 0) {
      float4 w[N][kSU];
#pragma unroll
      for (int u = 0; u < kSU; ++u) {
        const int v = u * kThreads + int(threadIdx.x);
        if (v < nv) {
#pragma unroll
          for (int q = 0; q < N; ++q) w[q][u] = WireIO<W>::template ld4<true>(slices + q * len + base, v);
          if (MODE != 3) t[u] = ldf4<true>(t0, v);
          if (MODE == 2) m[u] = ldf4<true>(m0, v);
        }
      }
#pragma unroll
      for (int u = 0; u < kSU; ++u) {
        g[u] = w[0][u];
#pragma unroll
        for (int q = 1; q < N; ++q)
          g[u] = make_float4(g[u].x + w[q][u].x, g[u].y + w[q][u].y, g[u].z + w[q][u].z,
                             g[u].w + w[q][u].w);
      }
    } else {
#pragma unroll
      for (int u = 0; u < kSU; ++u) {
        const int v = u * kThreads + int(threadIdx.x);
        if (v < nv) {
          if (MODE != 3) t[u] = ldf4<true>(t0, v);
          if (MODE == 2) m[u] = ldf4<true>(m0, v);
          g[u] = WireIO<W>::template ld4<true>(slices + base, v);
          for (int q = 1; q < nn; ++q) {
            const float4 d = WireIO<W>::template ld4<true>(slices + q * len + base, v);
            g[u] = make_float4(g[u].x + d.x, g[u].y + d.y, g[u].z + d.z, g[u].w + d.w);
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kSU; ++u) {
      const int v = u * kThreads + int(threadIdx.x);
      if (v < nv) {
        const float4 gg = nn > 1 ? div4(g[u], float(nn)) : g[u];
        if constexpr (MODE == 3) {
          stf4<kStNT>(t0, v, gg);
        } else {
          sgd1<MODE>(gg.x, m[u].x, t[u].x, a);
          sgd1<MODE>(gg.y, m[u].y, t[u].y, a);
          sgd1<MODE>(gg.z, m[u].z, t[u].z, a);
          sgd1<MODE>(gg.w, m[u].w, t[u].w, a);
          stf4<kStNT>(t0, v, t[u]);
          if (MODE != 0) stf4<kStNT>(m0, v, m[u]);
        }
      }
    }
  }
}

template <int N, typename W>
static hipError_t slices_sgd_n(const W* w, int32_t n, int64_t len, float* th, float* mom,
                               SgdArgs a, hipStream_t s, bool avg_only) {
  const int64_t step = kThreads * slice_rows<N>() * 4;
  const int64_t blocks = (len + step - 1) / step;
  const int32_t grid = int32_t(blocks < (1 << 20) ? blocks : (1 << 20));
  if (avg_only)
    hipLaunchKernelGGL((k_slices_sgd<N, W, 3>), dim3(grid), dim3(kThreads), 0, s, w, n, len, th, mom, a);
  else if (a.momentum == 0.f)
    hipLaunchKernelGGL((k_slices_sgd<N, W, 0>), dim3(grid), dim3(kThreads), 0, s, w, n, len, th, mom, a);
  else if (a.first)
    hipLaunchKernelGGL((k_slices_sgd<N, W, 1>), dim3(grid), dim3(kThreads), 0, s, w, n, len, th, mom, a);
  else
    hipLaunchKernelGGL((k_slices_sgd<N, W, 2>), dim3(grid), dim3(kThreads), 0, s, w, n, len, th, mom, a);
  return hipGetLastError();
}

template <typename W>
static hipError_t slices_sgd_t(const W* w, int32_t n, int64_t len, float* th, float* mom,
                               SgdArgs a, hipStream_t s, bool avg) {
  switch (n) {
    case 1: return slices_sgd_n<1>(w, n, len, th, mom, a, s, avg);
    case 2: return slices_sgd_n<2>(w, n, len, th, mom, a, s, avg);
    case 3: return slices_sgd_n<3>(w, n, len, th, mom, a, s, avg);
    case 4: return slices_sgd_n<4>(w, n, len, th, mom, a, s, avg);
    case 5: return slices_sgd_n<5>(w, n, len, th, mom, a, s, avg);
    case 6: return slices_sgd_n<6>(w, n, len, th, mom, a, s, avg);
    case 7: return slices_sgd_n<7>(w, n, len, th, mom, a, s, avg);
    case 8: return slices_sgd_n<8>(w, n, len, th, mom, a, s, avg);
    default: return slices_sgd_n<0>(w, n, len, th, mom, a, s, avg);
  }
}

// avg_only: out (`outer`) = Σ/n, no SGD, `mom` unused (dl_shard_reduce_avg)
hipError_t launch_slices_sgd(const void* slices, int wire_dtype, int32_t n, int64_t len,
                             float* outer, float* mom, SgdArgs a, hipStream_t s, bool avg_only) {
  if (len <= 0) return hipSuccess;
  if (wire_dtype == DL_BF16)
    return slices_sgd_t(static_cast<const bf16_t*>(slices), n, len, outer, mom, a, s, avg_only);
  return slices_sgd_t(static_cast<const float*>(slices), n, len, outer, mom, a, s, avg_only);
}

hipError_t launch_delta_sgd(const Launch& L, int inner_slot, float* outer, float* mom, SgdArgs a) {
  if (a.momentum == 0.f) return run(L, DeltaSgd<0>{outer, mom, a, inner_slot});
  if (a.first) return run(L, DeltaSgd<1>{outer, mom, a, inner_slot});
  return run(L, DeltaSgd<2>{outer, mom, a, inner_slot});
}

template <typename W>
static hipError_t delta_pack_sgd_t(const Launch& L, int inner_slot, float* outer, W* wire,
                                   float* mom, SgdArgs a) {
  if (a.momentum == 0.f) return run(L, DeltaPackSgd<W, 0>{outer, wire, mom, a, inner_slot});
  if (a.first) return run(L, DeltaPackSgd<W, 1>{outer, wire, mom, a, inner_slot});
  return run(L, DeltaPackSgd<W, 2>{outer, wire, mom, a, inner_slot});
}

hipError_t launch_delta_pack_sgd(const Launch& L, int inner_slot, float* outer, void* wire,
                                 int wire_dtype, float* mom, SgdArgs a) {
  if (wire_dtype == DL_BF16)
    return delta_pack_sgd_t(L, inner_slot, outer, static_cast<bf16_t*>(wire), mom, a);
  return delta_pack_sgd_t(L, inner_slot, outer, static_cast<float*>(wire), mom, a);
}

hipError_t launch_gather(const Launch& L, int src_slot, void* packed, int dtype) {
#ifdef DL_TUNING
  if (dtype == DL_BF16) {
    const Gather<bf16_t> one{src_slot, static_cast<bf16_t*>(packed)};
    return L.pairs ? run_pairs(L, GatherPair<bf16_t>{one}) : run(L, one);
  }
  const Gather<float> one{src_slot, static_cast<float*>(packed)};
  return L.pairs ? run_pairs(L, GatherPair<float>{one}) : run(L, one);
#else
  if (dtype == DL_BF16) return run(L, Gather<bf16_t>{src_slot, static_cast<bf16_t*>(packed)});
  return run(L, Gather<float>{src_slot, static_cast<float*>(packed)});
#endif
}

hipError_t launch_scatter(const Launch& L, const float* packed, int dst_slot) {
  return run(L, Scatter{packed, dst_slot});
}

static int grid_for(int64_t work) {
  int64_t g = (work + kThreads - 1) / kThreads;
  if (g > 4096) g = 4096;
  return g < 1 ? 1 : int(g);
}

hipError_t launch_serialize(const void* src, int src_dtype, int64_t numel, float m0, float m1,
                            float* out, hipStream_t s) {
  if (src_dtype == DL_F32 && (numel & 3) == 0 && aligned16_host(src) && aligned16_host(out)) {
    const int64_t nv = numel >> 2;
    hipLaunchKernelGGL(k_serialize_f32x4, dim3(grid_for(nv)), dim3(kThreads), 0, s,
                       static_cast<const float4*>(src), nv, m0, m1,
                       reinterpret_cast<float4*>(out + numel), out);
  } else if (src_dtype == DL_F32) {
    hipLaunchKernelGGL(k_serialize<float>, dim3(grid_for(numel)), dim3(kThreads), 0, s,
                       static_cast<const float*>(src), numel, m0, m1, out);
  } else if (src_dtype == DL_BF16) {
    hipLaunchKernelGGL(k_serialize<uint16_t>, dim3(grid_for(numel)), dim3(kThreads), 0, s,
                       static_cast<const uint16_t*>(src), numel, m0, m1, out);
  } else {
    hipLaunchKernelGGL(k_serialize<half_bits>, dim3(grid_for(numel)), dim3(kThreads), 0, s,
                       static_cast<const half_bits*>(src), numel, m0, m1, out);
  }
  return hipGetLastError();
}

hipError_t launch_serialize_f64(const double* src, int64_t numel, float m0, float m1, double* out,
                                hipStream_t s) {
  hipLaunchKernelGGL(k_serialize_f64, dim3(grid_for(numel)), dim3(kThreads), 0, s, src, numel, m0,
                     m1, out);
  return hipGetLastError();
}

// the device wall clock (100 MHz on MI355X; the launcher converts with the reported rate)
__global__ void __launch_bounds__(64) k_spin(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
}

hipError_t launch_spin(uint64_t ns, hipStream_t s) {
  // the wall-clock rate of the device the stream launches on (not the caller's current one)
  hipDevice_t dev = 0;
  int khz = 0;
  hipError_t e = hipStreamGetDevice(s, &dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  if (e != hipSuccess) return e;
  const uint64_t ticks = ns * uint64_t(khz > 0 ? khz : 100000) / 1000000ull;
  hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, ticks);
  return hipGetLastError();
}

hipError_t launch_fill_synth(float* dst, int64_t n, uint64_t seed, uint64_t stream_id, float base,
                             float scale, const float* add, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const uint64_t key0 = seed * 0xD1B54A32D192ED03ull + (stream_id << 40);
  // one workgroup per 256 elements (the grid-stride loop only past 2^38 elements): short-lived
  // workgroups like the outer-step kernels' (with eight processes time-sharing the
  // GPU, a long-lived grid-stride fill lost one XCD's share of its stores)
  int64_t g = (n + kThreads - 1) / kThreads;
  if (g > (1ll << 30)) g = 1ll << 30;
  hipLaunchKernelGGL(k_fill_synth, dim3(unsigned(g)), dim3(kThreads), 0, s, dst, n, key0, base,
                     scale, add);
  return hipGetLastError();
}

}  // namespace dl
