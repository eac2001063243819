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
#include "dl_internal.h"

namespace dl {
namespace {

__device__ __forceinline__ bool aligned16(const void* p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

// ---- element types on the wire / in packed buffers -----------------------------------------
__device__ __forceinline__ uint16_t f2bf(float x) {
  __bf16 b = static_cast<__bf16>(x);  // v_cvt_pk_bf16_f32: RNE, NaN stays NaN
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }
__device__ __forceinline__ float h2f(uint16_t h) {
  return static_cast<float>(__builtin_bit_cast(_Float16, h));
}

struct bf16_t {
  uint16_t bits;
};

// Streaming memory ops. NT = non-temporal (`global_load/store_dwordx4 ... nt`): the operands
// are touched once per outer step and are larger than the 256 MiB Infinity Cache, so keeping
// them out of the caches measured +10-15 % on streaming loads (tools/hbm_bench.hip,
// DESIGN.md "Kernels"). Whether stores are NT is a per-tree tuning flag (dl_tree_tune).
typedef float f32x4 __attribute__((ext_vector_type(4)));
// Pointers from the device pointer table are generic (flat) to the compiler; casting to the
// global address space turns flat_load/store (counted on vmcnt AND lgkmcnt, completed out of
// order) into global_load/store.
#define DL_GLOBAL __attribute__((address_space(1)))
typedef DL_GLOBAL const f32x4* gcf4;
typedef DL_GLOBAL f32x4* gf4;
typedef DL_GLOBAL const uint64_t* gcu64;
typedef DL_GLOBAL uint64_t* gu64;

template <bool NT>
__device__ __forceinline__ float4 ldf4(const float* p, int v) {
  gcf4 q = (gcf4)(p) + v;
  f32x4 r;
  if constexpr (NT) r = __builtin_nontemporal_load(q);
  else r = *q;
  return make_float4(r.x, r.y, r.z, r.w);
}
template <bool NT>
__device__ __forceinline__ void stf4(float* p, int v, float4 x) {
  gf4 q = (gf4)(p) + v;
  const f32x4 r = {x.x, x.y, x.z, x.w};
  if constexpr (NT) __builtin_nontemporal_store(r, q);
  else *q = r;
}
template <bool NT>
__device__ __forceinline__ uint64_t ld8(const void* p, int v) {
  gcu64 q = (gcu64)(p) + v;
  if constexpr (NT) return __builtin_nontemporal_load(q);
  else return *q;
}
template <bool NT>
__device__ __forceinline__ void st8(void* p, int v, uint64_t x) {
  gu64 q = (gu64)(p) + v;
  if constexpr (NT) __builtin_nontemporal_store(x, q);
  else *q = x;
}

template <typename W>
struct WireIO;

template <>
struct WireIO<float> {
  template <bool NT>
  static __device__ __forceinline__ float4 ld4(const float* p, int v) { return ldf4<NT>(p, v); }
  template <bool NT>
  static __device__ __forceinline__ void st4(float* p, int v, float4 x) { stf4<NT>(p, v, x); }
  static __device__ __forceinline__ float ld1(const float* p, int i) { return p[i]; }
  static __device__ __forceinline__ void st1(float* p, int i, float x) { p[i] = x; }
};

template <>
struct WireIO<bf16_t> {
  template <bool NT>
  static __device__ __forceinline__ float4 ld4(const bf16_t* p, int v) {
    const uint64_t r = ld8<NT>(p, v);
    return make_float4(bf2f(uint16_t(r)), bf2f(uint16_t(r >> 16)), bf2f(uint16_t(r >> 32)),
                       bf2f(uint16_t(r >> 48)));
  }
  template <bool NT>
  static __device__ __forceinline__ void st4(bf16_t* p, int v, float4 x) {
    const uint64_t r = uint64_t(f2bf(x.x)) | (uint64_t(f2bf(x.y)) << 16) |
                       (uint64_t(f2bf(x.z)) << 32) | (uint64_t(f2bf(x.w)) << 48);
    st8<NT>(p, v, r);
  }
  static __device__ __forceinline__ float ld1(const bf16_t* p, int i) { return bf2f(p[i].bits); }
  static __device__ __forceinline__ void st1(bf16_t* p, int i, float x) { p[i].bits = f2bf(x); }
};


__device__ __forceinline__ float4 sub4(float4 a, float4 b) {
  return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
}
__device__ __forceinline__ float4 div4(float4 a, float d) {
  return make_float4(a.x / d, a.y / d, a.z / d, a.w / d);
}

template <typename T>
__device__ __forceinline__ T* slot_ptr(void* const* caddr, int nchunk, int slot, int c) {
  return static_cast<T*>(caddr[slot * nchunk + c]);
}

// ---- the walker ----------------------------------------------------------------------------
// Body::operator() is instantiated per (NTL, NTS) policy: non-temporal loads / stores.
template <class Body, bool NTL, bool NTS>
__global__ void __launch_bounds__(kThreads)
    k_walk(const Chunk* __restrict__ chunks, int32_t c0, int32_t c1, void* const* __restrict__ caddr,
           int32_t nchunk, Body body) {
  for (int32_t c = c0 + int32_t(blockIdx.x); c < c1; c += int32_t(gridDim.x)) {
    const Chunk ck = chunks[c];
    body.template run<NTL, NTS>(ck, c, caddr, nchunk, int(threadIdx.x));
  }
}

// a2: wire = outer - inner
template <typename W>
struct DeltaPack {
  int inner_slot;
  const float* outer;
  W* wire;
  template <bool NTL, bool NTS>
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

// a3 unpack: dst = wire / d
template <typename W, bool DIV>
struct UnpackAvg {
  const W* wire;
  int dst_slot;
  float* dst_packed;
  float d;
  template <bool NTL, bool NTS>
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

// a3+a4+a5 fused. MODE 0: momentum 0; 1: first step (buf = g); 2: buf = buf*m + g.
template <int MODE>
__device__ __forceinline__ void sgd1(float g, float& buf, float& th, const SgdArgs& a) {
  if (MODE == 0) {
    th = __builtin_fmaf(g, a.neg_lr, th);
  } else {
    buf = (MODE == 1) ? g : (buf * a.momentum) + g;  // contract off: two roundings
    const float u = a.nesterov ? __builtin_fmaf(buf, a.momentum, g) : buf;
    th = __builtin_fmaf(u, a.neg_lr, th);
  }
}

template <typename W, bool DIV, int MODE>
struct UnpackSgd {
  const W* wire;
  float* outer;
  float* mom;
  float d;
  SgdArgs a;
  int inner_slot;
  template <bool NTL, bool NTS>
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
        const int v = u * kThreads + tid;
        if (v < nv) {
          const float4 gg = DIV ? div4(g[u], d) : g[u];
          sgd1<MODE>(gg.x, m[u].x, t[u].x, a);
          sgd1<MODE>(gg.y, m[u].y, t[u].y, a);
          sgd1<MODE>(gg.z, m[u].z, t[u].z, a);
          sgd1<MODE>(gg.w, m[u].w, t[u].w, a);
          stf4<NTS>(th, v, t[u]);
          if (MODE != 0) stf4<NTS>(mb, v, m[u]);
          if (in) stf4<NTS>(in, v, t[u]);
        }
      }
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
  template <bool NTL, bool NTS>
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
        const int v = u * kThreads + tid;
        if (v < nv) {
          const float4 g = sub4(t[u], x[u]);
          sgd1<MODE>(g.x, m[u].x, t[u].x, a);
          sgd1<MODE>(g.y, m[u].y, t[u].y, a);
          sgd1<MODE>(g.z, m[u].z, t[u].z, a);
          sgd1<MODE>(g.w, m[u].w, t[u].w, a);
          stf4<NTS>(th, v, t[u]);
          if (MODE != 0) stf4<NTS>(mb, v, m[u]);
          stf4<NTS>(in, v, t[u]);
        }
      }
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

// per-tensor fp32 -> packed W
template <typename W>
struct Gather {
  int src_slot;
  W* packed;
  template <bool NTL, bool NTS>
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

// packed fp32 -> per-tensor fp32
struct Scatter {
  const float* packed;
  int dst_slot;
  template <bool NTL, bool NTS>
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

template <class Body, bool NTL, bool NTS>
hipError_t run_policy(const Launch& L, const Body& body, int32_t grid) {
  hipLaunchKernelGGL((k_walk<Body, NTL, NTS>), dim3(grid), dim3(kThreads), 0, L.stream, L.chunks,
                     L.c0, L.c1, L.caddr, L.nchunk, body);
  return hipGetLastError();
}

template <class Body>
hipError_t run(const Launch& L, const Body& body) {
  const int32_t n = L.c1 - L.c0;
  if (n <= 0) return hipSuccess;
  const int32_t grid = (L.grid > 0 && L.grid < n) ? L.grid : n;  // default: one workgroup per chunk
  const bool ntl = (L.flags & DL_TUNE_NT_LOADS) != 0, nts = (L.flags & DL_TUNE_NT_STORES) != 0;
  if (ntl && nts) return run_policy<Body, true, true>(L, body, grid);
  if (ntl) return run_policy<Body, true, false>(L, body, grid);
  if (nts) return run_policy<Body, false, true>(L, body, grid);
  return run_policy<Body, false, false>(L, body, grid);
}

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

}  // namespace

// ---- launchers -------------------------------------------------------------------------------
hipError_t launch_delta_pack(const Launch& L, int inner_slot, const float* outer, void* wire,
                             int wire_dtype) {
  if (wire_dtype == DL_BF16)
    return run(L, DeltaPack<bf16_t>{inner_slot, outer, static_cast<bf16_t*>(wire)});
  return run(L, DeltaPack<float>{inner_slot, outer, static_cast<float*>(wire)});
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

hipError_t launch_delta_sgd(const Launch& L, int inner_slot, float* outer, float* mom, SgdArgs a) {
  if (a.momentum == 0.f) return run(L, DeltaSgd<0>{outer, mom, a, inner_slot});
  if (a.first) return run(L, DeltaSgd<1>{outer, mom, a, inner_slot});
  return run(L, DeltaSgd<2>{outer, mom, a, inner_slot});
}

hipError_t launch_gather(const Launch& L, int src_slot, void* packed, int dtype) {
  if (dtype == DL_BF16) return run(L, Gather<bf16_t>{src_slot, static_cast<bf16_t*>(packed)});
  return run(L, Gather<float>{src_slot, static_cast<float*>(packed)});
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

hipError_t launch_fill_synth(float* dst, int64_t n, uint64_t seed, uint64_t stream_id, float base,
                             float scale, const float* add, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const uint64_t key0 = seed * 0xD1B54A32D192ED03ull + (stream_id << 40);
  hipLaunchKernelGGL(k_fill_synth, dim3(grid_for(n)), dim3(kThreads), 0, s, dst, n, key0, base,
                     scale, add);
  return hipGetLastError();
}

}  // namespace dl
