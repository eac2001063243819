// Device-side building blocks shared by the kernel translation units (dl_kernels.hip,
// dl_q8.hip): streaming memory ops, element conversions, the segment walker and its launcher.
#pragma once
#include <type_traits>

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
// Store policies (the walker's NTS template argument, dl_tree_tune's flags): plain, `nt`
// (non-temporal), or write-through (`sc1`: the line leaves the XCD's L2 at once instead of
// staying there dirty until evicted; tools/store_policy.hip). A write-through store goes
// through a buffer descriptor of the stream's base, which is wave-uniform in every caller (a
// chunk's stream base from the chunk table), so the descriptor lives in SGPRs; v < 2^27.
enum : int { kStPlain = 0, kStNT = 1, kStWT = 2 };
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
constexpr int kAuxSc1 = 16;  // buffer-op cache policy bits, gfx950: sc0 = 1, nt = 2, sc1 = 16
__device__ __forceinline__ __amdgpu_buffer_rsrc_t stream_rsrc(void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7fffffff, 0x00020000);
}
// Store-order A/B of dl_delta_pack_sgd (tools/store_order_ab.py builds the variants; the
// product build uses the defaults): DL_DPS_ORDER picks the order of its four output streams,
// DL_DPS_WIRE_PLAIN stores the wire with plain stores while θ, momentum and inner follow the
// launch's store policy.
#ifndef DL_DPS_ORDER
#define DL_DPS_ORDER 0
#endif
#ifdef DL_DPS_WIRE_PLAIN
#define DL_DPS_WIRE_NTS(n) kStPlain
#else
#define DL_DPS_WIRE_NTS(n) (n)
#endif
template <int SP>
__device__ __forceinline__ void stf4(float* p, int v, float4 x) {
  const f32x4 r = {x.x, x.y, x.z, x.w};
  if constexpr (SP == kStWT) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, r), stream_rsrc(p), v * 16, 0,
                                           kAuxSc1);
  } else {
    gf4 q = (gf4)(p) + v;
    if constexpr (SP == kStNT) __builtin_nontemporal_store(r, q);
    else *q = r;
  }
}
template <bool NT>
__device__ __forceinline__ uint64_t ld8(const void* p, int v) {
  gcu64 q = (gcu64)(p) + v;
  if constexpr (NT) return __builtin_nontemporal_load(q);
  else return *q;
}
template <int SP>
__device__ __forceinline__ void st8(void* p, int v, uint64_t x) {
  if constexpr (SP == kStWT) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, x), stream_rsrc(p), v * 8, 0,
                                          kAuxSc1);
  } else {
    gu64 q = (gu64)(p) + v;
    if constexpr (SP == kStNT) __builtin_nontemporal_store(x, q);
    else *q = x;
  }
}

template <typename W>
struct WireIO;

template <>
struct WireIO<float> {
  template <bool NT>
  static __device__ __forceinline__ float4 ld4(const float* p, int v) { return ldf4<NT>(p, v); }
  template <int SP>
  static __device__ __forceinline__ void st4(float* p, int v, float4 x) { stf4<SP>(p, v, x); }
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
  template <int SP>
  static __device__ __forceinline__ void st4(bf16_t* p, int v, float4 x) {
    const uint64_t r = uint64_t(f2bf(x.x)) | (uint64_t(f2bf(x.y)) << 16) |
                       (uint64_t(f2bf(x.z)) << 32) | (uint64_t(f2bf(x.w)) << 48);
    st8<SP>(p, v, r);
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

// The stores of a chunk, one stream at a time: the kUnroll rows of one buffer, then the next
// buffer's, so each wave writes 4 KiB of one stream back to back. The flat microbenchmark of
// the 7-stream shape gained 4 % from it (tools/mem_ceiling.hip dps_o); in the product kernels
// the cold A/B against the row-by-row order is neutral within noise (tools/gpu_ab_cold.sh,
// profiles/r02_ab_store_order.txt). Rows past the chunk (v >= nv) hold no data and are skipped.
template <int NTS>
__device__ __forceinline__ void store_rows(float* p, const float4 (&x)[kUnroll], int nv, int tid) {
#pragma unroll
  for (int u = 0; u < kUnroll; ++u) {
    const int v = u * kThreads + tid;
    if (v < nv) stf4<NTS>(p, v, x[u]);
  }
}

template <typename T>
__device__ __forceinline__ T* slot_ptr(void* const* caddr, int nchunk, int slot, int c) {
  return static_cast<T*>(caddr[slot * nchunk + c]);
}

// ---- the walker ----------------------------------------------------------------------------
// Body::run is instantiated per (NTL, NTS) policy. The product build instantiates what
// DL_TUNE_AUTO selects: non-temporal loads with plain or non-temporal stores. `make TUNING=1`
// (-DDL_TUNING) instantiates the whole matrix -- plain loads, write-through for every body --
// for the measurement tools (tools/cold_sweep.py); dl_tree_tune rejects the rest otherwise.
// Workgroup -> chunk. The dispatcher hands workgroup b to XCD (b + k) mod 8 (k fixed within a
// dispatch: tools/fill_census.hip), so by default the eight XCDs walk the range interleaved
// chunk by chunk. With one workgroup per chunk, xlog > 0 makes XCD x walk runs of B = 2^xlog
// consecutive chunks -- its k-th workgroup takes chunk ((k >> xlog) * 8 + x) * B + (k & (B-1))
// -- over the whole super-blocks of 8B chunks, the tail as by default; xlog = -1 gives XCD x
// the x-th eighth of the range in order (n = 8q + r: XCDs below r take q + 1 chunks). Both
// are bijections on [0, n). The product launches with xlog = 0; the others are A/B builds
// (tools/store_order_ab.py: no mapping gains on every box).
__device__ __forceinline__ int32_t walk_index(int32_t b, int32_t n, int32_t xlog) {
  if (xlog == 0 || int32_t(gridDim.x) != n) return b;
  const int32_t x = b & 7, k = b >> 3;
  if (xlog < 0) {
    const int32_t q = n >> 3, r = n & 7;
    return x * q + (x < r ? x : r) + k;
  }
  const int32_t full = (n >> (xlog + 3)) << (xlog + 3);
  if (b >= full) return b;
  return (((k >> xlog) << 3) + x) * (1 << xlog) + (k & ((1 << xlog) - 1));
}

template <class Body, bool NTL, int NTS>
__global__ void __launch_bounds__(kThreads)
    k_walk(const Chunk* __restrict__ chunks, int32_t c0, int32_t c1, void* const* __restrict__ caddr,
           int32_t nchunk, int32_t xlog, Body body) {
  for (int32_t i0 = int32_t(blockIdx.x); i0 < c1 - c0; i0 += int32_t(gridDim.x)) {
    const int32_t c = c0 + walk_index(i0, c1 - c0, xlog);
    const Chunk ck = chunks[c];
    body.template run<NTL, NTS>(ck, c, caddr, nchunk, int(threadIdx.x));
  }
}

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

template <class Body, bool NTL, int NTS>
hipError_t launch_walk(const Launch& L, const Body& body, int32_t grid) {
  hipLaunchKernelGGL((k_walk<Body, NTL, NTS>), dim3(grid), dim3(kThreads), 0, L.stream, L.chunks,
                     L.c0, L.c1, L.caddr, L.nchunk, L.xlog, body);
  return hipGetLastError();
}

#ifdef DL_TUNING
// The pair walker (tuning build): workgroup i takes chunks 2i and 2i+1 of the range (run2 issues both
// chunks' loads before any store); a last odd chunk goes through run. Grid = ceil(n / 2), or
// the tree's cap with a grid-stride over pairs.
template <class Body, bool NTL, int NTS>
__global__ void __launch_bounds__(kThreads)
    k_walk_pairs(const Chunk* __restrict__ chunks, int32_t c0, int32_t c1,
                 void* const* __restrict__ caddr, int32_t nchunk, Body body) {
  const int32_t n = c1 - c0;
  for (int32_t i = 2 * int32_t(blockIdx.x); i < n; i += 2 * int32_t(gridDim.x)) {
    const int32_t c = c0 + i;
    const Chunk k0 = chunks[c];
    if (i + 1 < n) {
      const Chunk k1 = chunks[c + 1];
      body.template run2<NTL, NTS>(k0, c, k1, c + 1, caddr, nchunk, int(threadIdx.x));
    } else {
      body.template run<NTL, NTS>(k0, c, caddr, nchunk, int(threadIdx.x));
    }
  }
}

template <class Body, bool NTL, int NTS>
hipError_t launch_pairs(const Launch& L, const Body& body, int32_t grid) {
  hipLaunchKernelGGL((k_walk_pairs<Body, NTL, NTS>), dim3(grid), dim3(kThreads), 0, L.stream,
                     L.chunks, L.c0, L.c1, L.caddr, L.nchunk, body);
  return hipGetLastError();
}

#endif  // DL_TUNING

template <class Body>
hipError_t run(const Launch& L, const Body& body) {
  const int32_t n = L.c1 - L.c0;
  if (n <= 0) return hipSuccess;
  const int32_t grid = (L.grid > 0 && L.grid < n) ? L.grid : n;  // default: one workgroup per chunk
  const bool ntl = (L.flags & DL_TUNE_NT_LOADS) != 0;
  const int sp = (L.flags & DL_TUNE_WT_STORES) ? kStWT : (L.flags & DL_TUNE_NT_STORES) ? kStNT : kStPlain;
#ifdef DL_TUNING
  if (!ntl) {
    if (sp == kStWT) return launch_walk<Body, false, kStWT>(L, body, grid);
    if (sp == kStNT) return launch_walk<Body, false, kStNT>(L, body, grid);
    return launch_walk<Body, false, kStPlain>(L, body, grid);
  }
  if (sp == kStWT) return launch_walk<Body, true, kStWT>(L, body, grid);
#else
  // not instantiated (dl_tree_tune rejects these flags first)
  if (!ntl || sp == kStWT) return hipErrorInvalidValue;
#endif
  if (sp == kStNT) return launch_walk<Body, true, kStNT>(L, body, grid);
  return launch_walk<Body, true, kStPlain>(L, body, grid);
}

#ifdef DL_TUNING
// run() for a pair-capable body (DeltaPackPair, GatherPair): NT loads, plain / NT stores
template <class Body>
hipError_t run_pairs(const Launch& L, const Body& body) {
  const int32_t n = L.c1 - L.c0;
  if (n <= 0) return hipSuccess;
  const int32_t np = (n + 1) / 2;
  const int32_t grid = (L.grid > 0 && L.grid < np) ? L.grid : np;
  if (!(L.flags & DL_TUNE_NT_LOADS) || (L.flags & DL_TUNE_WT_STORES)) return run(L, body);
  if (L.flags & DL_TUNE_NT_STORES) return launch_pairs<Body, true, kStNT>(L, body, grid);
  return launch_pairs<Body, true, kStPlain>(L, body, grid);
}
#endif  // DL_TUNING

}  // namespace
}  // namespace dl
