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
// Body::run is instantiated per (NTL, NTS) policy: non-temporal loads; plain / NT / WT stores.
// rev: walk the range last chunk first (workgroups are dispatched in blockIdx order), so a
// kernel that follows one which streamed the same buffers front to back starts on the bytes
// most likely still in the Infinity Cache.
template <class Body, bool NTL, int NTS>
__global__ void __launch_bounds__(kThreads)
    k_walk(const Chunk* __restrict__ chunks, int32_t c0, int32_t c1, void* const* __restrict__ caddr,
           int32_t nchunk, int32_t rev, Body body) {
  for (int32_t i = int32_t(blockIdx.x); i < c1 - c0; i += int32_t(gridDim.x)) {
    const int32_t c = rev ? c1 - 1 - i : c0 + i;
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

// ---- clock-slotted walker (dl_tree_slot) ----------------------------------------------------
// HBM serves a streaming kernel's reads at ~7 TB/s and its writes at 5.5-6.9, but the steady
// mix of both that a one-workgroup-per-chunk walker produces runs ~10 % below the time the
// reads and the writes take separately (tools/rw_mix.hip). The slotted walker
// separates them in time without any communication between workgroups: a resident grid, each
// workgroup pacing its rounds by the chip's 100 MHz real-time counter (s_memrealtime) from its
// own start -- all loads of a round issued at the round's start, all stores `read` ticks
// later, the next round `period` ticks after the last -- so the whole chip reads, then writes. A workgroup behind schedule goes at once
// instead of skipping a slot; every wait ends when the counter passes a target at most one
// period ahead. Results do not depend on the timing (same arithmetic, same stores).
__device__ __forceinline__ uint64_t rtc() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void wait_until(uint64_t t) {
  while (rtc() < t) __builtin_amdgcn_s_sleep(2);
  __asm__ volatile("" ::: "memory");
}

// called by a body between its loads (and arithmetic) and its stores
struct NoGate {
  __device__ __forceinline__ void operator()() const {}
};
struct SlotGate {
  uint64_t t;
  __device__ __forceinline__ void operator()() const {
    __asm__ volatile("" ::: "memory");
    wait_until(t);
  }
};

template <class Body, bool NTL, int NTS>
__global__ void __launch_bounds__(kThreads)
    k_walk_slotted(const Chunk* __restrict__ chunks, int32_t c0, int32_t c1,
                   void* const* __restrict__ caddr, int32_t nchunk, uint32_t period,
                   uint32_t read, Body body) {
  // the first round starts at once: the resident grid is dispatched within a few us, so the
  // workgroups' own start times already agree to a small fraction of a period
  uint64_t slot = rtc();
  for (int32_t i = int32_t(blockIdx.x); i < c1 - c0; i += int32_t(gridDim.x), slot += period) {
    const int32_t c = c0 + i;
    const Chunk ck = chunks[c];
    wait_until(slot);
    body.template run<NTL, NTS>(ck, c, caddr, nchunk, int(threadIdx.x), SlotGate{slot + read});
  }
}

// workgroups of k that fit on the device at once (the slotted walker's grid)
template <class K>
int32_t resident_grid(K kernel) {
  int per_cu = 0, cus = 0, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kThreads, 0) != hipSuccess)
    return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return per_cu * cus;
}

// bodies that take a gate between their loads and their stores declare kSlotted = true
template <class B, class = void>
struct slotted : std::false_type {};
template <class B>
struct slotted<B, std::void_t<decltype(B::kSlotted)>> : std::bool_constant<B::kSlotted> {};

template <class Body, bool NTL, int NTS>
hipError_t run_policy(const Launch& L, const Body& body, int32_t grid) {
  if constexpr (slotted<Body>::value) {
    if (L.slot_period > 0) {
      static const int32_t resident = resident_grid(k_walk_slotted<Body, NTL, NTS>);
      const int32_t n = L.c1 - L.c0;
      const int32_t g = resident > 0 && resident < n ? resident : n;
      hipLaunchKernelGGL((k_walk_slotted<Body, NTL, NTS>), dim3(g), dim3(kThreads), 0, L.stream,
                         L.chunks, L.c0, L.c1, L.caddr, L.nchunk, uint32_t(L.slot_period),
                         uint32_t(L.slot_read), body);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((k_walk<Body, NTL, NTS>), dim3(grid), dim3(kThreads), 0, L.stream, L.chunks,
                     L.c0, L.c1, L.caddr, L.nchunk, (L.flags & DL_TUNE_REVERSE) ? 1 : 0, body);
  return hipGetLastError();
}

template <class Body>
hipError_t run(const Launch& L, const Body& body) {
  const int32_t n = L.c1 - L.c0;
  if (n <= 0) return hipSuccess;
  const int32_t grid = (L.grid > 0 && L.grid < n) ? L.grid : n;  // default: one workgroup per chunk
  const bool ntl = (L.flags & DL_TUNE_NT_LOADS) != 0;
  const int sp = (L.flags & DL_TUNE_WT_STORES) ? kStWT : (L.flags & DL_TUNE_NT_STORES) ? kStNT : kStPlain;
  if (ntl) {
    if (sp == kStWT) return run_policy<Body, true, kStWT>(L, body, grid);
    if (sp == kStNT) return run_policy<Body, true, kStNT>(L, body, grid);
    return run_policy<Body, true, kStPlain>(L, body, grid);
  }
  if (sp == kStWT) return run_policy<Body, false, kStWT>(L, body, grid);
  if (sp == kStNT) return run_policy<Body, false, kStNT>(L, body, grid);
  return run_policy<Body, false, kStPlain>(L, body, grid);
}

}  // namespace
}  // namespace dl
