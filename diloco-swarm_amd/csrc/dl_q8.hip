// int8 wire codec for the pseudo-gradient exchange ("wire codecs beyond
// bf16, int8 with a per-bucket scale, for the cross-DC stand-in").
//
// Wire = one fixed-size SLOT per tree chunk: a 64-B header whose first 4 bytes are the fp32
// scale, then DL_CHUNK_ELEMS int8 values (bytes past the chunk's length stay zero). A bucket's
// slots are contiguous, in chunk order, padded with zero slots to a multiple of the peer count,
// so the exchange is two equal-split RCCL collectives ("int8 wire"):
//   dl_delta_q8       d = θ - inner; amax over the chunk (wave shuffles + LDS); q = rint(d/s)
//   all_to_all        every peer receives its 1/n of the slots from every peer
//   dl_q8_reduce      avg = (Σ_r q_r·s_r) / n in rank order; re-quantised with its own amax
//   all_gather        every peer receives every averaged slot (identical on all peers)
//   dl_unpack_sgd_q8  g = q·s; SGD exactly as dl_unpack_sgd; inner = θ
// Quantiser: s = amax / 127 (IEEE division); q = s == 0 ? 0 : clamp(rint(x / s), -127, 127);
// dequantised value q·s. Bus bytes per peer 2(n-1)/n · 1.016 B/param vs 8(n-1)/n for fp32.
#include "dl_device.h"

namespace dl {
namespace {

constexpr int kQ8Header = DL_Q8_SLOT_BYTES - DL_CHUNK_ELEMS;  // 64 B: fp32 scale + padding

__device__ __forceinline__ float block_amax(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));  // 64-lane wave
  __shared__ float part[kThreads / 64];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  v = fmaxf(fmaxf(part[0], part[1]), fmaxf(part[2], part[3]));
  __syncthreads();  // `part` is reused by the workgroup's next chunk
  return v;
}

__device__ __forceinline__ int q8(float x, float s) {
  if (s == 0.f) return 0;
  const float r = fminf(fmaxf(__builtin_rintf(x / s), -127.f), 127.f);
  return int(r);
}

__device__ __forceinline__ uint32_t pack4(float4 x, float s) {
  return (uint32_t(q8(x.x, s)) & 0xffu) | ((uint32_t(q8(x.y, s)) & 0xffu) << 8) |
         ((uint32_t(q8(x.z, s)) & 0xffu) << 16) | ((uint32_t(q8(x.w, s)) & 0xffu) << 24);
}

__device__ __forceinline__ float4 unpack4(uint32_t w, float s) {
  return make_float4(float(int8_t(w & 0xffu)) * s, float(int8_t((w >> 8) & 0xffu)) * s,
                     float(int8_t((w >> 16) & 0xffu)) * s, float(int8_t(w >> 24)) * s);
}

__device__ __forceinline__ float amax4(float4 x) {
  return fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w)));
}

// The slot header: the scale, then zeros, written whole as four 16-B stores (lanes 0-3) so
// consecutive slots leave as one gap-free stream. A lone 4-B store of the scale left 60 B of
// every 4160 unwritten: the encoder ran 1.1-1.8 % slower cold in three interleaved A/B pairs
// on T1.3B and T125 (profiles/r03_ab_q8_header_*.txt); the zeros match the zero-filled wire.
template <int NTS>
__device__ __forceinline__ void store_header(uint8_t* slot, float s, int tid) {
  if (tid < kQ8Header / 16) {
    const u32x4 w = {tid == 0 ? __float_as_uint(s) : 0u, 0u, 0u, 0u};
    DL_GLOBAL u32x4* h = (DL_GLOBAL u32x4*)slot + tid;
    if constexpr (NTS == kStNT)
      __builtin_nontemporal_store(w, h);
    else
      *h = w;
  }
}

typedef DL_GLOBAL uint32_t* gu32;
typedef DL_GLOBAL const uint32_t* gcu32;

// a2 with the int8 codec: slot(c) <- quantise(θ - inner) over chunk c.
// The 4096-B payload is assembled in LDS (zero beyond the chunk's length) and leaves in ONE
// 16-B store per lane: four 4-B-per-lane stores per lane (256 B per wave instruction) cost
// ~10 % of the kernel cold at T1.3B size against one 1-KB-per-wave store (tools/q8_layout.hip,
// profiles/r02_q8_layout.txt).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct DeltaQ8 {
  int inner_slot;
  const float* outer;
  uint8_t* slots;  // slot of chunk c at (c - c0) * DL_Q8_SLOT_BYTES
  int c0;
  template <bool NTL, int NTS>
  __device__ __forceinline__ void run(const Chunk& ck, int c, void* const* caddr, int nchunk, int tid) const {
    __shared__ u32x4 stage[DL_CHUNK_ELEMS / 16];  // the payload, 16 B per lane
    uint32_t* st32 = reinterpret_cast<uint32_t*>(stage);
    uint8_t* st8 = reinterpret_cast<uint8_t*>(stage);
    const float* in = slot_ptr<const float>(caddr, nchunk, inner_slot, c);
    const float* th = outer + ck.poff;
    uint8_t* slot = slots + size_t(c - c0) * DL_Q8_SLOT_BYTES;
    const int nv = ck.len >> 2;
    const bool vec = aligned16(in);
    stage[tid] = u32x4{0u, 0u, 0u, 0u};  // bytes past the chunk's length stay zero
    float4 d[kUnroll];
    float dt = 0.f;  // vector path: the < 4 tail elements
    float am = 0.f;
    if (vec) {
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        d[u] = v < nv ? sub4(ldf4<NTL>(th, v), ldf4<NTL>(in, v)) : make_float4(0.f, 0.f, 0.f, 0.f);
        am = fmaxf(am, amax4(d[u]));
      }
      const int i = (nv << 2) + tid;
      if (i < ck.len) dt = th[i] - in[i];
    } else {  // 4-B-aligned tensor storage: element k*256 + tid of the chunk in d[k/4].k%4
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        float e[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = (4 * u + j) * kThreads + tid;
          e[j] = i < ck.len ? th[i] - in[i] : 0.f;
        }
        d[u] = make_float4(e[0], e[1], e[2], e[3]);
        am = fmaxf(am, amax4(d[u]));
      }
    }
    am = fmaxf(am, fabsf(dt));
    const float s = block_amax(am) / 127.f;  // its barriers also order the zeroing above
    if (vec) {
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) st32[v] = pack4(d[u], s);
      }
      const int i = (nv << 2) + tid;
      if (i < ck.len) st8[i] = uint8_t(q8(dt, s));
    } else {
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const float e[4] = {d[u].x, d[u].y, d[u].z, d[u].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = (4 * u + j) * kThreads + tid;
          if (i < ck.len) st8[i] = uint8_t(q8(e[j], s));
        }
      }
    }
    __syncthreads();
    const u32x4 w = stage[tid];
    DL_GLOBAL u32x4* q = (DL_GLOBAL u32x4*)(slot + kQ8Header);
    if constexpr (NTS)
      __builtin_nontemporal_store(w, q + tid);
    else
      q[tid] = w;
    store_header<NTS>(slot, s, tid);
    __syncthreads();  // `stage` is reused by the workgroup's next chunk
  }
};

// a3 /n happened in dl_q8_reduce; a4 + a5 from the averaged int8 slots
template <int MODE>
struct UnpackSgdQ8 {
  const uint8_t* slots;
  int c0;
  float* outer;
  float* mom;
  SgdArgs a;
  int inner_slot;
  template <bool NTL, int NTS>
  __device__ __forceinline__ void run(const Chunk& ck, int c, void* const* caddr, int nchunk, int tid) const {
    float* in = inner_slot >= 0 ? slot_ptr<float>(caddr, nchunk, inner_slot, c) : nullptr;
    const uint8_t* slot = slots + size_t(c - c0) * DL_Q8_SLOT_BYTES;
    const uint8_t* q = slot + kQ8Header;
    const float s = *reinterpret_cast<const float*>(slot);
    float* th = outer + ck.poff;
    float* mb = mom + ck.poff;
    if (in == nullptr || aligned16(in)) {
      const int nv = ck.len >> 2;
      uint32_t w[kUnroll];
      float4 t[kUnroll], m[kUnroll];
      // the slot's 4 KB payload arrives as one non-temporal 16-B load per lane, staged in LDS
      // (tools/gpu_ab_q8.sh: -1 % at T1.3B against four 4-B loads per lane)
      __shared__ u32x4 stage[DL_CHUNK_ELEMS / 16];
      const u32x4 qv = __builtin_nontemporal_load((const DL_GLOBAL u32x4*)q + tid);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) {
          t[u] = ldf4<NTL>(th, v);
          if (MODE == 2) m[u] = ldf4<NTL>(mb, v);
        }
      }
      stage[tid] = qv;
      __syncthreads();
      const uint32_t* st32 = reinterpret_cast<const uint32_t*>(stage);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) w[u] = st32[u * kThreads + tid];
      __syncthreads();  // `stage` is reused by the workgroup's next chunk
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int v = u * kThreads + tid;
        if (v < nv) {
          const float4 g = unpack4(w[u], s);
          sgd1<MODE>(g.x, m[u].x, t[u].x, a);
          sgd1<MODE>(g.y, m[u].y, t[u].y, a);
          sgd1<MODE>(g.z, m[u].z, t[u].z, a);
          sgd1<MODE>(g.w, m[u].w, t[u].w, a);
          stf4<NTS>(th, v, t[u]);
          if (MODE != 0) stf4<NTS>(mb, v, m[u]);
          if (in) stf4<NTS>(in, v, t[u]);
        }
      }
      const int i = (nv << 2) + tid;
      if (i < ck.len) {
        const float g = float(int8_t(q[i])) * s;
        float b = (MODE == 2) ? mb[i] : 0.f, t1 = th[i];
        sgd1<MODE>(g, b, t1, a);
        th[i] = t1;
        if (MODE != 0) mb[i] = b;
        if (in) in[i] = t1;
      }
    } else {
      for (int i = tid; i < ck.len; i += kThreads) {
        const float g = float(int8_t(q[i])) * s;
        float b = (MODE == 2) ? mb[i] : 0.f, t1 = th[i];
        sgd1<MODE>(g, b, t1, a);
        th[i] = t1;
        if (MODE != 0) mb[i] = b;
        in[i] = t1;
      }
    }
  }
};

// Σ over n peers' copies of m slots (recv laid out [peer][slot]) -> averaged, re-quantised slots
__global__ void __launch_bounds__(kThreads)
    k_q8_reduce(const uint8_t* recv, int32_t n, int32_t m, int32_t divisor,
                uint8_t* out) {  // recv == out at one peer (in place): no __restrict__
  const int j = blockIdx.x;
  const int tid = threadIdx.x;
  float4 acc[kUnroll];
#pragma unroll
  for (int u = 0; u < kUnroll; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int r = 0; r < n; ++r) {  // rank order: the sum is identical on every peer
    const uint8_t* slot = recv + (size_t(r) * m + j) * DL_Q8_SLOT_BYTES;
    const float s = *reinterpret_cast<const float*>(slot);
    const uint8_t* q = slot + kQ8Header;
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const float4 x = unpack4(((gcu32)q)[u * kThreads + tid], s);
      acc[u] = make_float4(acc[u].x + x.x, acc[u].y + x.y, acc[u].z + x.z, acc[u].w + x.w);
    }
  }
  float am = 0.f;
#pragma unroll
  for (int u = 0; u < kUnroll; ++u) {
    if (divisor > 1) acc[u] = div4(acc[u], float(divisor));
    am = fmaxf(am, amax4(acc[u]));
  }
  const float s = block_amax(am) / 127.f;
  // the averaged payload leaves as one non-temporal 16-B store per lane (as in DeltaQ8)
  __shared__ u32x4 stage[DL_CHUNK_ELEMS / 16];
  uint32_t* st32 = reinterpret_cast<uint32_t*>(stage);
#pragma unroll
  for (int u = 0; u < kUnroll; ++u) st32[u * kThreads + tid] = pack4(acc[u], s);
  __syncthreads();
  uint8_t* o = out + size_t(j) * DL_Q8_SLOT_BYTES;
  __builtin_nontemporal_store(stage[tid], (DL_GLOBAL u32x4*)(o + kQ8Header) + tid);
  store_header<kStNT>(o, s, tid);
}

}  // namespace

hipError_t launch_delta_q8(const Launch& L, int inner_slot, const float* outer, uint8_t* slots) {
  return run(L, DeltaQ8{inner_slot, outer, slots, L.c0});
}

hipError_t launch_unpack_sgd_q8(const Launch& L, const uint8_t* slots, float* outer, float* mom,
                                SgdArgs a, int inner_slot) {
  if (a.momentum == 0.f) return run(L, UnpackSgdQ8<0>{slots, L.c0, outer, mom, a, inner_slot});
  if (a.first) return run(L, UnpackSgdQ8<1>{slots, L.c0, outer, mom, a, inner_slot});
  return run(L, UnpackSgdQ8<2>{slots, L.c0, outer, mom, a, inner_slot});
}

hipError_t launch_q8_reduce(const uint8_t* recv, int32_t n, int32_t m, int32_t divisor,
                            uint8_t* out, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_q8_reduce, dim3(m), dim3(kThreads), 0, s, recv, n, m, divisor, out);
  return hipGetLastError();
}

}  // namespace dl
