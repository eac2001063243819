// Why the int8 encoder (dl_delta_q8) runs below the 2-stream read rate: the same access shape on
// flat arrays of T1.3B's size, cold (a 1 GiB default-policy read+write evicts the Infinity
// Cache before every launch), variants interleaved round by round in one process.
//
//   read2      read θ, in (16 KB each per workgroup), nothing stored     8 B/elem, the ceiling
//   pack       read θ, in; write θ - in                                12 B/elem (dl_delta_pack)
//   q8_4160    read θ, in; amax over the chunk (LDS); quantise; 4 KB payload + 4-B scale into a
//              4160-B slot (the current wire: slots are not 128-B aligned)
//   q8_4224    the same into 4224-B slots (128-B header: every slot starts on a cache line)
//   q8_split   4096-B payload slots (aligned) + a dense fp32 scale array
//   q8_noscale q8_4160 without the 4-B scale store (payload only)
//   q8_nobar   q8_4160 with the amax taken per wave (no workgroup barrier; a per-1024 scale)
//   q8_lds*    the payload staged in LDS, one 16-B store per lane (plain / non-temporal);
//              _4224_h128: a 128-B header, so every payload starts on a cache line; plain ld:
//              default-policy loads instead of non-temporal
//   packbf_*   the bf16 wire's delta_pack (10 B/elem): 8-B stores per lane vs LDS-staged 16-B
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -fhip-fp32-correctly-rounded-divide-sqrt tools/q8_layout.hip -o build/q8_layout
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t err_ = (x);                                                     \
    if (err_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(err_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
#define G __attribute__((address_space(1)))
constexpr int T = 256;
constexpr int CH = 4096;  // elements per chunk (one workgroup)
constexpr int U = 4;      // float4 per lane per stream

__device__ __forceinline__ f4 ld(const float* p, long v) {
  return __builtin_nontemporal_load((const G f4*)(p) + v);
}
__device__ __forceinline__ f4 ldp(const float* p, long v) { return ((const G f4*)(p))[v]; }

__device__ __forceinline__ float amax4(f4 x) {
  return fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w)));
}

template <bool BAR>
__device__ __forceinline__ float chunk_amax(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  if constexpr (!BAR) return v;
  __shared__ float part[T / 64];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  v = fmaxf(fmaxf(part[0], part[1]), fmaxf(part[2], part[3]));
  __syncthreads();
  return v;
}

__device__ __forceinline__ int q8(float x, float s) {
  if (s == 0.f) return 0;
  return int(fminf(fmaxf(__builtin_rintf(x / s), -127.f), 127.f));
}

__device__ __forceinline__ unsigned pack4(f4 x, float s) {
  return (unsigned(q8(x.x, s)) & 0xffu) | ((unsigned(q8(x.y, s)) & 0xffu) << 8) |
         ((unsigned(q8(x.z, s)) & 0xffu) << 16) | ((unsigned(q8(x.w, s)) & 0xffu) << 24);
}

__global__ void __launch_bounds__(T) read2(const float* th, const float* in, float* sink) {
  const long base = long(blockIdx.x) * (CH / 4);
  f4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < U; ++u) acc += ld(th, base + u * T + threadIdx.x) - ld(in, base + u * T + threadIdx.x);
  if (acc.x == 123.456f) sink[threadIdx.x] = acc.y;  // never true: keeps the loads live
}

__global__ void __launch_bounds__(T) pack(const float* th, const float* in, float* w) {
  const long base = long(blockIdx.x) * (CH / 4);
  f4 d[U];
#pragma unroll
  for (int u = 0; u < U; ++u) d[u] = ld(th, base + u * T + threadIdx.x) - ld(in, base + u * T + threadIdx.x);
#pragma unroll
  for (int u = 0; u < U; ++u) ((G f4*)w)[base + u * T + threadIdx.x] = d[u];
}

// SLOT: slot stride in bytes, HDR: payload offset in the slot; SPLIT: scales in their own array
template <int SLOT, int HDR, bool SPLIT, bool SCALE, bool BAR>
__global__ void __launch_bounds__(T) q8enc(const float* th, const float* in, unsigned char* slots,
                                           float* scales) {
  const long base = long(blockIdx.x) * (CH / 4);
  f4 d[U];
  float am = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    d[u] = ld(th, base + u * T + threadIdx.x) - ld(in, base + u * T + threadIdx.x);
    am = fmaxf(am, amax4(d[u]));
  }
  const float s = chunk_amax<BAR>(am) / 127.f;
  unsigned char* slot = slots + size_t(blockIdx.x) * SLOT;
  G unsigned* q = (G unsigned*)(slot + HDR);
#pragma unroll
  for (int u = 0; u < U; ++u) q[u * T + threadIdx.x] = pack4(d[u], s);
  if (SCALE && (BAR ? threadIdx.x == 0 : (threadIdx.x & 63) == 0)) {
    if (SPLIT) scales[blockIdx.x * (BAR ? 1 : 4) + (BAR ? 0 : threadIdx.x >> 6)] = s;
    else *(G float*)(slot + (BAR ? 0 : 4 * (threadIdx.x >> 6))) = s;
  }
}

// the payload staged through LDS, then one 16-B store per lane (1 KB per wave instruction
// instead of four 256-B ones); NTS: non-temporal payload stores
template <int SLOT, int HDR, bool SPLIT, bool NTS, bool FULLHDR = false, bool NTL = true>
__global__ void __launch_bounds__(T) q8lds(const float* th, const float* in, unsigned char* slots,
                                           float* scales) {
  __shared__ unsigned stage[CH / 4];
  const long base = long(blockIdx.x) * (CH / 4);
  f4 d[U];
  float am = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    d[u] = NTL ? ld(th, base + u * T + threadIdx.x) - ld(in, base + u * T + threadIdx.x)
               : ldp(th, base + u * T + threadIdx.x) - ldp(in, base + u * T + threadIdx.x);
    am = fmaxf(am, amax4(d[u]));
  }
  const float s = chunk_amax<true>(am) / 127.f;
#pragma unroll
  for (int u = 0; u < U; ++u) stage[u * T + threadIdx.x] = pack4(d[u], s);
  __syncthreads();
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  const u4 v = reinterpret_cast<const u4*>(stage)[threadIdx.x];
  unsigned char* slot = slots + size_t(blockIdx.x) * SLOT;
  G u4* q = (G u4*)(slot + HDR);
  if constexpr (NTS) __builtin_nontemporal_store(v, q + threadIdx.x);
  else q[threadIdx.x] = v;
  if constexpr (FULLHDR && !SPLIT) {  // the whole header, scale then zeros, as 16-B stores
    if (threadIdx.x < HDR / 16) {
      const u4 h = {threadIdx.x == 0 ? __float_as_uint(s) : 0u, 0u, 0u, 0u};
      if constexpr (NTS) __builtin_nontemporal_store(h, (G u4*)slot + threadIdx.x);
      else ((G u4*)slot)[threadIdx.x] = h;
    }
  } else if (threadIdx.x == 0) {
    if (SPLIT) scales[blockIdx.x] = s;
    else *(G float*)slot = s;
  }
}

// bf16 wire (dl_delta_pack's bf16 shape, 10 B/elem): 4 bf16 = 8 B per lane per store as the
// product stores them, or the chunk's 8 KB staged in LDS and written as two 16-B stores per lane
__device__ __forceinline__ unsigned short bf16_rne(float x) {
  unsigned u = __float_as_uint(x);
  return (unsigned short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
typedef unsigned u2 __attribute__((ext_vector_type(2)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u2 bf4(f4 x) {
  return u2{unsigned(bf16_rne(x.x)) | (unsigned(bf16_rne(x.y)) << 16),
            unsigned(bf16_rne(x.z)) | (unsigned(bf16_rne(x.w)) << 16)};
}
template <bool NTS>
__global__ void __launch_bounds__(T) packbf_8(const float* th, const float* in, unsigned short* w) {
  const long base = long(blockIdx.x) * (CH / 4);
  f4 d[U];
#pragma unroll
  for (int u = 0; u < U; ++u) d[u] = ld(th, base + u * T + threadIdx.x) - ld(in, base + u * T + threadIdx.x);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    G u2* p = (G u2*)w + base + u * T + threadIdx.x;
    if constexpr (NTS) __builtin_nontemporal_store(bf4(d[u]), p);
    else *p = bf4(d[u]);
  }
}
template <bool NTS>
__global__ void __launch_bounds__(T) packbf_lds(const float* th, const float* in, unsigned short* w) {
  __shared__ u2 stage[CH / 4];
  const long base = long(blockIdx.x) * (CH / 4);
  f4 d[U];
#pragma unroll
  for (int u = 0; u < U; ++u) d[u] = ld(th, base + u * T + threadIdx.x) - ld(in, base + u * T + threadIdx.x);
#pragma unroll
  for (int u = 0; u < U; ++u) stage[u * T + threadIdx.x] = bf4(d[u]);
  __syncthreads();
  const u4v* s4 = reinterpret_cast<const u4v*>(stage);
  G u4v* o = (G u4v*)(w + base * 4);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const u4v v = s4[k * T + threadIdx.x];
    if constexpr (NTS) __builtin_nontemporal_store(v, o + k * T + threadIdx.x);
    else o[k * T + threadIdx.x] = v;
  }
}

__global__ void __launch_bounds__(T) flush_k(float* p, long n4) {
  for (long v = blockIdx.x * long(T) + threadIdx.x; v < n4; v += long(gridDim.x) * T) {
    f4 x = ((G f4*)p)[v];
    ((G f4*)p)[v] = x + 1.0f;
  }
}

__global__ void fill(float* p, long n, unsigned seed) {
  for (long i = blockIdx.x * long(T) + threadIdx.x; i < n; i += long(gridDim.x) * T) {
    unsigned z = unsigned(i) * 2654435761u + seed;
    z ^= z >> 15;
    p[i] = float(int(z & 0xFFFFF) - 0x80000) * 1e-6f;
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 9;
  const long nch = argc > 2 ? atol(argv[2]) : 320000;  // T1.3B: 320,734 chunks
  const long n = nch * CH;
  float *th, *in, *w, *sink, *flush, *scales;
  unsigned char* slots;
  CK(hipMalloc(&th, n * 4));
  CK(hipMalloc(&in, n * 4));
  CK(hipMalloc(&w, n * 4));
  CK(hipMalloc(&sink, 4096));
  CK(hipMalloc(&slots, nch * 4224));
  CK(hipMalloc(&scales, nch * 4 * 4));
  const long nf = 1L << 28;
  CK(hipMalloc(&flush, nf * 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(T), 0, 0, th, n, 1u);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(T), 0, 0, in, n, 2u);
  CK(hipMemset(flush, 0, nf * 4));
  CK(hipMemset(slots, 0, nch * 4224));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V {
    std::string name;
    double bytes;
    std::function<void()> run;
    std::vector<float> ms;
  };
  std::vector<V> vs;
  const dim3 g{unsigned(nch)}, b{unsigned(T)};
  const double q8b = 8.0 * n + 4160.0 * nch;  // algorithmic bytes of the current wire
#define ADD(name, bytes, ...) vs.push_back({name, double(bytes), [&]() { __VA_ARGS__; }, {}})
  ADD("read2      (8 B/elem ceiling)", 8.0 * n, hipLaunchKernelGGL(read2, g, b, 0, 0, th, in, sink));
  ADD("pack       (12 B/elem)       ", 12.0 * n, hipLaunchKernelGGL(pack, g, b, 0, 0, th, in, w));
  ADD("q8_4160    current wire      ", q8b, hipLaunchKernelGGL((q8enc<4160, 64, false, true, true>), g, b, 0, 0, th, in, slots, scales));
  ADD("q8_4224    128-B slots       ", q8b, hipLaunchKernelGGL((q8enc<4224, 128, false, true, true>), g, b, 0, 0, th, in, slots, scales));
  ADD("q8_split   4096 + scale array", q8b, hipLaunchKernelGGL((q8enc<4096, 0, true, true, true>), g, b, 0, 0, th, in, slots, scales));
  ADD("q8_noscale no scale store    ", q8b, hipLaunchKernelGGL((q8enc<4160, 64, false, false, true>), g, b, 0, 0, th, in, slots, scales));
  ADD("q8_nobar   per-wave amax     ", q8b, hipLaunchKernelGGL((q8enc<4160, 64, false, true, false>), g, b, 0, 0, th, in, slots, scales));
  ADD("q8_split_nobar               ", q8b, hipLaunchKernelGGL((q8enc<4096, 0, true, true, false>), g, b, 0, 0, th, in, slots, scales));
  ADD("q8_lds     4160, 16-B stores ", q8b, hipLaunchKernelGGL((q8lds<4160, 64, false, false>), g, b, 0, 0, th, in, slots, scales));
  ADD("q8_lds_nt  4160, NT 16-B     ", q8b, hipLaunchKernelGGL((q8lds<4160, 64, false, true>), g, b, 0, 0, th, in, slots, scales));
  ADD("q8_lds_nt_fullhdr (product) ", q8b, hipLaunchKernelGGL((q8lds<4160, 64, false, true, true>), g, b, 0, 0, th, in, slots, scales));
  ADD("q8_lds_nt_4224_h128 (aligned)", q8b, hipLaunchKernelGGL((q8lds<4224, 128, false, true, true>), g, b, 0, 0, th, in, slots, scales));
  ADD("q8_lds_nt_fullhdr plain loads", q8b, hipLaunchKernelGGL((q8lds<4160, 64, false, true, true, false>), g, b, 0, 0, th, in, slots, scales));
  ADD("q8_lds_nt_4224_h128 plain ld ", q8b, hipLaunchKernelGGL((q8lds<4224, 128, false, true, true, false>), g, b, 0, 0, th, in, slots, scales));
  ADD("q8_lds_split 4096+scales     ", q8b, hipLaunchKernelGGL((q8lds<4096, 0, true, false>), g, b, 0, 0, th, in, slots, scales));
  ADD("q8_lds_split_nt              ", q8b, hipLaunchKernelGGL((q8lds<4096, 0, true, true>), g, b, 0, 0, th, in, slots, scales));
  unsigned short* wb = reinterpret_cast<unsigned short*>(w);
  ADD("packbf_8   8-B stores        ", 10.0 * n, hipLaunchKernelGGL(packbf_8<false>, g, b, 0, 0, th, in, wb));
  ADD("packbf_8   8-B NT stores     ", 10.0 * n, hipLaunchKernelGGL(packbf_8<true>, g, b, 0, 0, th, in, wb));
  ADD("packbf_lds 16-B stores       ", 10.0 * n, hipLaunchKernelGGL(packbf_lds<false>, g, b, 0, 0, th, in, wb));
  ADD("packbf_lds 16-B NT stores    ", 10.0 * n, hipLaunchKernelGGL(packbf_lds<true>, g, b, 0, 0, th, in, wb));
  for (int r = 0; r < rounds; ++r) {
    for (auto& v : vs) {
      hipLaunchKernelGGL(flush_k, dim3(8192), dim3(T), 0, 0, flush, nf / 4);
      CK(hipEventRecord(e0, 0));
      v.run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
  }
  CK(hipGetLastError());
  printf("int8 encoder shapes, %ld chunks (%ld fp32 per stream), %d rounds, cold\n", nch, n, rounds);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("%s med %8.4f ms %7.1f GB/s  best %7.1f GB/s\n", v.name.c_str(), med,
           v.bytes / med / 1e6, v.bytes / v.ms[0] / 1e6);
  }
  return 0;
}
