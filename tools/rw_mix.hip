// Does the fused one-replica step (read 3 streams, write 4: dl_delta_pack_sgd's 12 + 16 B per
// element) lose bandwidth to mixing reads and writes, or is it at the rate its read half and
// write half reach on their own? Cold (a 1 GiB default-policy read+write evicts the Infinity
// Cache before every timed launch), T125-size arrays, variants interleaved round by round.
//
//   read3        read θ, in, m                    the step's read half, 12 B/elem
//   write4       write w, θ', m', in'             the step's write half, 16 B/elem
//   read3+write4 the two as back-to-back kernels in one timed window (phase-separated)
//   fused        read 3, write 4 per workgroup    the product kernel's shape, 28 B/elem
//   read1 / write1 / copy                         single-stream reference points
//   fused, phased   persistent cooperative grid, a grid barrier between every round's loads
//                   and its stores (chip-wide read-only / write-only periods)
//   staged          phases split by kernel boundaries, results staged in the Infinity Cache
// If t(fused) ~= t(read3) + t(write4), the mix costs nothing and the step is bounded by the
// time HBM needs for its read bytes plus its write bytes: t >= R/BW_read + W/BW_write.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/rw_mix.hip -o build/rw_mix
//   build/rw_mix [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
#define G __attribute__((address_space(1)))
constexpr int T = 256;
constexpr int U = 4;  // float4 per lane per stream: one workgroup = 4096 elements, as the walker

template <bool NT = true>
__device__ __forceinline__ f4 ld(const float* p, long v) {
  if constexpr (NT) return __builtin_nontemporal_load((const G f4*)(p) + v);
  else return *((const G f4*)(p) + v);
}
template <bool NT = true>
__device__ __forceinline__ void st(float* p, long v, f4 x) {
  if constexpr (NT) __builtin_nontemporal_store(x, (G f4*)(p) + v);
  else *((G f4*)(p) + v) = x;
}

__device__ __forceinline__ long tile_base() { return long(blockIdx.x) * (U * T); }

// read S streams, keep the sum live
template <int S>
__global__ void __launch_bounds__(T) readS(const float* a, const float* b, const float* c,
                                           float* sink) {
  const float* src[3] = {a, b, c};
  f4 x[S][U];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int u = 0; u < U; ++u) x[s][u] = ld(src[s], tile_base() + u * T + threadIdx.x);
  f4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int u = 0; u < U; ++u) acc += x[s][u];
  if (acc.x == 123.456f) st(sink, threadIdx.x, acc);  // never true: keeps the loads live
}

// write S streams of a value computed from the index
template <int S, bool NT>
__global__ void __launch_bounds__(T) writeS(float* a, float* b, float* c, float* d) {
  float* dst[4] = {a, b, c, d};
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long v = tile_base() + u * T + threadIdx.x;
      const float f = float(v) * 1e-9f + float(s);
      st<NT>(dst[s], v, f4{f, f, f, f});
    }
}

__global__ void __launch_bounds__(T) copy1(const float* a, float* b) {
  f4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = ld(a, tile_base() + u * T + threadIdx.x);
#pragma unroll
  for (int u = 0; u < U; ++u) st(b, tile_base() + u * T + threadIdx.x, x[u]);
}

// the product kernel's shape: read θ, in, m; write w (plain), θ, m, in (non-temporal)
__global__ void __launch_bounds__(T) fused(float* th, float* in, float* mb, float* w) {
  f4 t[U], x[U], m[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long v = tile_base() + u * T + threadIdx.x;
    t[u] = ld(th, v);
    x[u] = ld(in, v);
    m[u] = ld(mb, v);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    x[u] = t[u] - x[u];
    m[u] = m[u] * 0.9f + x[u];
    t[u] = t[u] - 0.7f * (x[u] + 0.9f * m[u]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) st<false>(w, tile_base() + u * T + threadIdx.x, x[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) st(th, tile_base() + u * T + threadIdx.x, t[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) st(mb, tile_base() + u * T + threadIdx.x, m[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) st(in, tile_base() + u * T + threadIdx.x, t[u]);
}

// fused with θ and momentum interleaved in ONE array (one stream fewer each way):
// IL = 0: per 4096-element tile (θ tile, then its m tile); IL = 1: per float4 (θ4, m4, θ4, ...)
template <int IL>
__global__ void __launch_bounds__(T) fused_il(float* tm, float* in, float* w) {
  f4 t[U], x[U], m[U];
  const long b = tile_base();
  auto ti = [&](int u) { return IL == 0 ? 2 * b + u * T + threadIdx.x : 2 * (b + u * T + threadIdx.x); };
  auto mi = [&](int u) { return IL == 0 ? 2 * b + U * T + u * T + threadIdx.x : 2 * (b + u * T + threadIdx.x) + 1; };
#pragma unroll
  for (int u = 0; u < U; ++u) {
    t[u] = ld(tm, ti(u));
    x[u] = ld(in, b + u * T + threadIdx.x);
    m[u] = ld(tm, mi(u));
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    x[u] = t[u] - x[u];
    m[u] = m[u] * 0.9f + x[u];
    t[u] = t[u] - 0.7f * (x[u] + 0.9f * m[u]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) st(w, b + u * T + threadIdx.x, x[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    st(tm, ti(u), t[u]);
    st(tm, mi(u), m[u]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) st(in, b + u * T + threadIdx.x, t[u]);
}

// the product kernel exactly (all four stores non-temporal)
__global__ void __launch_bounds__(T) fused_nt(float* th, float* in, float* mb, float* w) {
  f4 t[U], x[U], m[U];
  const long b = tile_base();
#pragma unroll
  for (int u = 0; u < U; ++u) {
    t[u] = ld(th, b + u * T + threadIdx.x);
    x[u] = ld(in, b + u * T + threadIdx.x);
    m[u] = ld(mb, b + u * T + threadIdx.x);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    x[u] = t[u] - x[u];
    m[u] = m[u] * 0.9f + x[u];
    t[u] = t[u] - 0.7f * (x[u] + 0.9f * m[u]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) st(w, b + u * T + threadIdx.x, x[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) st(th, b + u * T + threadIdx.x, t[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) st(mb, b + u * T + threadIdx.x, m[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) st(in, b + u * T + threadIdx.x, t[u]);
}

// The fused step with chip-wide phases: a persistent grid (every workgroup resident,
// cooperative launch) where each round every workgroup loads one tile (3 streams), all meet at a
// grid barrier, then every workgroup stores (4 streams) and all meet again -- HBM sees read-only
// and write-only periods instead of a steady mix. The barrier spins a bounded number of times
// (a non-resident workgroup would make it fall through, recorded in bar[2], never hang).
__device__ __forceinline__ void grid_barrier(unsigned* bar, unsigned nwg) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (atomicAdd(&bar[0], 1u) == nwg - 1) {
      __hip_atomic_store(&bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&bar[1], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned budget = 1u << 22;
      while (__hip_atomic_load(&bar[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g && --budget)
        __builtin_amdgcn_s_sleep(1);
      if (!budget) atomicAdd(&bar[2], 1u);
    }
  }
  __syncthreads();
}

__global__ void __launch_bounds__(T) fused_phased(float* th, float* in, float* mb, float* w,
                                                  long ntiles, unsigned* bar) {
  const unsigned nwg = gridDim.x;
  for (long t0 = 0; t0 < ntiles; t0 += nwg) {
    const long tile = t0 + blockIdx.x;
    const bool on = tile < ntiles;
    const long b = tile * (U * T);
    f4 t[U], x[U], m[U];
    if (on) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        t[u] = ld(th, b + u * T + threadIdx.x);
        x[u] = ld(in, b + u * T + threadIdx.x);
        m[u] = ld(mb, b + u * T + threadIdx.x);
      }
    }
    grid_barrier(bar, nwg);
    if (on) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        x[u] = t[u] - x[u];
        m[u] = m[u] * 0.9f + x[u];
        t[u] = t[u] - 0.7f * (x[u] + 0.9f * m[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) st(w, b + u * T + threadIdx.x, x[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) st(th, b + u * T + threadIdx.x, t[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) st(mb, b + u * T + threadIdx.x, m[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) st(in, b + u * T + threadIdx.x, t[u]);
    }
    grid_barrier(bar, nwg);
  }
}

// the same persistent loop without the barriers (is the persistent shape itself slower?)
__global__ void __launch_bounds__(T) fused_persistent(float* th, float* in, float* mb, float* w,
                                                      long ntiles) {
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const long b = tile * (U * T);
    f4 t[U], x[U], m[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      t[u] = ld(th, b + u * T + threadIdx.x);
      x[u] = ld(in, b + u * T + threadIdx.x);
      m[u] = ld(mb, b + u * T + threadIdx.x);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = t[u] - x[u];
      m[u] = m[u] * 0.9f + x[u];
      t[u] = t[u] - 0.7f * (x[u] + 0.9f * m[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st(w, b + u * T + threadIdx.x, x[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) st(th, b + u * T + threadIdx.x, t[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) st(mb, b + u * T + threadIdx.x, m[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) st(in, b + u * T + threadIdx.x, t[u]);
  }
}

// Phases separated by kernel boundaries, the step's results staged in the Infinity Cache: per
// tile of `tile` workgroups, stage_a reads θ, in, m from HBM (non-temporal) and stores θ', m', w
// into a small staging area with default (allocating) stores -- reused every tile, so its lines
// stay in the 256 MiB Infinity Cache and never go to HBM; stage_b reads the staging area back
// (cache hits) and stores w, θ, m, in to HBM (non-temporal). HBM sees a read-only kernel, then a
// write-only kernel, tile after tile.
__global__ void __launch_bounds__(T) stage_a(const float* th, const float* in, const float* mb,
                                             long t0, float* stg) {
  const long b = (t0 + blockIdx.x) * long(U * T);
  const long sb = long(blockIdx.x) * (3 * U * T);
  f4 t[U], x[U], m[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    t[u] = ld(th, b + u * T + threadIdx.x);
    x[u] = ld(in, b + u * T + threadIdx.x);
    m[u] = ld(mb, b + u * T + threadIdx.x);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    x[u] = t[u] - x[u];
    m[u] = m[u] * 0.9f + x[u];
    t[u] = t[u] - 0.7f * (x[u] + 0.9f * m[u]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    st<false>(stg, sb + u * T + threadIdx.x, x[u]);
    st<false>(stg, sb + (U + u) * T + threadIdx.x, t[u]);
    st<false>(stg, sb + (2 * U + u) * T + threadIdx.x, m[u]);
  }
}

template <bool NTL>
__global__ void __launch_bounds__(T) stage_b(const float* stg, long t0, float* th, float* in,
                                             float* mb, float* w) {
  const long b = (t0 + blockIdx.x) * long(U * T);
  const long sb = long(blockIdx.x) * (3 * U * T);
  f4 x[U], t[U], m[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    x[u] = ld<NTL>(stg, sb + u * T + threadIdx.x);
    t[u] = ld<NTL>(stg, sb + (U + u) * T + threadIdx.x);
    m[u] = ld<NTL>(stg, sb + (2 * U + u) * T + threadIdx.x);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) st(w, b + u * T + threadIdx.x, x[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) st(th, b + u * T + threadIdx.x, t[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) st(mb, b + u * T + threadIdx.x, m[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) st(in, b + u * T + threadIdx.x, t[u]);
}

// The fused step with clock-slotted phases and no communication: a persistent grid where every
// workgroup aligns its rounds to absolute slots of the chip's 100 MHz real-time counter
// (s_memrealtime): loads at the slot's start, stores `rt` ticks later, next round at the next
// slot -- all workgroups read together, then write together, so HBM sees read and write
// periods without a barrier. Every wait ends when the counter passes a target within one
// period of the current time.
__device__ __forceinline__ unsigned long long rtc() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void wait_until(unsigned long long t) {
  while (rtc() < t) __builtin_amdgcn_s_sleep(2);
  __asm__ volatile("" ::: "memory");
}

template <bool NTW>
__global__ void __launch_bounds__(T) fused_slotted(float* th, float* in, float* mb, float* w,
                                                   long ntiles, unsigned period, unsigned rt) {
  // round k of this workgroup runs in slot epoch + k * period; a workgroup behind schedule
  // (target already past) goes at once instead of skipping a slot
  const unsigned long long epoch = (rtc() / period + 1) * period;
  unsigned long long slot = epoch;
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x, slot += period) {
    wait_until(slot);
    const long b = tile * (U * T);
    f4 t[U], x[U], m[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      t[u] = ld(th, b + u * T + threadIdx.x);
      x[u] = ld(in, b + u * T + threadIdx.x);
      m[u] = ld(mb, b + u * T + threadIdx.x);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = t[u] - x[u];
      m[u] = m[u] * 0.9f + x[u];
      t[u] = t[u] - 0.7f * (x[u] + 0.9f * m[u]);
    }
    __asm__ volatile("" ::: "memory");
    wait_until(slot + rt);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTW>(w, b + u * T + threadIdx.x, x[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) st(th, b + u * T + threadIdx.x, t[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) st(mb, b + u * T + threadIdx.x, m[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) st(in, b + u * T + threadIdx.x, t[u]);
  }
}

// default-policy (allocating) loads and stores over 1 GiB: evicts the Infinity Cache
__global__ void __launch_bounds__(T) flush_k(float* p) {
  f4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = ld<false>(p, tile_base() + u * T + threadIdx.x);
#pragma unroll
  for (int u = 0; u < U; ++u) st<false>(p, tile_base() + u * T + threadIdx.x, x[u] + 1.0f);
}

__global__ void fill(float* p, long n, unsigned seed) {
  for (long i = blockIdx.x * long(T) + threadIdx.x; i < n; i += long(gridDim.x) * T) {
    unsigned z = unsigned(i) * 2654435761u + seed;
    z ^= z >> 15;
    p[i] = float(int(z & 0xFFFFF) - 0x80000) * 1e-6f;
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 15;
  // T125 (124,475,904) or, with a second argument "t1.3b", T1.3B (1,313,722,368), rounded
  // down to whole 4096-element tiles
  const bool big = argc > 2 && std::string(argv[2]) == "t1.3b";
  const long n = big ? 1313722368L / 4096 * 4096 : 124473344L;
  const unsigned grid = unsigned(n / (U * T * 4));
  float* buf[7];
  for (auto& p : buf) {
    CK(hipMalloc(&p, n * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(T), 0, 0, p, n, unsigned(&p - buf) + 1);
  }
  float *sink, *flush;
  CK(hipMalloc(&sink, 4096));
  const long nf = 1L << 28;  // 1 GiB
  CK(hipMalloc(&flush, nf * 4));
  CK(hipMemset(flush, 0, nf * 4));
  const unsigned fgrid = unsigned(nf / (U * T * 4));
  float* tm;  // θ and m interleaved: 2n floats
  CK(hipMalloc(&tm, 2 * n * 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(T), 0, 0, tm, 2 * n, 99u);
  float *th = buf[0], *in = buf[1], *mb = buf[2], *w = buf[3], *x = buf[4], *y = buf[5], *z = buf[6];
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
#define ADD(name, bytes, ...) vs.push_back({name, double(bytes) * n, [&]() { __VA_ARGS__; }, {}})
  ADD("read1                 ", 4, hipLaunchKernelGGL(readS<1>, dim3(grid), dim3(T), 0, 0, th, in, mb, sink));
  ADD("read3  (step's reads) ", 12, hipLaunchKernelGGL(readS<3>, dim3(grid), dim3(T), 0, 0, th, in, mb, sink));
  ADD("write1 NT             ", 4, hipLaunchKernelGGL((writeS<1, true>), dim3(grid), dim3(T), 0, 0, x, y, z, w));
  ADD("write1 plain          ", 4, hipLaunchKernelGGL((writeS<1, false>), dim3(grid), dim3(T), 0, 0, x, y, z, w));
  ADD("write2 NT             ", 8, hipLaunchKernelGGL((writeS<2, true>), dim3(grid), dim3(T), 0, 0, x, y, z, w));
  ADD("write3 NT             ", 12, hipLaunchKernelGGL((writeS<3, true>), dim3(grid), dim3(T), 0, 0, x, y, z, w));
  ADD("write4 NT (step's wr.)", 16, hipLaunchKernelGGL((writeS<4, true>), dim3(grid), dim3(T), 0, 0, x, y, z, w));
  ADD("write4 plain          ", 16, hipLaunchKernelGGL((writeS<4, false>), dim3(grid), dim3(T), 0, 0, x, y, z, w));
  ADD("copy                  ", 8, hipLaunchKernelGGL(copy1, dim3(grid), dim3(T), 0, 0, th, x));
  ADD("read3 + write4 (2 k.) ", 28,
      hipLaunchKernelGGL(readS<3>, dim3(grid), dim3(T), 0, 0, th, in, mb, sink);
      hipLaunchKernelGGL((writeS<4, true>), dim3(grid), dim3(T), 0, 0, x, y, z, w));
  ADD("fused (3 r + 4 w)     ", 28, hipLaunchKernelGGL(fused, dim3(grid), dim3(T), 0, 0, th, in, mb, w));
  ADD("fused, all NT stores  ", 28, hipLaunchKernelGGL(fused_nt, dim3(grid), dim3(T), 0, 0, th, in, mb, w));
  int per_cu = 0, cus = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fused_phased, T, 0));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  unsigned* bar;
  CK(hipMalloc(&bar, 16));
  CK(hipMemset(bar, 0, 16));
  long ntiles = long(grid);
  const unsigned pgrid = unsigned(per_cu * cus);
  printf("persistent grid: %d workgroups per CU x %d CUs = %u\n", per_cu, cus, pgrid);
  auto coop = [&](unsigned g) {
    void* args[] = {&th, &in, &mb, &w, &ntiles, &bar};
    CK(hipLaunchCooperativeKernel((const void*)fused_phased, dim3(g), dim3(T), args, 0, 0));
  };
  float* stg;
  CK(hipMalloc(&stg, 256L << 20));
  auto staged = [&](long tile) {
    for (long t0 = 0; t0 < ntiles; t0 += tile) {
      const unsigned g = unsigned(std::min(tile, ntiles - t0));
      hipLaunchKernelGGL(stage_a, dim3(g), dim3(T), 0, 0, th, in, mb, t0, stg);
      hipLaunchKernelGGL(stage_b<false>, dim3(g), dim3(T), 0, 0, stg, t0, th, in, mb, w);
    }
  };
  // tile = workgroups per kernel; staging = 48 KiB per workgroup
  ADD("staged, 32 MiB tiles  ", 28, staged(683));
  ADD("staged, 64 MiB tiles  ", 28, staged(1365));
  ADD("staged, 96 MiB tiles  ", 28, staged(2048));
  ADD("staged, 128 MiB tiles ", 28, staged(2730));
  ADD("staged, 192 MiB tiles ", 28, staged(4096));
  ADD("fused, persistent     ", 28, hipLaunchKernelGGL(fused_persistent, dim3(pgrid), dim3(T), 0, 0, th, in, mb, w, ntiles));
  ADD("fused, phased (grid barrier)", 28, coop(pgrid));
  int per_cu_s = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_s, fused_slotted<true>, T, 0));
  const unsigned sgrid = unsigned(per_cu_s * cus);
  printf("slotted grid: %d workgroups per CU x %d CUs = %u\n", per_cu_s, cus, sgrid);
  // (period, read window) in 10-ns ticks; one round moves sgrid x 48 KiB in, x 64 KiB out
  static const unsigned periods[] = {3400, 3600, 3800, 4000, 4200};
  for (int ntw = 1; ntw >= 0; --ntw)
    for (unsigned P : periods) {
      char nm[64];
      snprintf(nm, sizeof nm, "fused, slotted P=%u%s", P, ntw ? "" : " plain w");
      const unsigned R = P * 38 / 100;
      vs.push_back({nm, 28.0 * n, [&, P, R, ntw]() {
        if (ntw)
          hipLaunchKernelGGL(fused_slotted<true>, dim3(sgrid), dim3(T), 0, 0, th, in, mb, w, ntiles, P, R);
        else
          hipLaunchKernelGGL(fused_slotted<false>, dim3(sgrid), dim3(T), 0, 0, th, in, mb, w, ntiles, P, R);
      }, {}});
    }
  ADD("fused, θ|m per tile   ", 28, hipLaunchKernelGGL(fused_il<0>, dim3(grid), dim3(T), 0, 0, tm, in, w));
  ADD("fused, θ|m per float4 ", 28, hipLaunchKernelGGL(fused_il<1>, dim3(grid), dim3(T), 0, 0, tm, in, w));
  for (int r = 0; r < rounds; ++r) {
    for (auto& v : vs) {
      hipLaunchKernelGGL(flush_k, dim3(fgrid), dim3(T), 0, 0, flush);
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
  unsigned hb[4] = {0, 0, 0, 0};
  CK(hipMemcpy(hb, bar, 16, hipMemcpyDeviceToHost));
  printf("grid barrier: %u generations, %u timed-out waits\n", hb[1], hb[2]);
  printf("%s-size arrays (n=%ld fp32), %d rounds, Infinity Cache evicted before each launch\n",
         big ? "T1.3B" : "T125", n, rounds);
  double med_r3 = 0, med_w4 = 0, med_f = 0;
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("%s med %8.4f ms %7.1f GB/s  best %7.1f GB/s\n", v.name.c_str(), med,
           v.bytes / med / 1e6, v.bytes / v.ms[0] / 1e6);
    if (v.name.rfind("read3  ", 0) == 0) med_r3 = med;
    if (v.name.rfind("write4 NT", 0) == 0) med_w4 = med;
    if (v.name.rfind("fused, all NT", 0) == 0) med_f = med;
  }
  printf("model t(read3) + t(write4 NT) = %.4f ms -> %.1f GB/s for 28 B/elem; fused %.4f ms (%.3f of the model's time)\n",
         med_r3 + med_w4, 28.0 * n / (med_r3 + med_w4) / 1e6, med_f, med_f / (med_r3 + med_w4));
  return 0;
}
