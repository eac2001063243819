// Which cache policy should the hot path's streaming stores carry? The walker stores through
// `global_store_dwordx4` either plain or `nt`; both keep the written line in the XCD's L2
// (write-back, evicted later), while `sc1` / `sc0 sc1` stores are write-through and drop it
// (MI355X_MICROARCH.md, stores of each flavour). This times the step's write shapes with every
// policy, cold (a 1 GiB default-policy read+write evicts the Infinity Cache before each timed
// launch), T125-size arrays (or T1.3B with a second argument "t1.3b"), variants interleaved
// round by round:
//   write1 / write4      1 or 4 write-only streams (the headline's write half)
//   copy                 1 NT read stream -> 1 write stream
//   fused                dl_delta_pack_sgd's shape: 3 NT read streams, 4 write streams
// Stores go through __builtin_amdgcn_raw_buffer_store_b128 with the policy in `aux`
// (gfx950: bit 0 = sc0, bit 1 = nt, bit 4 = sc1); the descriptor covers the workgroup's
// 16 KiB tile of each stream and is built from blockIdx-derived (wave-uniform) values.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/store_policy.hip -o build/store_policy
//   build/store_policy [rounds] [t1.3b]
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
typedef unsigned u4 __attribute__((ext_vector_type(4)));
#define G __attribute__((address_space(1)))
constexpr int T = 256;
constexpr int U = 4;  // float4 per lane per stream: one workgroup = 4096 elements, as the walker
constexpr int kTileBytes = U * T * 16;

// the workgroup's first float4 (one workgroup = U * T float4 = 4096 elements)
__device__ __forceinline__ long tile_base() { return long(blockIdx.x) * (U * T); }

__device__ __forceinline__ f4 ldnt(const float* p, long v) {
  return __builtin_nontemporal_load((const G f4*)(p) + v);
}

// the workgroup's tile of one stream as a buffer resource (wave-uniform inputs only)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(p + 4 * tile_base(), 0, kTileBytes, 0x00020000);
}

template <int AUX>
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, int u, f4 x) {
  const int off = (u * T + int(threadIdx.x)) * 16;
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, x), r, off, 0, AUX);
}

template <int S, int AUX>
__global__ void __launch_bounds__(T) writeS(float* a, float* b, float* c, float* d) {
  float* dst[4] = {a, b, c, d};
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const __amdgpu_buffer_rsrc_t r = tile_rsrc(dst[s]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float f = float(tile_base() + u * T + threadIdx.x) * 1e-9f + float(s);
      st<AUX>(r, u, f4{f, f, f, f});
    }
  }
}

template <int AUX>
__global__ void __launch_bounds__(T) copy1(const float* a, float* b) {
  f4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = ldnt(a, tile_base() + u * T + threadIdx.x);
  const __amdgpu_buffer_rsrc_t r = tile_rsrc(b);
#pragma unroll
  for (int u = 0; u < U; ++u) st<AUX>(r, u, x[u]);
}

// dl_delta_pack_sgd's shape: read θ, in, m; write w, θ', m', in' one stream at a time
template <int AUX>
__global__ void __launch_bounds__(T) fused(float* th, float* in, float* mb, float* w) {
  f4 t[U], x[U], m[U];
  const long b = tile_base();
#pragma unroll
  for (int u = 0; u < U; ++u) {
    t[u] = ldnt(th, b + u * T + threadIdx.x);
    x[u] = ldnt(in, b + u * T + threadIdx.x);
    m[u] = ldnt(mb, b + u * T + threadIdx.x);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    x[u] = t[u] - x[u];
    m[u] = m[u] * 0.9f + x[u];
    t[u] = t[u] - 0.7f * (x[u] + 0.9f * m[u]);
  }
  const __amdgpu_buffer_rsrc_t rw = tile_rsrc(w), rt = tile_rsrc(th), rm = tile_rsrc(mb),
                               ri = tile_rsrc(in);
#pragma unroll
  for (int u = 0; u < U; ++u) st<AUX>(rw, u, x[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) st<AUX>(rt, u, t[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) st<AUX>(rm, u, m[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) st<AUX>(ri, u, t[u]);
}

// default-policy (allocating) loads and stores over 1 GiB: evicts the Infinity Cache
__global__ void __launch_bounds__(T) flush_k(float* p) {
  f4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = *((const G f4*)(p) + tile_base() + u * T + threadIdx.x);
#pragma unroll
  for (int u = 0; u < U; ++u) *((G f4*)(p) + tile_base() + u * T + threadIdx.x) = x[u] + 1.0f;
}

__global__ void fill(float* p, long n, unsigned seed) {
  for (long i = blockIdx.x * long(T) + threadIdx.x; i < n; i += long(gridDim.x) * T) {
    unsigned z = unsigned(i) * 2654435761u + seed;
    z ^= z >> 15;
    p[i] = float(int(z & 0xFFFFF) - 0x80000) * 1e-6f;
  }
}

__global__ void check_k(const float* p, long n, unsigned* bad) {
  for (long i = blockIdx.x * long(T) + threadIdx.x; i < n; i += long(gridDim.x) * T) {
    const float f = float(i >> 2) * 1e-9f;  // stream 0 of writeS (one value per float4)
    if (p[i] != f) atomicAdd(bad, 1u);
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 11;
  const bool big = argc > 2 && std::string(argv[2]) == "t1.3b";
  const long n = big ? 1313722368L / 4096 * 4096 : 124473344L;  // whole 4096-element tiles
  const unsigned grid = unsigned(n / (U * T * 4));
  float* buf[7];
  for (auto& p : buf) {
    CK(hipMalloc(&p, n * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(T), 0, 0, p, n, unsigned(&p - buf) + 1);
  }
  float* flush;
  const long nf = 1L << 28;  // 1 GiB
  CK(hipMalloc(&flush, nf * 4));
  CK(hipMemset(flush, 0, nf * 4));
  const unsigned fgrid = unsigned(nf / (U * T * 4));
  float *th = buf[0], *in = buf[1], *mb = buf[2], *w = buf[3], *x = buf[4], *y = buf[5], *z = buf[6];

  // every policy stores what it should (stream 0 of write1 checked element by element)
  unsigned* bad;
  CK(hipMalloc(&bad, 4));
  auto verify = [&](const char* nm, auto launch) {
    CK(hipMemset(x, 0, n * 4));
    CK(hipMemset(bad, 0, 4));
    launch();
    hipLaunchKernelGGL(check_k, dim3(4096), dim3(T), 0, 0, x, n, bad);
    unsigned h = 0;
    CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
    printf("check %-8s %s (%u wrong)\n", nm, h ? "FAILED" : "ok", h);
  };
#define VER(nm, AUX) \
  verify(nm, [&]() { hipLaunchKernelGGL((writeS<1, AUX>), dim3(grid), dim3(T), 0, 0, x, y, z, w); })
  VER("plain", 0);
  VER("nt", 2);
  VER("sc1", 16);
  VER("sc0 sc1", 17);
  VER("sc1 nt", 18);

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
#define POLICY(tag, AUX)                                                                        \
  ADD("write1 " tag, 4, hipLaunchKernelGGL((writeS<1, AUX>), dim3(grid), dim3(T), 0, 0, x, y, z, w)); \
  ADD("write4 " tag, 16, hipLaunchKernelGGL((writeS<4, AUX>), dim3(grid), dim3(T), 0, 0, x, y, z, w)); \
  ADD("copy   " tag, 8, hipLaunchKernelGGL((copy1<AUX>), dim3(grid), dim3(T), 0, 0, th, x));          \
  ADD("fused  " tag, 28, hipLaunchKernelGGL((fused<AUX>), dim3(grid), dim3(T), 0, 0, th, in, mb, w))
  POLICY("plain  ", 0);
  POLICY("nt     ", 2);
  POLICY("sc1    ", 16);
  POLICY("sc0 sc1", 17);
  POLICY("sc1 nt ", 18);
  POLICY("sc0 nt ", 3);
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
  printf("%s-size arrays (n=%ld fp32), %d rounds, Infinity Cache evicted before each launch\n",
         big ? "T1.3B" : "T125", n, rounds);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("%s med %8.4f ms %7.1f GB/s  best %7.1f GB/s\n", v.name.c_str(), med,
           v.bytes / med / 1e6, v.bytes / v.ms[0] / 1e6);
  }
  return 0;
}
