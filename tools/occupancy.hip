// Does the headline step lose HBM efficiency to too many concurrent streams? With one
// workgroup per 4096-element tile and ~7 workgroups per CU, ~1,800 workgroups each stream 7
// separate 16 KiB runs (3 reads, 4 writes) at once: ~12,600 concurrent runs spread over the
// HBM banks, far more bytes in flight than the latency-bandwidth product needs
// (8 TB/s x ~1.3 us ~ 10 MiB chip-wide). Fewer concurrent runs might keep DRAM rows open
// longer. Two ways to cut them, cold (a 1 GiB default-policy read+write evicts the Infinity
// Cache before every timed launch), T125-size arrays (T1.3B with a second argument "t1.3b"),
// variants interleaved round by round:
//   k WG/CU   dynamic LDS reserved per workgroup so that only k workgroups fit on a CU
//   M tiles   each workgroup walks M consecutive tiles one after another (grid / M): every
//             stream is read and written in runs of M x 16 KiB by one workgroup
// for the fused 7-stream shape (dl_delta_pack_sgd's: read θ, in, m; write w, θ', m', in',
// NT loads and stores), its write half alone (4 NT streams) and its read half alone.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/occupancy.hip -o build/occupancy
//   build/occupancy [rounds] [t1.3b]
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
constexpr int U = 4;  // float4 per lane per stream: one tile = 4096 elements, as the walker

__device__ __forceinline__ f4 ld(const float* p, long v) {
  return __builtin_nontemporal_load((const G f4*)(p) + v);
}
__device__ __forceinline__ void st(float* p, long v, f4 x) {
  __builtin_nontemporal_store(x, (G f4*)(p) + v);
}

// The dynamic LDS of the launch (and so the occupancy limit) is reserved by the dispatcher
// whether or not the kernel touches it; this reference only runs for ntiles < 0 (never).
__device__ __forceinline__ void keep_lds(long ntiles) {
  extern __shared__ float lds[];
  if (ntiles < 0) lds[threadIdx.x] = 0.f;
}

__device__ __forceinline__ void fused_tile(float* th, float* in, float* mb, float* w, long tile) {
  f4 t[U], x[U], m[U];
  const long b = tile * (U * T);
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

template <int M>
__global__ void __launch_bounds__(T) fused(float* th, float* in, float* mb, float* w, long ntiles) {
  for (int j = 0; j < M; ++j) {
    const long tile = long(blockIdx.x) * M + j;
    keep_lds(ntiles);
    if (tile < ntiles) fused_tile(th, in, mb, w, tile);
  }
}

template <int M>
__global__ void __launch_bounds__(T) write4(float* a, float* b, float* c, float* d, long ntiles) {
  float* dst[4] = {a, b, c, d};
  for (int j = 0; j < M; ++j) {
    const long tile = long(blockIdx.x) * M + j;
    keep_lds(ntiles);
    if (tile >= ntiles) break;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long v = tile * (U * T) + u * T + threadIdx.x;
        const float f = float(v) * 1e-9f + float(s);
        st(dst[s], v, f4{f, f, f, f});
      }
  }
}

template <int M>
__global__ void __launch_bounds__(T) read3(const float* a, const float* b, const float* c,
                                           float* sink, long ntiles) {
  f4 acc = {0, 0, 0, 0};
  for (int j = 0; j < M; ++j) {
    const long tile = long(blockIdx.x) * M + j;
    keep_lds(ntiles);
    if (tile >= ntiles) break;
    f4 x[3][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long v = tile * (U * T) + u * T + threadIdx.x;
      x[0][u] = ld(a, v);
      x[1][u] = ld(b, v);
      x[2][u] = ld(c, v);
    }
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int u = 0; u < U; ++u) acc += x[s][u];
  }
  if (acc.x == 123.456f) st(sink, threadIdx.x, acc);  // never true: keeps the loads live
}

// default-policy (allocating) loads and stores over 1 GiB: evicts the Infinity Cache
__global__ void __launch_bounds__(T) flush_k(float* p) {
  const long b = long(blockIdx.x) * (U * T);
  f4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = *((const G f4*)(p) + b + u * T + threadIdx.x);
#pragma unroll
  for (int u = 0; u < U; ++u) *((G f4*)(p) + b + u * T + threadIdx.x) = x[u] + 1.0f;
}

__global__ void fill(float* p, long n, unsigned seed) {
  for (long i = blockIdx.x * long(T) + threadIdx.x; i < n; i += long(gridDim.x) * T) {
    unsigned z = unsigned(i) * 2654435761u + seed;
    z ^= z >> 15;
    p[i] = float(int(z & 0xFFFFF) - 0x80000) * 1e-6f;
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 11;
  const bool big = argc > 2 && std::string(argv[2]) == "t1.3b";
  const long n = big ? 1313722368L / 4096 * 4096 : 124473344L;  // whole 4096-element tiles
  const long ntiles = n / (U * T * 4);
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
  float *th = buf[0], *in = buf[1], *mb = buf[2], *w = buf[3], *x = buf[4], *y = buf[5], *z = buf[6];
  int dev = 0, lds_cu = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  int lds_max = 0;
  CK(hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
  printf("LDS per CU %d B, per workgroup max %d B, %d CUs\n", lds_cu, lds_max, cus);

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
  // LDS bytes per workgroup that leave room for k workgroups per CU (0 = none reserved)
  auto lds_for = [&](int k) -> size_t {
    if (k == 0) return 0;
    size_t b = size_t(lds_cu) / k - 1024;
    return std::min(b, size_t(lds_max)) / 256 * 256;
  };
  auto occ = [&](auto kern, size_t lds) {
    int per = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, T, lds));
    return per;
  };
#define VARIANT(KIND, M, K, BYTES, LAUNCH)                                                  \
  {                                                                                         \
    const size_t L = lds_for(K);                                                            \
    if (L > 0) CK(hipFuncSetAttribute((const void*)KIND<M>,                                  \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, int(L))); \
    const int per = occ(KIND<M>, L);                                                        \
    char nm[96];                                                                            \
    snprintf(nm, sizeof nm, "%-7s M=%d  %d WG/CU%s", #KIND, M, per, K ? "" : " (no LDS)");  \
    const unsigned g = unsigned((ntiles + M - 1) / M);                                      \
    vs.push_back({nm, double(BYTES) * n, [=]() { LAUNCH; }, {}});                           \
  }
#define FUSED(M, K) VARIANT(fused, M, K, 28, hipLaunchKernelGGL(fused<M>, dim3(g), dim3(T), L, 0, th, in, mb, w, ntiles))
#define WRITE(M, K) VARIANT(write4, M, K, 16, hipLaunchKernelGGL(write4<M>, dim3(g), dim3(T), L, 0, x, y, z, w, ntiles))
#define READ(M, K) VARIANT(read3, M, K, 12, hipLaunchKernelGGL(read3<M>, dim3(g), dim3(T), L, 0, th, in, mb, sink, ntiles))
  FUSED(1, 0) FUSED(1, 6) FUSED(1, 4) FUSED(1, 3) FUSED(1, 2) FUSED(1, 1)
  FUSED(2, 0) FUSED(4, 0) FUSED(8, 0) FUSED(4, 4) FUSED(8, 2)
  WRITE(1, 0) WRITE(1, 4) WRITE(1, 2) WRITE(1, 1) WRITE(4, 0) WRITE(8, 2)
  READ(1, 0) READ(1, 4) READ(1, 2) READ(1, 1) READ(4, 0)
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
  printf("%s-size arrays (n=%ld fp32, %ld tiles), %d rounds, Infinity Cache evicted before each launch\n",
         big ? "T1.3B" : "T125", n, ntiles, rounds);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("%-32s med %8.4f ms %7.1f GB/s  best %7.1f GB/s\n", v.name.c_str(), med,
           v.bytes / med / 1e6, v.bytes / v.ms[0] / 1e6);
  }
  return 0;
}
