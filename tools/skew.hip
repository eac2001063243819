// Does the relative placement of the streams' base addresses matter? The fused one-replica
// step's shape (read θ, in, m; write w, θ, m, in: 28 B/elem, one 4096-element chunk per
// workgroup, the product's NT policy) and the 2-stream copy, on T125-size arrays carved out of
// ONE allocation at offsets k * (512 MiB + skew) for stream k (skew 0: every base congruent
// modulo 512 MiB, as large power-of-two-aligned allocations are), cold (1 GiB default-policy
// flush before every launch), skews interleaved round by round in one process.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/skew.hip -o build/skew
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t err_ = (x);                                                         \
    if (err_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(err_));  \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
#define G __attribute__((address_space(1)))
constexpr int T = 256;
constexpr long CH = 4096;

__device__ __forceinline__ f4 ld(const float* p, long v) {
  return __builtin_nontemporal_load((const G f4*)(p) + v);
}
__device__ __forceinline__ void st(float* p, long v, f4 x) {
  __builtin_nontemporal_store(x, (G f4*)(p) + v);
}

__global__ void __launch_bounds__(T) dps(float* in, float* th, float* mb, float* w) {
  const long poff = long(blockIdx.x) * CH;
  float *tp = th + poff, *mp = mb + poff, *wp = w + poff, *ip = in + poff;
  f4 x[4], t[4], m[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = u * T + threadIdx.x;
    t[u] = ld(tp, v);
    x[u] = ld(ip, v);
    m[u] = ld(mp, v);
  }
  f4 g[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    g[u] = t[u] - x[u];
    m[u] = m[u] * 0.9f + g[u];
    const f4 uu = {__builtin_fmaf(m[u].x, 0.9f, g[u].x), __builtin_fmaf(m[u].y, 0.9f, g[u].y),
                   __builtin_fmaf(m[u].z, 0.9f, g[u].z), __builtin_fmaf(m[u].w, 0.9f, g[u].w)};
    t[u] = f4{__builtin_fmaf(uu.x, -0.7f, t[u].x), __builtin_fmaf(uu.y, -0.7f, t[u].y),
              __builtin_fmaf(uu.z, -0.7f, t[u].z), __builtin_fmaf(uu.w, -0.7f, t[u].w)};
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) st(wp, u * T + threadIdx.x, g[u]);
#pragma unroll
  for (int u = 0; u < 4; ++u) st(tp, u * T + threadIdx.x, t[u]);
#pragma unroll
  for (int u = 0; u < 4; ++u) st(mp, u * T + threadIdx.x, m[u]);
#pragma unroll
  for (int u = 0; u < 4; ++u) st(ip, u * T + threadIdx.x, t[u]);
}

__global__ void __launch_bounds__(T) copy(const float* a, float* b) {
  const long base = long(blockIdx.x) * (CH / 4);
  f4 x[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) x[u] = ld(a, base + u * T + threadIdx.x);
#pragma unroll
  for (int u = 0; u < 4; ++u) st(b, base + u * T + threadIdx.x, x[u]);
}

__global__ void __launch_bounds__(T) flush_k(float* p, long n4) {
  for (long v = blockIdx.x * long(T) + threadIdx.x; v < n4; v += long(gridDim.x) * T) {
    f4 x = ((G f4*)p)[v];
    ((G f4*)p)[v] = x + 1.0f;
  }
}

__global__ void fill(float* p, long n) {
  for (long i = blockIdx.x * long(T) + threadIdx.x; i < n; i += long(gridDim.x) * T)
    p[i] = float(int(unsigned(i) * 2654435761u & 0xFFFFF) - 0x80000) * 1e-9f;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 9;
  const long nch = 30390;  // T125: 124,477,440 elements
  const long n = nch * CH;
  const long skews[] = {0, 64, 256, 1024, 4096, 16384, 65536, 262144, 1 << 20, 3 << 19};
  const int ns = sizeof(skews) / sizeof(skews[0]);
  const long maxskew = 2L << 20;  // elements
  const long S = 128L << 20;      // elements: 512 MiB >= one stream
  float* pool;
  CK(hipMalloc(&pool, 4 * (4 * (S + maxskew))));  // 4 streams
  hipLaunchKernelGGL(fill, dim3(8192), dim3(T), 0, 0, pool, 4 * (S + maxskew));
  float* flush;
  const long nf = 1L << 28;
  CK(hipMalloc(&flush, nf * 4));
  CK(hipMemset(flush, 0, nf * 4));
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
  for (int k = 0; k < ns; ++k) {
    const long sk = skews[k];  // elements added to each stream's 512-MiB-aligned base
    float* s0 = pool;
    float* s1 = s0 + S + sk;
    float* s2 = s1 + S + sk;
    float* s3 = s2 + S + sk;
    char nm[64];
    snprintf(nm, sizeof nm, "fused 28 B, skew %8ld B", sk * 4);
    vs.push_back({nm, 28.0 * n, [=]() { hipLaunchKernelGGL(dps, dim3(nch), dim3(T), 0, 0, s0, s1, s2, s3); }, {}});
    snprintf(nm, sizeof nm, "copy   8 B, skew %8ld B", sk * 4);
    vs.push_back({nm, 8.0 * n, [=]() { hipLaunchKernelGGL(copy, dim3(nch), dim3(T), 0, 0, s0, s1); }, {}});
  }
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
  printf("stream base skew, T125 size (%ld elements per stream), %d rounds, cold\n", n, rounds);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("%s med %8.4f ms %7.1f GB/s  best %7.1f GB/s\n", v.name.c_str(), med,
           v.bytes / med / 1e6, v.bytes / v.ms[0] / 1e6);
  }
  return 0;
}
