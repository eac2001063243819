// Does the end of a walker launch (the last round of chunks draining while fewer and fewer
// workgroups keep HBM busy) cost measurable time, and do smaller chunks at the end recover it?
// The fused one-replica shape (read θ, in, m; write w, θ, m, in; all non-temporal) over T125's
// element count, the last `tail` chunk-equivalents cut into 1024-element pieces. Warm (back to
// back) and cold (a 1 GiB default-policy copy before each launch), interleaved round by round.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tail_split.hip -o build/tail_split
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

__device__ __forceinline__ f4 ld(const float* p, long v) {
  return __builtin_nontemporal_load((const G f4*)(p) + v);
}
__device__ __forceinline__ void st(float* p, long v, f4 x) {
  __builtin_nontemporal_store(x, (G f4*)(p) + v);
}

// workgroups [0, nbig) take 4096-element chunks, the rest 1024-element pieces after them
__global__ void __launch_bounds__(T) fused(float* th, float* in, float* mb, float* w, long nbig) {
  const long b = blockIdx.x;
  const long base4 = b < nbig ? b * 1024 : nbig * 1024 + (b - nbig) * 256;  // in float4
  const int n4 = b < nbig ? 1024 : 256;
  f4 t[4], x[4], m[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = u * T + threadIdx.x;
    if (v < n4) {
      t[u] = ld(th, base4 + v);
      x[u] = ld(in, base4 + v);
      m[u] = ld(mb, base4 + v);
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    x[u] = t[u] - x[u];
    m[u] = m[u] * 0.9f + x[u];
    t[u] = t[u] - 0.7f * (x[u] + 0.9f * m[u]);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = u * T + threadIdx.x;
    if (v < n4) st(w, base4 + v, x[u]);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = u * T + threadIdx.x;
    if (v < n4) st(th, base4 + v, t[u]);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = u * T + threadIdx.x;
    if (v < n4) st(mb, base4 + v, m[u]);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = u * T + threadIdx.x;
    if (v < n4) st(in, base4 + v, t[u]);
  }
}

__global__ void __launch_bounds__(T) flush_k(float* p) {
  const long b = long(blockIdx.x) * 1024;
  f4 x[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) x[u] = *((const G f4*)(p) + b + u * T + threadIdx.x);
#pragma unroll
  for (int u = 0; u < 4; ++u) *((G f4*)(p) + b + u * T + threadIdx.x) = x[u] + 1.0f;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 15;
  const long nch = 30389;  // T125 in whole 4096-element chunks
  const long n = nch * 4096;
  float *th, *in, *mb, *w, *fl;
  for (float** p : {&th, &in, &mb, &w}) {
    CK(hipMalloc(p, n * 4));
    CK(hipMemset(*p, 0, n * 4));
  }
  const long nf = 1L << 28;
  CK(hipMalloc(&fl, nf * 4));
  CK(hipMemset(fl, 0, nf * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const long tails[] = {0, 896, 1792, 3584, 7168};  // chunk-equivalents cut into quarters
  std::vector<std::vector<float>> cold(5), warm(5);
  for (int r = 0; r < rounds; ++r)
    for (int k = 0; k < 5; ++k) {
      const long nbig = nch - tails[k];
      const unsigned grid = unsigned(nbig + 4 * tails[k]);
      for (int c = 0; c < 2; ++c) {
        if (c == 0) hipLaunchKernelGGL(flush_k, dim3(unsigned(nf / 4096)), dim3(T), 0, 0, fl);
        else hipLaunchKernelGGL(fused, dim3(grid), dim3(T), 0, 0, th, in, mb, w, nbig);  // warm-up
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(fused, dim3(grid), dim3(T), 0, 0, th, in, mb, w, nbig);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        (c == 0 ? cold : warm)[k].push_back(ms);
      }
    }
  CK(hipGetLastError());
  printf("fused shape over %ld elements (T125), %d rounds; tail = chunk-equivalents cut into 1024-element pieces\n", n, rounds);
  for (int k = 0; k < 5; ++k) {
    for (auto* v : {&cold[k], &warm[k]}) std::sort(v->begin(), v->end());
    const float mc = cold[k][rounds / 2], mw = warm[k][rounds / 2];
    printf("tail %5ld  cold %.4f ms %7.1f GB/s   warm %.4f ms %7.1f GB/s\n", tails[k], mc,
           28.0 * n / mc / 1e6, mw, 28.0 * n / mw / 1e6);
  }
  return 0;
}
