// Does the number of concurrent HBM streams limit the 3-read/3-write SGD kernels?
// Flat arrays of N fp32 (T125 size), one 256-lane workgroup per 4096-element chunk, NT loads
// and stores, the SGD arithmetic of dl_unpack_sgd. Variants with the same bytes per element:
//   sgd6   read w, θ, m           write θ, m, inner          6 streams, 24 B/elem
//   sgd4i  read w, [θ|m]          write [θ|m], inner         4 streams, 24 B/elem: θ and m of a
//          chunk interleaved as two consecutive 16-KiB blocks (one read and one write stream)
//   sgd5   read w, θ, m           write θ, m                 5 streams, 20 B/elem
//   copy2  read a                 write b                    2 streams,  8 B/elem
// Interleaved rounds in one process; median GB/s per variant.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/stream_bench.hip -o build/stream_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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
constexpr int T = 256, U = 4, CH = T * U * 4;

__device__ __forceinline__ f4 ld(const float* p, long v) {
  return __builtin_nontemporal_load((const G f4*)(p) + v);
}
__device__ __forceinline__ void st(float* p, long v, f4 x) {
  __builtin_nontemporal_store(x, (G f4*)(p) + v);
}
__device__ __forceinline__ void sgd4(f4 g, f4& b, f4& t) {
  b = b * 0.9f + g;
  const f4 u = {__builtin_fmaf(b.x, 0.9f, g.x), __builtin_fmaf(b.y, 0.9f, g.y),
                __builtin_fmaf(b.z, 0.9f, g.z), __builtin_fmaf(b.w, 0.9f, g.w)};
  t = f4{__builtin_fmaf(u.x, -0.7f, t.x), __builtin_fmaf(u.y, -0.7f, t.y),
         __builtin_fmaf(u.z, -0.7f, t.z), __builtin_fmaf(u.w, -0.7f, t.w)};
}

__global__ void __launch_bounds__(T) sgd6(const float* w, float* th, float* mb, float* in) {
  const long base = long(blockIdx.x) * (CH / 4);
  f4 g[U], t[U], m[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long v = base + u * T + threadIdx.x;
    g[u] = ld(w, v);
    t[u] = ld(th, v);
    m[u] = ld(mb, v);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long v = base + u * T + threadIdx.x;
    sgd4(g[u], m[u], t[u]);
    st(th, v, t[u]);
    st(mb, v, m[u]);
    st(in, v, t[u]);
  }
}

// tm: chunk c holds θ at [2c*CH, 2c*CH + CH) and m at [(2c+1)*CH, (2c+2)*CH)
__global__ void __launch_bounds__(T) sgd4i(const float* w, float* tm, float* in) {
  const long base = long(blockIdx.x) * (CH / 4);
  const long tb = long(blockIdx.x) * 2 * (CH / 4), mbase = tb + CH / 4;
  f4 g[U], t[U], m[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long v = u * T + threadIdx.x;
    g[u] = ld(w, base + v);
    t[u] = ld(tm, tb + v);
    m[u] = ld(tm, mbase + v);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long v = u * T + threadIdx.x;
    sgd4(g[u], m[u], t[u]);
    st(tm, tb + v, t[u]);
    st(tm, mbase + v, m[u]);
    st(in, base + v, t[u]);
  }
}

__global__ void __launch_bounds__(T) sgd5(const float* w, float* th, float* mb) {
  const long base = long(blockIdx.x) * (CH / 4);
  f4 g[U], t[U], m[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long v = base + u * T + threadIdx.x;
    g[u] = ld(w, v);
    t[u] = ld(th, v);
    m[u] = ld(mb, v);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long v = base + u * T + threadIdx.x;
    sgd4(g[u], m[u], t[u]);
    st(th, v, t[u]);
    st(mb, v, m[u]);
  }
}

// the product's walker shape: a 16-B chunk descriptor + a pre-resolved inner address per
// workgroup, loads predicated on the chunk length (here every chunk is full)
struct Chunk {
  long poff;
  int len;
  int seg;
};

__global__ void __launch_bounds__(T) sgd6w(const Chunk* __restrict__ ch, void* const* __restrict__ ca,
                                           const float* w, float* th, float* mb) {
  const Chunk ck = ch[blockIdx.x];
  float* in = (float*)ca[blockIdx.x];
  const int nv = ck.len >> 2;
  const float* wp = w + ck.poff;
  float* tp = th + ck.poff;
  float* mp = mb + ck.poff;
  f4 g[U], t[U], m[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int v = u * T + threadIdx.x;
    if (v < nv) {
      g[u] = ld(wp, v);
      t[u] = ld(tp, v);
      m[u] = ld(mp, v);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int v = u * T + threadIdx.x;
    if (v < nv) {
      sgd4(g[u], m[u], t[u]);
      st(tp, v, t[u]);
      st(mp, v, m[u]);
      st(in, v, t[u]);
    }
  }
}

__global__ void __launch_bounds__(T) copy2(const float* a, float* b) {
  const long base = long(blockIdx.x) * (CH / 4);
  f4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = ld(a, base + u * T + threadIdx.x);
#pragma unroll
  for (int u = 0; u < U; ++u) st(b, base + u * T + threadIdx.x, x[u]);
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 20;
  const long nch = 30400;  // ~T125: 124.5 M elements
  const long n = nch * CH;
  float *w, *th, *mb, *in, *tm, *a, *b, *flush;
  CK(hipMalloc(&w, n * 4));
  CK(hipMalloc(&th, n * 4));
  CK(hipMalloc(&mb, n * 4));
  CK(hipMalloc(&in, n * 4));
  CK(hipMalloc(&tm, 2 * n * 4));
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  const long nf = 1L << 28;  // 1 GiB to evict the 256 MiB Infinity Cache between launches
  CK(hipMalloc(&flush, nf * 4));
  for (float* p : {w, th, mb, in, a, b}) CK(hipMemset(p, 0, n * 4));
  CK(hipMemset(tm, 0, 2 * n * 4));
  CK(hipMemset(flush, 0, nf * 4));
  std::vector<Chunk> hc(nch);
  std::vector<void*> hca(nch);
  for (long c = 0; c < nch; ++c) {
    hc[c] = Chunk{c * CH, CH, int(c / 200)};
    hca[c] = in + c * CH;
  }
  Chunk* dch;
  void** dca;
  CK(hipMalloc(&dch, nch * sizeof(Chunk)));
  CK(hipMalloc(&dca, nch * sizeof(void*)));
  CK(hipMemcpy(dch, hc.data(), nch * sizeof(Chunk), hipMemcpyHostToDevice));
  CK(hipMemcpy(dca, hca.data(), nch * sizeof(void*), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V {
    std::string name;
    double bytes;
    std::vector<float> ms;
  };
  std::vector<V> vs = {{"sgd6  (6 streams, 24 B)", 24.0 * n, {}},
                       {"sgd4i (4 streams, 24 B)", 24.0 * n, {}},
                       {"sgd5  (5 streams, 20 B)", 20.0 * n, {}},
                       {"copy2 (2 streams,  8 B)", 8.0 * n, {}},
                       {"sgd6w (walker, 24 B)   ", 24.0 * n, {}}};
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      hipLaunchKernelGGL(copy2, dim3(unsigned(nf / CH)), dim3(T), 0, 0, flush, flush);  // evict
      CK(hipEventRecord(e0, 0));
      if (i == 0) hipLaunchKernelGGL(sgd6, dim3(nch), dim3(T), 0, 0, w, th, mb, in);
      if (i == 1) hipLaunchKernelGGL(sgd4i, dim3(nch), dim3(T), 0, 0, w, tm, in);
      if (i == 2) hipLaunchKernelGGL(sgd5, dim3(nch), dim3(T), 0, 0, w, th, mb);
      if (i == 3) hipLaunchKernelGGL(copy2, dim3(nch), dim3(T), 0, 0, a, b);
      if (i == 4) hipLaunchKernelGGL(sgd6w, dim3(nch), dim3(T), 0, 0, dch, dca, w, th, mb);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      vs[i].ms.push_back(ms);
    }
  }
  printf("flat arrays n=%ld, rounds=%d, cache flushed before each launch\n", n, rounds);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("%s  med %8.4f ms  %7.1f GB/s   best %7.1f GB/s\n", v.name.c_str(), med,
           v.bytes / med / 1e6, v.bytes / v.ms[0] / 1e6);
  }
  return 0;
}
