// Launch-shape study for the segment walker on the T125 layout (gfx950).
// Table-driven like the product: 16-B chunk descriptors + pre-resolved per-chunk addresses.
// OP 1 = delta (2R1W, 12 B/elem), OP 2 = sgd (3R3W, 24 B/elem), OP 3 = fused delta+sgd (3R3W).
// Interleaved rounds in one process; prints median GB/s per variant.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/hbm_bench2.hip -o build/hbm_bench2
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

template <bool NT>
__device__ __forceinline__ f4 ld(const float* p, int v) {
  const G f4* q = (const G f4*)(p) + v;
  if constexpr (NT) return __builtin_nontemporal_load(q);
  else return *q;
}
template <bool NT>
__device__ __forceinline__ void st(float* p, int v, f4 x) {
  G f4* q = (G f4*)(p) + v;
  if constexpr (NT) __builtin_nontemporal_store(x, q);
  else *q = x;
}

struct Chunk {
  long poff;
  int len;
  int seg;
};

__device__ __forceinline__ void sgd4(f4 g, f4& b, f4& t) {
  b = b * 0.9f + g;
  const f4 u = {__builtin_fmaf(b.x, 0.9f, g.x), __builtin_fmaf(b.y, 0.9f, g.y),
                __builtin_fmaf(b.z, 0.9f, g.z), __builtin_fmaf(b.w, 0.9f, g.w)};
  t = f4{__builtin_fmaf(u.x, -0.7f, t.x), __builtin_fmaf(u.y, -0.7f, t.y),
         __builtin_fmaf(u.z, -0.7f, t.z), __builtin_fmaf(u.w, -0.7f, t.w)};
}

// T threads per WG, U float4 per lane per stream; chunk = T*U*4 elements
template <int T, int U, bool NTL, bool NTS, int OP>
__global__ void __launch_bounds__(T) k(const Chunk* __restrict__ ch, int nch, void* const* __restrict__ ca,
                                       float* w, float* th, float* mb) {
  for (int c = blockIdx.x; c < nch; c += gridDim.x) {
    const Chunk kk = ch[c];
    float* in = (float*)ca[c];
    const long pv = kk.poff;
    float* W = w + pv;
    float* TH = th + pv;
    float* M = mb + pv;
    const int nv = kk.len >> 2;
    f4 a[U], b[U], m[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = u * T + threadIdx.x;
      if (v < nv) {
        if (OP == 1 || OP == 4) {
          a[u] = ld<NTL>(TH, v);
          b[u] = ld<NTL>(in, v);
        } else if (OP == 5) {
          a[u] = ld<NTL>(TH, v);
        } else if (OP == 2) {
          a[u] = ld<NTL>(W, v);
          b[u] = ld<NTL>(TH, v);
          m[u] = ld<NTL>(M, v);
        } else {
          a[u] = ld<NTL>(TH, v);
          b[u] = ld<NTL>(in, v);
          m[u] = ld<NTL>(M, v);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = u * T + threadIdx.x;
      if (v < nv) {
        if (OP == 1) {
          st<NTS>(W, v, a[u] - b[u]);
        } else if (OP == 4) {
          const f4 d = a[u] - b[u];
          if (d.x == 12345.f) W[0] = d.y;  // never true: keeps the loads live
        } else if (OP == 5) {
          st<NTS>(W, v, a[u]);
        } else {
          f4 g = OP == 2 ? a[u] : a[u] - b[u];
          f4 t = OP == 2 ? b[u] : a[u];
          f4 mm = m[u];
          sgd4(g, mm, t);
          st<NTS>(TH, v, t);
          st<NTS>(M, v, mm);
          st<NTS>(in, v, t);
        }
      }
    }
  }
}

struct Tab {
  Chunk* ch;
  void** ca;
  int n;
};
std::vector<long> g_numel, g_off;
float* g_inner;

Tab make_tab(long CH) {
  std::vector<Chunk> v;
  std::vector<void*> a;
  for (size_t i = 0; i < g_numel.size(); ++i)
    for (long o = 0; o < g_numel[i]; o += CH) {
      v.push_back({g_off[i] + o, int(std::min(CH, g_numel[i] - o)), int(i)});
      a.push_back(g_inner + g_off[i] + o);
    }
  Tab t;
  CK(hipMalloc(&t.ch, v.size() * sizeof(Chunk)));
  CK(hipMemcpy(t.ch, v.data(), v.size() * sizeof(Chunk), hipMemcpyHostToDevice));
  CK(hipMalloc(&t.ca, a.size() * sizeof(void*)));
  CK(hipMemcpy(t.ca, a.data(), a.size() * sizeof(void*), hipMemcpyHostToDevice));
  t.n = int(v.size());
  return t;
}

struct Var {
  std::string name;
  int bpe;
  void (*fn)(float**, hipStream_t);
  std::vector<float> ms;
};

template <int T, int U, bool NTL, bool NTS, int OP>
void L(float** p, hipStream_t s) {
  static Tab t = make_tab(long(T) * U * 4);
  hipLaunchKernelGGL((k<T, U, NTL, NTS, OP>), dim3(t.n), dim3(T), 0, s, t.ch, t.n, t.ca, p[0], p[1], p[2]);
}

int main(int argc, char** argv) {
  int rounds = argc > 1 ? atoi(argv[1]) : 15;
  const long V = 50304, C = 768, B = 1024;
  g_numel = {V * C, B * C};
  for (int l = 0; l < 12; ++l)
    for (long x : {C, C, 3 * C * C, 3 * C, C * C, C, C, C, 4 * C * C, 4 * C, 4 * C * C, C}) g_numel.push_back(x);
  g_numel.push_back(C);
  g_numel.push_back(C);
  g_off.assign(g_numel.size() + 1, 0);
  for (size_t i = 0; i < g_numel.size(); ++i) g_off[i + 1] = (g_off[i] + g_numel[i] + 63) / 64 * 64;
  long n = g_off.back();
  float* p[3];
  for (int i = 0; i < 3; ++i) {
    CK(hipMalloc(&p[i], n * 4));
    CK(hipMemset(p[i], 0, n * 4));
  }
  CK(hipMalloc(&g_inner, n * 4));
  CK(hipMemset(g_inner, 0, n * 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::vector<Var> vs = {
      {"copy  256x4 ntL        ", 8, L<256, 4, true, false, 5>, {}},
      {"copy  256x4 ntLS       ", 8, L<256, 4, true, true, 5>, {}},
      {"copy  256x4 plain      ", 8, L<256, 4, false, false, 5>, {}},
      {"read2 256x4 ntL        ", 8, L<256, 4, true, false, 4>, {}},
      {"read2 256x4 plain      ", 8, L<256, 4, false, false, 4>, {}},
      {"delta 256x4 ntLS       ", 12, L<256, 4, true, true, 1>, {}},
      {"delta 256x4 plain      ", 12, L<256, 4, false, false, 1>, {}},
      {"delta 256x4 ntS        ", 12, L<256, 4, false, true, 1>, {}},
      {"delta 256x4 ntL        ", 12, L<256, 4, true, false, 1>, {}},
      {"delta 256x2 ntL        ", 12, L<256, 2, true, false, 1>, {}},
      {"delta 512x2 ntL        ", 12, L<512, 2, true, false, 1>, {}},
      {"delta 512x4 ntL        ", 12, L<512, 4, true, false, 1>, {}},
      {"delta 1024x1 ntL       ", 12, L<1024, 1, true, false, 1>, {}},
      {"delta 256x8 ntL        ", 12, L<256, 8, true, false, 1>, {}},
      {"sgd   256x4 ntLS       ", 24, L<256, 4, true, true, 2>, {}},
      {"sgd   256x4 ntL        ", 24, L<256, 4, true, false, 2>, {}},
      {"sgd   256x2 ntLS       ", 24, L<256, 2, true, true, 2>, {}},
      {"sgd   512x2 ntLS       ", 24, L<512, 2, true, true, 2>, {}},
      {"sgd   512x4 ntLS       ", 24, L<512, 4, true, true, 2>, {}},
      {"sgd   1024x1 ntLS      ", 24, L<1024, 1, true, true, 2>, {}},
      {"sgd   1024x2 ntLS      ", 24, L<1024, 2, true, true, 2>, {}},
      {"fused 256x4 ntLS       ", 24, L<256, 4, true, true, 3>, {}},
      {"fused 512x2 ntLS       ", 24, L<512, 2, true, true, 3>, {}},
      {"fused 1024x1 ntLS      ", 24, L<1024, 1, true, true, 3>, {}},
  };
  // cold caches for every timed launch: 1 GiB written between launches (4x the Infinity Cache)
  void* scratch;
  CK(hipMalloc(&scratch, 1l << 30));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs) v.fn(p, s);
  CK(hipStreamSynchronize(s));
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      CK(hipMemsetAsync(scratch, r & 0xff, 1l << 30, s));
      CK(hipEventRecord(e0, s));
      v.fn(p, s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
  printf("T125 layout n=%ld rounds=%d\n", n, rounds);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    double med = v.ms[v.ms.size() / 2];
    printf("%s med %8.4f ms %7.1f GB/s  best %7.1f GB/s\n", v.name.c_str(), med,
           v.bpe * 124475904.0 / med / 1e6, v.bpe * 124475904.0 / v.ms[0] / 1e6);
  }
  return 0;
}
