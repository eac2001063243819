// Micro-benchmark of streaming access patterns for the outer-step kernels on gfx950.
// Flat buffers of N fp32 (default: the T125 tree, 124,475,904 elements). Interleaved rounds
// in one process (cdna_hip_programming.md §5.4 rule 24); prints median/min GB/s per variant.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/hbm_bench.hip -o build/hbm_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));         \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

template <bool NT>
__device__ __forceinline__ float4 ld(const float4* p) {
  if constexpr (NT) {
    float4 r;
    r.x = __builtin_nontemporal_load(&reinterpret_cast<const float*>(p)[0]);
    r.y = __builtin_nontemporal_load(&reinterpret_cast<const float*>(p)[1]);
    r.z = __builtin_nontemporal_load(&reinterpret_cast<const float*>(p)[2]);
    r.w = __builtin_nontemporal_load(&reinterpret_cast<const float*>(p)[3]);
    return r;
  } else {
    return *p;
  }
}
template <bool NT>
__device__ __forceinline__ void st(float4* p, float4 v) {
  if constexpr (NT) {
    __builtin_nontemporal_store(v.x, &reinterpret_cast<float*>(p)[0]);
    __builtin_nontemporal_store(v.y, &reinterpret_cast<float*>(p)[1]);
    __builtin_nontemporal_store(v.z, &reinterpret_cast<float*>(p)[2]);
    __builtin_nontemporal_store(v.w, &reinterpret_cast<float*>(p)[3]);
  } else {
    *p = v;
  }
}

// chunked walker: block takes chunks of U*256 float4 round-robin
template <int U, bool NTL, bool NTS, int OP>
__global__ void __launch_bounds__(256) k_chunk(const float4* __restrict__ a, const float4* __restrict__ b,
                                               const float4* __restrict__ c, float4* __restrict__ x,
                                               float4* __restrict__ y, float4* __restrict__ z, long nv) {
  const long chunk = long(U) * 256;
  const long nch = (nv + chunk - 1) / chunk;
  for (long ci = blockIdx.x; ci < nch; ci += gridDim.x) {
    const long base = ci * chunk + threadIdx.x;
    float4 ra[U], rb[U], rc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long v = base + long(u) * 256;
      if (v < nv) {
        ra[u] = ld<NTL>(a + v);
        if (OP >= 1) rb[u] = ld<NTL>(b + v);
        if (OP >= 2) rc[u] = ld<NTL>(c + v);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long v = base + long(u) * 256;
      if (v < nv) {
        if (OP == 0) {
          st<NTS>(x + v, ra[u]);
        } else if (OP == 1) {
          st<NTS>(x + v, make_float4(ra[u].x - rb[u].x, ra[u].y - rb[u].y, ra[u].z - rb[u].z,
                                     ra[u].w - rb[u].w));
        } else {
          float4 g = ra[u], t = rb[u], m = rc[u];
          m.x = m.x * 0.9f + g.x; m.y = m.y * 0.9f + g.y; m.z = m.z * 0.9f + g.z; m.w = m.w * 0.9f + g.w;
          t.x = __builtin_fmaf(__builtin_fmaf(m.x, 0.9f, g.x), -0.7f, t.x);
          t.y = __builtin_fmaf(__builtin_fmaf(m.y, 0.9f, g.y), -0.7f, t.y);
          t.z = __builtin_fmaf(__builtin_fmaf(m.z, 0.9f, g.z), -0.7f, t.z);
          t.w = __builtin_fmaf(__builtin_fmaf(m.w, 0.9f, g.w), -0.7f, t.w);
          st<NTS>(x + v, t);
          st<NTS>(y + v, m);
          st<NTS>(z + v, t);
        }
      }
    }
  }
}

// contiguous range per block (persistent style)
template <int U, bool NT, int OP>
__global__ void __launch_bounds__(256) k_range(const float4* __restrict__ a, const float4* __restrict__ b,
                                               const float4* __restrict__ c, float4* __restrict__ x,
                                               float4* __restrict__ y, float4* __restrict__ z, long nv) {
  const long chunk = long(U) * 256;
  const long nch = (nv + chunk - 1) / chunk;
  const long per = (nch + gridDim.x - 1) / gridDim.x;
  const long c0 = blockIdx.x * per, c1 = std::min(nch, c0 + per);
  for (long ci = c0; ci < c1; ++ci) {
    const long base = ci * chunk + threadIdx.x;
    float4 ra[U], rb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long v = base + long(u) * 256;
      if (v < nv) {
        ra[u] = ld<NT>(a + v);
        if (OP >= 1) rb[u] = ld<NT>(b + v);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long v = base + long(u) * 256;
      if (v < nv) {
        if (OP == 0) st<NT>(x + v, ra[u]);
        else st<NT>(x + v, make_float4(ra[u].x - rb[u].x, ra[u].y - rb[u].y, ra[u].z - rb[u].z,
                                       ra[u].w - rb[u].w));
      }
    }
  }
}


struct Chunk { long poff; long loff; int seg; int len; long pad; };

// table-driven: one block per chunk entry, pointer table for the per-tensor operand (b)
template <int U, bool NTL, bool NTS, int OP>
__global__ void __launch_bounds__(256) k_table(const Chunk* __restrict__ ch, int nch, const float* const* __restrict__ ptab,
                                               const float4* __restrict__ a, const float4* __restrict__ c,
                                               float4* __restrict__ x, float4* __restrict__ y, float4* __restrict__ z) {
  for (int ci = blockIdx.x; ci < nch; ci += gridDim.x) {
    const Chunk k = ch[ci];
    const float4* b = reinterpret_cast<const float4*>(ptab[k.seg] + k.loff);
    const long pv = k.poff >> 2;
    const int nv = k.len >> 2;
    float4 ra[U], rb[U], rc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = u * 256 + threadIdx.x;
      if (v < nv) {
        ra[u] = ld<NTL>(a + pv + v);
        if (OP >= 1) rb[u] = ld<NTL>(b + v);
        if (OP >= 2) rc[u] = ld<NTL>(c + pv + v);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = u * 256 + threadIdx.x;
      if (v < nv) {
        if (OP == 1) {
          st<NTS>(x + pv + v, make_float4(ra[u].x - rb[u].x, ra[u].y - rb[u].y, ra[u].z - rb[u].z, ra[u].w - rb[u].w));
        } else {
          float4 g = ra[u], t = rb[u], m = rc[u];
          m.x = m.x * 0.9f + g.x; m.y = m.y * 0.9f + g.y; m.z = m.z * 0.9f + g.z; m.w = m.w * 0.9f + g.w;
          t.x = __builtin_fmaf(__builtin_fmaf(m.x, 0.9f, g.x), -0.7f, t.x);
          t.y = __builtin_fmaf(__builtin_fmaf(m.y, 0.9f, g.y), -0.7f, t.y);
          t.z = __builtin_fmaf(__builtin_fmaf(m.z, 0.9f, g.z), -0.7f, t.z);
          t.w = __builtin_fmaf(__builtin_fmaf(m.w, 0.9f, g.w), -0.7f, t.w);
          st<NTS>(x + pv + v, t);
          st<NTS>(y + pv + v, m);
          st<NTS>(reinterpret_cast<float4*>(const_cast<float4*>(b)) + v, t);
        }
      }
    }
  }
}

Chunk* g_ch[5]; int g_nch[5]; const float** g_ptab;
template <int U, bool NTL, bool NTS, int OP>
void L_table(int grid, float4** p, long nv, hipStream_t s) {
  int ti = U == 1 ? 0 : U == 2 ? 1 : U == 4 ? 2 : 3;
  int g = grid > 0 ? grid : g_nch[ti];
  hipLaunchKernelGGL((k_table<U, NTL, NTS, OP>), dim3(g), dim3(256), 0, s, g_ch[ti], g_nch[ti], g_ptab,
                     p[0], p[2], p[3], p[4], p[5]);
}

struct Var {
  std::string name;
  int op;  // 0 copy (8B), 1 delta (12B), 2 sgd (24B)
  int grid;
  void (*launch)(int grid, float4**, long, hipStream_t);
  std::vector<float> ms;
};

template <int U, bool NTL, bool NTS, int OP>
void L_chunk(int grid, float4** p, long nv, hipStream_t s) {
  hipLaunchKernelGGL((k_chunk<U, NTL, NTS, OP>), dim3(grid), dim3(256), 0, s, p[0], p[1], p[2], p[3], p[4], p[5], nv);
}
template <int U, bool NT, int OP>
void L_range(int grid, float4** p, long nv, hipStream_t s) {
  hipLaunchKernelGGL((k_range<U, NT, OP>), dim3(grid), dim3(256), 0, s, p[0], p[1], p[2], p[3], p[4], p[5], nv);
}

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 124475904L;
  int rounds = argc > 2 ? atoi(argv[2]) : 15;
  long nv = n / 4;
  float4* p[6];
  for (int i = 0; i < 6; ++i) {
    CK(hipMalloc(&p[i], nv * 16));
    CK(hipMemset(p[i], 0x3c + i, nv * 16));
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<Var> vs;
  // T125-shaped chunk tables: segments = the 148 tensors (per-tensor operand b via ptab)
  {
    std::vector<long> numel;
    const long V = 50304, C = 768, B = 1024;
    numel.push_back(V * C); numel.push_back(B * C);
    for (int l = 0; l < 12; ++l) {
      long blk[12] = {C, C, 3 * C * C, 3 * C, C * C, C, C, C, 4 * C * C, 4 * C, 4 * C * C, C};
      for (long x : blk) numel.push_back(x);
    }
    numel.push_back(C); numel.push_back(C);
    std::vector<long> off(numel.size() + 1, 0);
    for (size_t i = 0; i < numel.size(); ++i) off[i + 1] = (off[i] + numel[i] + 63) / 64 * 64;
    if (off.back() > n) { fprintf(stderr, "n too small\n"); return 1; }
    std::vector<const float*> ptab(numel.size());
    for (size_t i = 0; i < numel.size(); ++i) ptab[i] = reinterpret_cast<float*>(p[1]) + off[i];
    CK(hipMalloc(&g_ptab, ptab.size() * sizeof(void*)));
    CK(hipMemcpy(g_ptab, ptab.data(), ptab.size() * sizeof(void*), hipMemcpyHostToDevice));
    int us[4] = {1, 2, 4, 8};
    for (int ti = 0; ti < 4; ++ti) {
      long CH = 1024L * us[ti];
      std::vector<Chunk> v;
      for (size_t i = 0; i < numel.size(); ++i)
        for (long o = 0; o < numel[i]; o += CH) v.push_back({off[i] + o, o, int(i), int(std::min(CH, numel[i] - o)), 0});
      CK(hipMalloc(&g_ch[ti], v.size() * sizeof(Chunk)));
      CK(hipMemcpy(g_ch[ti], v.data(), v.size() * sizeof(Chunk), hipMemcpyHostToDevice));
      g_nch[ti] = int(v.size());
    }
  }
  long g1 = (nv + 1023) / 1024, g2 = (nv + 511) / 512, g4 = (nv + 255) / 256;
  vs.push_back({"copy   U4 ntL  1blk", 0, int(g1), L_chunk<4, true, false, 0>, {}});
  vs.push_back({"copy   U2 ntL  1blk", 0, int(g2), L_chunk<2, true, false, 0>, {}});
  vs.push_back({"copy   U1 ntL  1blk", 0, int(g4), L_chunk<1, true, false, 0>, {}});
  vs.push_back({"delta  U1 ntL  1blk", 1, int(g4), L_chunk<1, true, false, 1>, {}});
  vs.push_back({"delta  U2 ntL  1blk", 1, int(g2), L_chunk<2, true, false, 1>, {}});
  vs.push_back({"delta  U2 ntLS 1blk", 1, int(g2), L_chunk<2, true, true, 1>, {}});
  vs.push_back({"delta  U4 ntL  1blk", 1, int(g1), L_chunk<4, true, false, 1>, {}});
  vs.push_back({"delta  U2 plain 1blk", 1, int(g2), L_chunk<2, false, false, 1>, {}});
  vs.push_back({"delta  TBL U1 ntL", 1, 0, L_table<1, true, false, 1>, {}});
  vs.push_back({"delta  TBL U2 ntL", 1, 0, L_table<2, true, false, 1>, {}});
  vs.push_back({"delta  TBL U2 ntLS", 1, 0, L_table<2, true, true, 1>, {}});
  vs.push_back({"delta  TBL U4 ntL", 1, 0, L_table<4, true, false, 1>, {}});
  vs.push_back({"delta  TBL U2 ntL g4096", 1, 4096, L_table<2, true, false, 1>, {}});
  vs.push_back({"sgd    U1 ntLS 1blk", 2, int(g4), L_chunk<1, true, true, 2>, {}});
  vs.push_back({"sgd    U2 ntLS 1blk", 2, int(g2), L_chunk<2, true, true, 2>, {}});
  vs.push_back({"sgd    U2 ntL  1blk", 2, int(g2), L_chunk<2, true, false, 2>, {}});
  vs.push_back({"sgd    U4 ntLS 1blk", 2, int(g1), L_chunk<4, true, true, 2>, {}});
  vs.push_back({"sgd    TBL U1 ntLS", 2, 0, L_table<1, true, true, 2>, {}});
  vs.push_back({"sgd    TBL U2 ntLS", 2, 0, L_table<2, true, true, 2>, {}});
  vs.push_back({"sgd    TBL U2 ntL", 2, 0, L_table<2, true, false, 2>, {}});
  vs.push_back({"sgd    TBL U4 ntLS", 2, 0, L_table<4, true, true, 2>, {}});
  vs.push_back({"sgd    TBL U2 ntLS g4096", 2, 4096, L_table<2, true, true, 2>, {}});
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs) v.launch(v.grid, p, nv, s);  // warm
  CK(hipStreamSynchronize(s));
  for (int r = 0; r < rounds; ++r) {
    for (auto& v : vs) {
      CK(hipEventRecord(e0, s));
      v.launch(v.grid, p, nv, s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
  }
  const double bpe[3] = {8, 12, 24};
  printf("n=%ld rounds=%d cus=%d\n", n, rounds, cus);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    double med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    double bytes = bpe[v.op] * n;
    printf("%-32s med %8.4f ms  %7.1f GB/s   best %7.1f GB/s\n", v.name.c_str(), med,
           bytes / med / 1e6, bytes / mn / 1e6);
  }
  return 0;
}
