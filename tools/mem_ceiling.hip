// What the MI355X memory system gives streaming kernels of the outer step's shapes, cold
// (a 1 GiB default-policy read+write evicts the Infinity Cache before every launch), in one process with the
// variants interleaved round by round (median and best GB/s of algorithmic bytes).
//
//   read1<U>    read a                                   (pure read; one store per workgroup)
//   copy<U>     read a, write b                          2 streams, 8 B/elem
//   pack<U>     read θ, in; write w                      dl_delta_pack's shape, 12 B/elem
//   sgd6<U>     read w, θ, m; write θ, m, in             dl_unpack_sgd's shape, 24 B/elem
//   rmw3<U>     read θ, in, m; write θ, m, in            dl_delta_sgd's shape (3 read-modify-
//                                                         write streams), 24 B/elem
//   rmw3s<U>    rmw3 with the `in` stream's loads issued first, stores in stream order
//   rmw3p       rmw3 with plain (default-policy) stores
// U = float4 loads per lane per stream (one 256-lane workgroup covers U*1024 elements), so
// bytes in flight per lane = 16*U*streams. Grid: one workgroup per tile (the walker's shape),
// or `per` workgroups per CU looping (persistent).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/mem_ceiling.hip \
//         -o build/mem_ceiling && build/mem_ceiling [rounds]
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
__device__ __forceinline__ void sgd4(f4 g, f4& b, f4& t) {
  b = b * 0.9f + g;
  const f4 u = {__builtin_fmaf(b.x, 0.9f, g.x), __builtin_fmaf(b.y, 0.9f, g.y),
                __builtin_fmaf(b.z, 0.9f, g.z), __builtin_fmaf(b.w, 0.9f, g.w)};
  t = f4{__builtin_fmaf(u.x, -0.7f, t.x), __builtin_fmaf(u.y, -0.7f, t.y),
         __builtin_fmaf(u.z, -0.7f, t.z), __builtin_fmaf(u.w, -0.7f, t.w)};
}

// tile loop: tiles of U*T float4; grid-stride over tiles (grid == tiles: one tile per WG)
#define TILE_LOOP(U, n4)                                                              \
  for (long tile = blockIdx.x; tile * (U * T) < (n4); tile += gridDim.x)              \
    if (const long base = tile * (U * T); true)

template <int U>
__global__ void __launch_bounds__(T) read1(const float* a, float* sink, long n4) {
  f4 acc = {0, 0, 0, 0};
  TILE_LOOP(U, n4) {
    f4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = ld(a, base + u * T + threadIdx.x);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += x[u];
  }
  if (acc.x == 123.456f) st(sink, threadIdx.x, acc);  // never true: keeps the loads live
}

template <int U, bool NTS = true>
__global__ void __launch_bounds__(T) copy(const float* a, float* b, long n4) {
  TILE_LOOP(U, n4) {
    f4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = ld(a, base + u * T + threadIdx.x);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTS>(b, base + u * T + threadIdx.x, x[u]);
  }
}

template <int U>
__global__ void __launch_bounds__(T) pack(const float* th, const float* in, float* w, long n4) {
  TILE_LOOP(U, n4) {
    f4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a[u] = ld(th, base + u * T + threadIdx.x);
      b[u] = ld(in, base + u * T + threadIdx.x);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st<false>(w, base + u * T + threadIdx.x, a[u] - b[u]);
  }
}

template <int U>
__global__ void __launch_bounds__(T) sgd6(const float* w, float* th, float* mb, float* in, long n4) {
  TILE_LOOP(U, n4) {
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
}

template <int U, bool NTS = true, bool INFIRST = false>
__global__ void __launch_bounds__(T) rmw3(float* th, float* mb, float* in, long n4) {
  TILE_LOOP(U, n4) {
    f4 x[U], t[U], m[U];
    if constexpr (INFIRST) {
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = ld(in, base + u * T + threadIdx.x);
#pragma unroll
      for (int u = 0; u < U; ++u) t[u] = ld(th, base + u * T + threadIdx.x);
#pragma unroll
      for (int u = 0; u < U; ++u) m[u] = ld(mb, base + u * T + threadIdx.x);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long v = base + u * T + threadIdx.x;
        t[u] = ld(th, v);
        x[u] = ld(in, v);
        m[u] = ld(mb, v);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long v = base + u * T + threadIdx.x;
      const f4 g = t[u] - x[u];
      sgd4(g, m[u], t[u]);
      st<NTS>(th, v, t[u]);
      st<NTS>(mb, v, m[u]);
      st<NTS>(in, v, t[u]);
    }
  }
}

// ---- the product's walker shape: a 16-B chunk descriptor and a pre-resolved per-tensor
// address per chunk (dl_device.h k_walk), here with full 4096-element chunks ----
struct Chunk {
  long poff;
  int len;
  int seg;
};
constexpr int CHE = 4096;  // elements per chunk: 4 float4 per lane

template <bool NTS>
__device__ __forceinline__ void pack_chunk(const Chunk& ck, const float* in, const float* th,
                                           float* w) {
  f4 a[4], b[4];
  const float* tp = th + ck.poff;
  float* wp = w + ck.poff;
  const int nv = ck.len >> 2;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = u * T + threadIdx.x;
    if (v < nv) {
      a[u] = ld(tp, v);
      b[u] = ld(in, v);
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = u * T + threadIdx.x;
    if (v < nv) st<NTS>(wp, v, a[u] - b[u]);
  }
}

// one chunk per workgroup (dl_delta_pack today)
template <bool NTS>
__global__ void __launch_bounds__(T) pack_w(const Chunk* __restrict__ ch, void* const* __restrict__ ca,
                                            const float* th, float* w) {
  const Chunk ck = ch[blockIdx.x];
  pack_chunk<NTS>(ck, (const float*)ca[blockIdx.x], th, w);
}

// K consecutive chunks per workgroup, the next chunk's descriptor and address loaded before
// the current chunk's data (descriptor latency off the critical path)
template <int K>
__global__ void __launch_bounds__(T) pack_wk(const Chunk* __restrict__ ch, void* const* __restrict__ ca,
                                             int nch, const float* th, float* w) {
  int c = blockIdx.x * K;
  if (c >= nch) return;
  Chunk ck = ch[c];
  const float* in = (const float*)ca[c];
  for (int k = 0; k < K && c < nch; ++k, ++c) {
    Chunk nx = ck;
    const float* nin = in;
    if (k + 1 < K && c + 1 < nch) {
      nx = ch[c + 1];
      nin = (const float*)ca[c + 1];
    }
    pack_chunk<false>(ck, in, th, w);
    ck = nx;
    in = nin;
  }
}

// the walker body with the descriptor computed, not loaded (isolates the descriptor loads)
__global__ void __launch_bounds__(T) pack_c(const float* inb, const float* th, float* w) {
  Chunk ck;
  ck.poff = long(blockIdx.x) * CHE;
  ck.len = CHE;
  ck.seg = 0;
  pack_chunk<false>(ck, inb + ck.poff, th, w);
}

// one chunk per workgroup, chunk index remapped so that the workgroups of one XCD (b % 8 under
// round-robin dispatch) walk consecutive chunks: their descriptors share 64-B lines in that
// XCD's L2
__global__ void __launch_bounds__(T) pack_x(const Chunk* __restrict__ ch, void* const* __restrict__ ca,
                                            int nch, const float* th, float* w) {
  const int b = blockIdx.x, per = (nch + 7) / 8;
  const int c = (b % 8) * per + b / 8;
  if (c >= nch) return;
  const Chunk ck = ch[c];
  pack_chunk<false>(ck, (const float*)ca[c], th, w);
}

// dl_delta_sgd + the wire (the fused one-replica step that keeps outer.grad): read θ, in, m;
// write w, θ, m, in -- 28 B/elem
template <bool WALK>
__global__ void __launch_bounds__(T) dps(const Chunk* __restrict__ ch, void* const* __restrict__ ca,
                                         const float* inb, float* th, float* mb, float* w) {
  long poff;
  float* in;
  if constexpr (WALK) {
    const Chunk ck = ch[blockIdx.x];
    poff = ck.poff;
    in = (float*)ca[blockIdx.x];
  } else {
    poff = long(blockIdx.x) * CHE;
    in = (float*)inb + poff;
  }
  float* tp = th + poff;
  float* mp = mb + poff;
  float* wp = w + poff;
  f4 x[4], t[4], m[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = u * T + threadIdx.x;
    t[u] = ld(tp, v);
    x[u] = ld(in, v);
    m[u] = ld(mp, v);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = u * T + threadIdx.x;
    const f4 g = t[u] - x[u];
    st<false>(wp, v, g);
    sgd4(g, m[u], t[u]);
    st(tp, v, t[u]);
    st(mp, v, m[u]);
    st(in, v, t[u]);
  }
}

// dps with the stores grouped by stream (all wire stores, then θ, then m, then in) instead of
// by float4 row; BYSTREAM=false is dps<true>'s order
template <bool BYSTREAM, bool NTW>
__global__ void __launch_bounds__(T) dps_o(const Chunk* __restrict__ ch, void* const* __restrict__ ca,
                                           float* th, float* mb, float* w) {
  const Chunk ck = ch[blockIdx.x];
  float* in = (float*)ca[blockIdx.x];
  float* tp = th + ck.poff;
  float* mp = mb + ck.poff;
  float* wp = w + ck.poff;
  f4 x[4], t[4], m[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = u * T + threadIdx.x;
    t[u] = ld(tp, v);
    x[u] = ld(in, v);
    m[u] = ld(mp, v);
  }
  if constexpr (BYSTREAM) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f4 g = t[u] - x[u];
      x[u] = g;
      sgd4(g, m[u], t[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) st<NTW>(wp, u * T + threadIdx.x, x[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) st(tp, u * T + threadIdx.x, t[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) st(mp, u * T + threadIdx.x, m[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) st(in, u * T + threadIdx.x, t[u]);
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int v = u * T + threadIdx.x;
      const f4 g = t[u] - x[u];
      st<NTW>(wp, v, g);
      sgd4(g, m[u], t[u]);
      st(tp, v, t[u]);
      st(mp, v, m[u]);
      st(in, v, t[u]);
    }
  }
}

template <bool NTS>
__global__ void __launch_bounds__(T) rmw3_w(const Chunk* __restrict__ ch, void* const* __restrict__ ca,
                                            float* th, float* mb) {
  const Chunk ck = ch[blockIdx.x];
  float* in = (float*)ca[blockIdx.x];
  float* tp = th + ck.poff;
  float* mp = mb + ck.poff;
  const int nv = ck.len >> 2;
  f4 x[4], t[4], m[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = u * T + threadIdx.x;
    if (v < nv) {
      t[u] = ld(tp, v);
      x[u] = ld(in, v);
      m[u] = ld(mp, v);
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = u * T + threadIdx.x;
    if (v < nv) {
      const f4 g = t[u] - x[u];
      sgd4(g, m[u], t[u]);
      st<NTS>(tp, v, t[u]);
      st<NTS>(mp, v, m[u]);
      st<NTS>(in, v, t[u]);
    }
  }
}

// default-policy (allocating) loads and stores: evicts the Infinity Cache; non-temporal
// accesses may not allocate there and would leave the previous variant's lines resident
__global__ void __launch_bounds__(T) flush_k(float* p, long n4) {
  TILE_LOOP(4, n4) {
    f4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = ld<false>(p, base + u * T + threadIdx.x);
#pragma unroll
    for (int u = 0; u < 4; ++u) st<false>(p, base + u * T + threadIdx.x, x[u] + 1.0f);
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
  const int rounds = argc > 1 ? atoi(argv[1]) : 15;
  const long n = 124475904L;  // T125
  const long n4 = n / 4;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float *a, *b, *c, *d, *sink, *flush;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  CK(hipMalloc(&c, n * 4));
  CK(hipMalloc(&d, n * 4));
  CK(hipMalloc(&sink, 4096));
  const long nf = 1L << 28;  // 1 GiB: evicts the 256 MiB Infinity Cache
  CK(hipMalloc(&flush, nf * 4));
  unsigned seed = 1;
  for (float* p : {a, b, c, d}) hipLaunchKernelGGL(fill, dim3(4096), dim3(T), 0, 0, p, n, seed++);
  CK(hipMemset(flush, 0, nf * 4));
  // walker tables: full chunks, a new "tensor" every 200 chunks; the inner stream is `e`
  const int nch = int(n / CHE);
  float* inb;
  CK(hipMalloc(&inb, n * 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(T), 0, 0, inb, n, seed++);
  std::vector<Chunk> hc(nch);
  std::vector<void*> hca(nch);
  for (int k = 0; k < nch; ++k) {
    hc[k] = Chunk{long(k) * CHE, CHE, k / 200};
    hca[k] = inb + long(k) * CHE;
  }
  Chunk* dch;
  void** dca;
  CK(hipMalloc(&dch, nch * sizeof(Chunk)));
  CK(hipMalloc(&dca, nch * sizeof(void*)));
  CK(hipMemcpy(dch, hc.data(), nch * sizeof(Chunk), hipMemcpyHostToDevice));
  CK(hipMemcpy(dca, hca.data(), nch * sizeof(void*), hipMemcpyHostToDevice));
  const double nw = double(nch) * CHE / n;  // walker variants cover nch*4096 elements
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto tiles = [&](int U) { return unsigned((n4 + U * T - 1) / (U * T)); };
  struct V {
    std::string name;
    double bytes;
    std::function<void()> run;
    std::vector<float> ms;
  };
  std::vector<V> vs;
#define ADD(name, bytes, ...) vs.push_back({name, double(bytes) * n, [&]() { __VA_ARGS__; }, {}})
  ADD("read1<4>  one WG/tile        ", 4, hipLaunchKernelGGL(read1<4>, dim3(tiles(4)), dim3(T), 0, 0, a, sink, n4));
  ADD("read1<8>  one WG/tile        ", 4, hipLaunchKernelGGL(read1<8>, dim3(tiles(8)), dim3(T), 0, 0, a, sink, n4));
  ADD("read1<4>  8 WG/CU persistent ", 4, hipLaunchKernelGGL(read1<4>, dim3(8 * cus), dim3(T), 0, 0, a, sink, n4));
  ADD("copy<4>   one WG/tile        ", 8, hipLaunchKernelGGL((copy<4>), dim3(tiles(4)), dim3(T), 0, 0, a, b, n4));
  ADD("copy<8>   one WG/tile        ", 8, hipLaunchKernelGGL((copy<8>), dim3(tiles(8)), dim3(T), 0, 0, a, b, n4));
  ADD("copy<16>  one WG/tile        ", 8, hipLaunchKernelGGL((copy<16>), dim3(tiles(16)), dim3(T), 0, 0, a, b, n4));
  ADD("copy<4>   plain stores       ", 8, hipLaunchKernelGGL((copy<4, false>), dim3(tiles(4)), dim3(T), 0, 0, a, b, n4));
  ADD("copy<4>   8 WG/CU persistent ", 8, hipLaunchKernelGGL((copy<4>), dim3(8 * cus), dim3(T), 0, 0, a, b, n4));
  ADD("pack<4>   (delta_pack shape) ", 12, hipLaunchKernelGGL(pack<4>, dim3(tiles(4)), dim3(T), 0, 0, a, b, c, n4));
  ADD("pack<8>                      ", 12, hipLaunchKernelGGL(pack<8>, dim3(tiles(8)), dim3(T), 0, 0, a, b, c, n4));
  ADD("sgd6<4>   (unpack_sgd shape) ", 24, hipLaunchKernelGGL(sgd6<4>, dim3(tiles(4)), dim3(T), 0, 0, a, b, c, d, n4));
  ADD("sgd6<2>                      ", 24, hipLaunchKernelGGL(sgd6<2>, dim3(tiles(2)), dim3(T), 0, 0, a, b, c, d, n4));
  ADD("rmw3<4>   (delta_sgd shape)  ", 24, hipLaunchKernelGGL((rmw3<4>), dim3(tiles(4)), dim3(T), 0, 0, b, c, d, n4));
  ADD("rmw3<2>                      ", 24, hipLaunchKernelGGL((rmw3<2>), dim3(tiles(2)), dim3(T), 0, 0, b, c, d, n4));
  ADD("rmw3<4>   in-stream first    ", 24, hipLaunchKernelGGL((rmw3<4, true, true>), dim3(tiles(4)), dim3(T), 0, 0, b, c, d, n4));
  ADD("rmw3<4>   plain stores       ", 24, hipLaunchKernelGGL((rmw3<4, false>), dim3(tiles(4)), dim3(T), 0, 0, b, c, d, n4));
  ADD("pack_w    walker, plain st   ", 12 * nw, hipLaunchKernelGGL(pack_w<false>, dim3(nch), dim3(T), 0, 0, dch, dca, a, c));
  ADD("pack_w    walker, NT st      ", 12 * nw, hipLaunchKernelGGL(pack_w<true>, dim3(nch), dim3(T), 0, 0, dch, dca, a, c));
  ADD("pack_wk<2> walker, prefetch  ", 12 * nw, hipLaunchKernelGGL(pack_wk<2>, dim3((nch + 1) / 2), dim3(T), 0, 0, dch, dca, nch, a, c));
  ADD("pack_wk<4> walker, prefetch  ", 12 * nw, hipLaunchKernelGGL(pack_wk<4>, dim3((nch + 3) / 4), dim3(T), 0, 0, dch, dca, nch, a, c));
  ADD("rmw3_w    walker, NT st      ", 24 * nw, hipLaunchKernelGGL(rmw3_w<true>, dim3(nch), dim3(T), 0, 0, dch, dca, b, d));
  ADD("rmw3_w    walker, plain st   ", 24 * nw, hipLaunchKernelGGL(rmw3_w<false>, dim3(nch), dim3(T), 0, 0, dch, dca, b, d));
  ADD("pack_c    computed descriptor", 12 * nw, hipLaunchKernelGGL(pack_c, dim3(nch), dim3(T), 0, 0, inb, a, c));
  ADD("pack_x    XCD-remapped chunks", 12 * nw, hipLaunchKernelGGL(pack_x, dim3(nch), dim3(T), 0, 0, dch, dca, nch, a, c));
  ADD("dps       flat (28 B)        ", 28 * nw, hipLaunchKernelGGL(dps<false>, dim3(nch), dim3(T), 0, 0, dch, dca, inb, b, d, c));
  ADD("dps       walker (28 B)      ", 28 * nw, hipLaunchKernelGGL(dps<true>, dim3(nch), dim3(T), 0, 0, dch, dca, inb, b, d, c));
  ADD("dps_o     rows, NT wire      ", 28 * nw, hipLaunchKernelGGL((dps_o<false, true>), dim3(nch), dim3(T), 0, 0, dch, dca, b, d, c));
  ADD("dps_o     by stream, NT wire ", 28 * nw, hipLaunchKernelGGL((dps_o<true, true>), dim3(nch), dim3(T), 0, 0, dch, dca, b, d, c));
  ADD("dps_o     by stream, plain w ", 28 * nw, hipLaunchKernelGGL((dps_o<true, false>), dim3(nch), dim3(T), 0, 0, dch, dca, b, d, c));
  for (int r = 0; r < rounds; ++r) {
    for (auto& v : vs) {
      hipLaunchKernelGGL(flush_k, dim3(unsigned(nf / 4 / (4 * T))), dim3(T), 0, 0, flush, nf / 4);
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
  printf("T125-size flat arrays (n=%ld fp32), %d rounds, %d CUs, Infinity Cache evicted before each launch\n",
         n, rounds, cus);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("%s med %8.4f ms %7.1f GB/s  best %7.1f GB/s\n", v.name.c_str(), med,
           v.bytes / med / 1e6, v.bytes / v.ms[0] / 1e6);
  }
  return 0;
}
