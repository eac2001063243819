// Direct peer-access exchange for the outer step (an alternative to RCCL's
// reduce-scatter + all-gather on one node): every rank's packed wire and θ_outer buffers are
// IPC-mapped into every peer, and ONE kernel per rank does, for its 1/n shard of the packed
// tree,
//     g = ((wire_0 + wire_1) + ... + wire_{n-1}) / n     rank order: identical on every rank,
//                                                        bit-exact vs oracle/or_sum_avg
//     Nesterov SGD on θ_rank and the momentum shard      (dl_unpack_sgd's arithmetic)
//     θ_q[k] = θ_new for every peer q                    (the all-gather, as remote stores)
// so the exchange crosses xGMI once per direction per byte, with no staging buffers. The
// caller orders it between two collective barriers (all wires written before any peer reads;
// all θ stores landed before any rank reads θ again); nothing in the kernel waits on a peer.
#include "dl_device.h"

namespace dl {
namespace {

constexpr int kXU = 2;                          // float4 per lane per stream
constexpr int kXChunk = kThreads * kXU * 4;     // 2048 elements per workgroup

// DELTA = false: p.wire[q] is rank q's packed pseudo-gradient (dl_delta_pack's wire).
// DELTA = true (dl_xgmi_delta_sgd): p.wire[q] is rank q's packed INNER parameters and the
// kernel forms the pseudo-gradient itself, θ_outer - inner_q -- the same single subtraction
// rank q would have made (src/utils.py:221; θ_outer is identical on every replica), so the
// result is bit-identical and no rank runs dl_delta_pack.
template <int N, bool DELTA>
__global__ void __launch_bounds__(kThreads)
    k_xgmi_reduce_sgd(XgmiPeers p, int32_t rank, int64_t lo, int64_t len, float* __restrict__ mom,
                      SgdArgs a, int32_t mode) {
  for (int64_t base = int64_t(blockIdx.x) * kXChunk; base < len;
       base += int64_t(gridDim.x) * kXChunk) {
    float4 w[N][kXU];
    float4 t[kXU], m[kXU];
    const int64_t k0 = lo + base;  // packed index of this workgroup's first element
#pragma unroll
    for (int u = 0; u < kXU; ++u) {
      const int64_t e = base + int64_t(u * kThreads + threadIdx.x) * 4;
      if (e < len) {
#pragma unroll
        for (int q = 0; q < N; ++q) w[q][u] = ldf4<true>(p.wire[q] + k0, u * kThreads + threadIdx.x);
        t[u] = ldf4<true>(p.theta[rank] + k0, u * kThreads + threadIdx.x);
        if (mode == 2) m[u] = ldf4<true>(mom + base, u * kThreads + threadIdx.x);
      }
    }
#pragma unroll
    for (int u = 0; u < kXU; ++u) {
      const int64_t e = base + int64_t(u * kThreads + threadIdx.x) * 4;
      if (e < len) {
        float4 g = DELTA ? sub4(t[u], w[0][u]) : w[0][u];
#pragma unroll
        for (int q = 1; q < N; ++q) {
          const float4 d = DELTA ? sub4(t[u], w[q][u]) : w[q][u];
          g = make_float4(g.x + d.x, g.y + d.y, g.z + d.z, g.w + d.w);
        }
        if (N > 1) g = div4(g, float(N));
        if (mode == 0) {
          sgd1<0>(g.x, m[u].x, t[u].x, a);
          sgd1<0>(g.y, m[u].y, t[u].y, a);
          sgd1<0>(g.z, m[u].z, t[u].z, a);
          sgd1<0>(g.w, m[u].w, t[u].w, a);
        } else if (mode == 1) {
          sgd1<1>(g.x, m[u].x, t[u].x, a);
          sgd1<1>(g.y, m[u].y, t[u].y, a);
          sgd1<1>(g.z, m[u].z, t[u].z, a);
          sgd1<1>(g.w, m[u].w, t[u].w, a);
        } else {
          sgd1<2>(g.x, m[u].x, t[u].x, a);
          sgd1<2>(g.y, m[u].y, t[u].y, a);
          sgd1<2>(g.z, m[u].z, t[u].z, a);
          sgd1<2>(g.w, m[u].w, t[u].w, a);
        }
        if (mode != 0) stf4<true>(mom + base, u * kThreads + threadIdx.x, m[u]);
#pragma unroll
        for (int q = 0; q < N; ++q) stf4<true>(p.theta[q] + k0, u * kThreads + threadIdx.x, t[u]);
      }
    }
  }
  // no per-thread system fence here: one per wave (buffer_wbl2 + buffer_inv of the whole L2)
  // made this kernel 23x slower than the same work in dl_shard_sgd (9.7 ms vs 0.41 ms on
  // T125). The caller orders the remote θ stores with dl_sys_fence after the kernel instead.
}

template <int N>
hipError_t launch_n(const XgmiPeers& p, int32_t rank, int64_t lo, int64_t len, float* mom,
                    SgdArgs a, bool delta, hipStream_t s) {
  const int32_t mode = a.momentum == 0.f ? 0 : (a.first ? 1 : 2);
  const int64_t blocks = (len + kXChunk - 1) / kXChunk;
  const int32_t grid = int32_t(blocks < 65536 ? blocks : 65536);
  if (delta)
    hipLaunchKernelGGL((k_xgmi_reduce_sgd<N, true>), dim3(grid), dim3(kThreads), 0, s, p, rank,
                       lo, len, mom, a, mode);
  else
    hipLaunchKernelGGL((k_xgmi_reduce_sgd<N, false>), dim3(grid), dim3(kThreads), 0, s, p, rank,
                       lo, len, mom, a, mode);
  return hipGetLastError();
}

// link probe: dst[i*each + k] = srcs[i][k] for every source, workgroups interleaved across the
// sources so all of them stream at once (each4 = float4 per source, < 2^31)
__global__ void __launch_bounds__(kThreads)
    k_peer_gather(XgmiPeers p, int32_t nsrc, int32_t each4, float* __restrict__ dst) {
  constexpr int U = 4;  // float4 loads in flight per lane
  const int32_t i = int32_t(blockIdx.x) % nsrc;
  const int32_t per = int32_t(gridDim.x) / nsrc;
  const float* src = p.wire[i];
  float* out = dst + int64_t(i) * each4 * 4;
  for (int32_t v0 = (int32_t(blockIdx.x) / nsrc) * kThreads * U; v0 < each4;
       v0 += per * kThreads * U) {
    float4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int32_t v = v0 + u * kThreads + int32_t(threadIdx.x);
      if (v < each4) x[u] = ldf4<true>(src, v);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int32_t v = v0 + u * kThreads + int32_t(threadIdx.x);
      if (v < each4) stf4<true>(out, v, x[u]);
    }
  }
}

// Cross-GPU ordering of coarse-grained buffers (dl_sys_fence): one workgroup per CU (grid =
// the device's multiProcessorCount), each issuing a system-scope fence (buffer_wbl2 sc0 sc1,
// then buffer_inv sc0 sc1) so that every XCD's L2 has written back its dirty lines (peers
// reading this GPU's memory over xGMI see them) and dropped its clean ones (stale copies of
// lines peers have since written here, or of peers' memory). An XCD is covered if at least
// one workgroup lands on it; with one workgroup per CU every XCD receives its share under
// any placement that uses every CU. `xcc` (census, tests): each workgroup records the XCD it
// ran on (s_getreg HW_REG_XCC_ID; a read, the record is a vector store), which
// tests/test_runtime_gpu.py::test_sys_fence_reaches_every_xcd checks covers all XCDs.
__global__ void __launch_bounds__(64) k_sys_fence(uint32_t* __restrict__ xcc) {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
    if (xcc) {
      uint32_t id;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
      xcc[blockIdx.x] = id & 0xFu;
    }
  }
}

int32_t cu_count() {
  static int32_t cached[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

}  // namespace

hipError_t launch_sys_fence(uint32_t* xcc, int32_t* grid_out, hipStream_t s) {
  const int32_t grid = cu_count();
  if (grid_out) *grid_out = grid;
  hipLaunchKernelGGL(k_sys_fence, dim3(grid), dim3(64), 0, s, xcc);
  return hipGetLastError();
}

hipError_t launch_peer_gather(const XgmiPeers& p, int32_t nsrc, int32_t each4, float* dst,
                              hipStream_t s) {
  if (nsrc <= 0 || each4 <= 0) return hipSuccess;
  const int32_t per = 1024;  // workgroups per source
  hipLaunchKernelGGL(k_peer_gather, dim3(per * nsrc), dim3(kThreads), 0, s, p, nsrc, each4, dst);
  return hipGetLastError();
}

hipError_t launch_xgmi_reduce_sgd(const XgmiPeers& p, int32_t n, int32_t rank, int64_t lo,
                                  int64_t len, float* mom, SgdArgs a, bool delta, hipStream_t s) {
  if (len <= 0) return hipSuccess;
  switch (n) {
    case 1: return launch_n<1>(p, rank, lo, len, mom, a, delta, s);
    case 2: return launch_n<2>(p, rank, lo, len, mom, a, delta, s);
    case 3: return launch_n<3>(p, rank, lo, len, mom, a, delta, s);
    case 4: return launch_n<4>(p, rank, lo, len, mom, a, delta, s);
    case 5: return launch_n<5>(p, rank, lo, len, mom, a, delta, s);
    case 6: return launch_n<6>(p, rank, lo, len, mom, a, delta, s);
    case 7: return launch_n<7>(p, rank, lo, len, mom, a, delta, s);
    case 8: return launch_n<8>(p, rank, lo, len, mom, a, delta, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dl
