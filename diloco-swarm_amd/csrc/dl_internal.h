// Internal declarations shared by the kernel TU (dl_kernels.hip) and the C-ABI TU (dl_abi.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/diloco_hip.h"

namespace dl {

constexpr int kThreads = 256;                          // 4 waves of 64 lanes
constexpr int kUnroll = DL_CHUNK_ELEMS / (kThreads * 4);  // float4 per lane per chunk (=4)
static_assert(kUnroll * kThreads * 4 == DL_CHUNK_ELEMS, "chunk must be a whole number of sweeps");

// One work unit: up to DL_CHUNK_ELEMS consecutive elements of one segment; 16 B, fetched by
// a workgroup with one scalar load. The address of the chunk's first element inside each
// bound per-tensor slot is pre-resolved at bind time (Launch::caddr), so a workgroup's two
// descriptor loads are independent instead of a chunk -> tensor -> pointer chain.
struct Chunk {
  int64_t poff;  // offset in the packed space
  int32_t len;   // elements, 1..DL_CHUNK_ELEMS
  int32_t seg;   // segment (tensor) index in parameters() order
};
static_assert(sizeof(Chunk) == 16, "Chunk layout");

inline bool aligned16_host(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

struct SgdArgs {
  float neg_lr;    // fp32(-lr): torch passes alpha=-lr, rounded to the tensor dtype
  float momentum;  // fp32(momentum)
  int32_t nesterov;
  int32_t first;   // momentum buffer not yet created (torch: buf = clone(grad))
};

struct Launch {
  const Chunk* chunks;  // device chunk table
  int32_t c0, c1;       // chunk range
  void* const* caddr;   // device table [DL_MAX_SLOTS][nchunk]: per-slot address of each chunk
  int32_t nchunk;
  int32_t grid;   // 0 = one workgroup per chunk
  int32_t flags;  // DL_TUNE_*
  hipStream_t stream;
  bool pairs;  // two chunks per workgroup, loads of both before the stores (run_pairs)
  // workgroup -> chunk mapping with one workgroup per chunk (walk_index, dl_device.h): XCD x
  // walks runs of 2^xlog consecutive chunks (0: one chunk, the dispatcher's own interleave;
  // -1: one contiguous eighth of the range per XCD)
  int32_t xlog;
};

// peers of the direct exchange (dl_xgmi.hip): each rank's packed wire and θ, IPC-mapped
constexpr int kMaxPeers = 8;
struct XgmiPeers {
  const float* wire[kMaxPeers];
  float* theta[kMaxPeers];
};
// delta: p.wire[] holds the peers' packed inner parameters (dl_xgmi_delta_sgd)
hipError_t launch_xgmi_reduce_sgd(const XgmiPeers& p, int32_t n, int32_t rank, int64_t lo,
                                  int64_t len, float* mom, SgdArgs a, bool delta, hipStream_t s);
// xcc (may be null): one entry per workgroup, the XCD (HW_REG_XCC_ID) it ran on; *grid_out
// (may be null) = the grid size used (one 64-lane workgroup per CU of the current device)
hipError_t launch_sys_fence(uint32_t* xcc, int32_t* grid_out, hipStream_t s);
hipError_t launch_peer_gather(const XgmiPeers& p, int32_t nsrc, int32_t each4, float* dst,
                              hipStream_t s);

// dl_last_error() text for entry points outside dl_abi.hip; returns `code`
int set_error(int code, const char* msg);

hipError_t launch_delta_pack(const Launch& L, int inner_slot, const float* outer, void* wire,
                             int wire_dtype);
hipError_t launch_unpack_avg(const Launch& L, const void* wire, int wire_dtype, int divisor,
                             int dst_slot, float* dst_packed);
hipError_t launch_unpack_sgd(const Launch& L, const void* wire, int wire_dtype, int divisor,
                             float* outer, float* mom, SgdArgs a, int inner_slot);
hipError_t launch_delta_sgd(const Launch& L, int inner_slot, float* outer, float* mom, SgdArgs a);
hipError_t launch_delta_pack_sgd(const Launch& L, int inner_slot, float* outer, void* wire,
                                 int wire_dtype, float* mom, SgdArgs a);
hipError_t launch_shard_sgd(const void* wire, int wire_dtype, int divisor, float* outer, float* mom,
                            int64_t n, SgdArgs a, hipStream_t s);
hipError_t launch_slices_sgd(const void* slices, int wire_dtype, int32_t n, int64_t len,
                             float* outer, float* mom, SgdArgs a, hipStream_t s,
                             bool avg_only = false);
hipError_t launch_delta_q8(const Launch& L, int inner_slot, const float* outer, uint8_t* slots);
hipError_t launch_unpack_sgd_q8(const Launch& L, const uint8_t* slots, float* outer, float* mom,
                                SgdArgs a, int inner_slot);
hipError_t launch_q8_reduce(const uint8_t* recv, int32_t n, int32_t m, int32_t divisor,
                            uint8_t* out, hipStream_t s);
hipError_t launch_gather(const Launch& L, int src_slot, void* packed, int dtype);
hipError_t launch_scatter(const Launch& L, const float* packed, int dst_slot);
hipError_t launch_serialize_f64(const double* src, int64_t numel, float m0, float m1, double* out,
                                hipStream_t s);
hipError_t launch_serialize(const void* src, int src_dtype, int64_t numel, float m0, float m1,
                            float* out, hipStream_t s);
hipError_t launch_fill_synth(float* dst, int64_t n, uint64_t seed, uint64_t stream_id,
                             float base, float scale, const float* add, hipStream_t s);
hipError_t launch_spin(uint64_t ns, hipStream_t s);
// dl_tree_bind: out[c] = segptr[chunks[c].seg] + 4 * loff[c] for every chunk c
hipError_t launch_resolve_chunks(const Chunk* chunks, const int64_t* loff, const uint64_t* segptr,
                                 int32_t nch, void** out, hipStream_t s);
// flat 16-B streaming copy (the same-run copy ceiling of bench.py): n16 float4, nt = NT
// policy, wide = 8 instead of 4 float4 loads in flight per lane
hipError_t launch_copy(const void* src, void* dst, int64_t n16, bool nt, bool wide,
                       hipStream_t s);
hipError_t launch_probe(bool write, int streams, const void* src, void* dst, int64_t per16,
                        bool nt, hipStream_t s);

}  // namespace dl
