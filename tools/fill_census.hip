// Diagnostic twin of dl_fill_synth (tools/stripe_diag.py --census): the same values
// (same key, same splitmix64 arithmetic, one workgroup per 256 elements), and every workgroup
// also records where and whether it ran -- start[b] before its stores, end[b] after them and a
// workgroup barrier -- as 0x80000000 | XCC_ID << 24 | VM_ID << 16 | SE_ID << 8 | CU_ID
// (s_getreg reads; the records are vector stores). A block whose data is missing afterwards then says which of
// three things happened: no start record (its workgroup never ran), a start but no end record
// (it stopped inside), or both records (it ran to the end and its data stores still did not
// land), and on which XCD.
//
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/fill_census.hip -o build_ab/libfill_census.so
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t where_am_i() {
  uint32_t xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  const uint32_t cu = (hw >> 8) & 0xF, se = (hw >> 13) & 0x7, vm = (hw >> 20) & 0xF;
  return 0x80000000u | ((xcc & 0xF) << 24) | (vm << 16) | (se << 8) | cu;
}

__global__ void __launch_bounds__(256)
    k_fill_census(float* __restrict__ dst, int64_t n, uint64_t key0, float base, float scale,
                  const float* __restrict__ add, uint32_t* __restrict__ start,
                  uint32_t* __restrict__ end) {
  const uint32_t me = where_am_i();
  if (threadIdx.x == 0) start[blockIdx.x] = me;
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i < n) {
    const uint64_t z = splitmix64(key0 + uint64_t(i));
    const float u = float(int32_t(z >> 40) - 8388608) * 1.1920928955078125e-07f;
    float x = base + u * scale;
    if (add) x = x + add[i];
    dst[i] = x;
  }
  __syncthreads();
  if (threadIdx.x == 0) end[blockIdx.x] = me;
}

}  // namespace

extern "C" int fc_fill(float* dst, int64_t n, uint64_t seed, uint64_t stream_id, float base,
                       float scale, const float* add, uint32_t* start, uint32_t* end,
                       hipStream_t s) {
  if (n <= 0) return 0;
  const uint64_t key0 = seed * 0xD1B54A32D192ED03ull + (stream_id << 40);
  const int64_t g = (n + 255) / 256;
  if (g >= (1ll << 31)) return 1;
  hipLaunchKernelGGL(k_fill_census, dim3(unsigned(g)), dim3(256), 0, s, dst, n, key0, base,
                     scale, add, start, end);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
