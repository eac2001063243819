/* A non-Python host driving the outer step through the C-ABI alone (include/diloco_hip.h):
 * plain C, the HIP runtime for device memory, libdiloco_hip.so for the work. Checks two outer
 * steps on a ragged tree bit for bit against the C oracle (oracle/diloco_oracle.c, the
 * restatement of src/utils.py:221, src/train.py:267 and src/utils.py:226):
 *   step 1: dl_delta_pack_sgd (one pass, first step, wire kept)
 *   step 2: dl_delta_pack -> dl_unpack_sgd (divisor 1: one peer, src/comm.py:118-119)
 *   step 3: per bucket dl_delta_pack -> dl_allreduce -> dl_unpack_sgd over a one-rank RCCL
 *           communicator the library creates (dl_rccl_load, dl_comm_unique_id, dl_comm_init)
 *   step 4: the sharded step per bucket: dl_delta_pack -> dl_reduce_scatter -> dl_shard_sgd
 *           -> dl_all_gather -> dl_scatter on the same communicator
 *   step 5: the ordered sharded step (OuterSync(exchange="a2a")) per bucket: dl_delta_pack ->
 *           the all_to_all as grouped dl_send / dl_recv (one rank: its own slice) ->
 *           dl_shard_reduce_sgd -> dl_all_gather -> dl_scatter
 * plus an argument error (unbound slot) reported through the return code and dl_last_error.
 * Built by __graft_entry__.build() (gcc, no GPU needed); run by tests/test_cabi_host.py.
 * Exit status 0 = every byte equal. */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/diloco_hip.h"

/* oracle/liboracle.so (the checker) */
void or_delta(const float* outer, const float* inner, float* out, int64_t n);
void or_sgd(float* theta, float* buf, const float* g, int64_t n, float lr, float momentum,
            int32_t nesterov, int32_t first);
void or_fill_synth(float* dst, int64_t n, uint64_t seed, uint64_t stream, float base, float scale,
                   const float* add);

#define NT 9
static const int64_t NUMEL[NT] = {1, 3, 4097, 0, 64, 65, 12345, 300007, 2};

#define HIP(x)                                                                 \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 2;                                                                \
    }                                                                          \
  } while (0)
#define DL(x)                                                                          \
  do {                                                                                 \
    int r_ = (x);                                                                      \
    if (r_ != DL_OK) {                                                                 \
      fprintf(stderr, "%s:%d rc %d: %s\n", __FILE__, __LINE__, r_, dl_last_error()); \
      return 3;                                                                        \
    }                                                                                  \
  } while (0)

static int same(const char* what, int t, const float* a, const float* b, int64_t n) {
  if (n && memcmp(a, b, (size_t)n * 4)) {
    fprintf(stderr, "mismatch: %s of tensor %d\n", what, t);
    return 0;
  }
  return 1;
}

int main(void) {
  const float lr = 0.7f, mom = 0.9f;
  dl_tree_t tree = NULL;
  DL(dl_tree_create(NUMEL, NT, 5000, &tree)); /* small cap: several buckets */
  int64_t total = 0;
  int32_t nseg = 0, nbkt = 0, nch = 0;
  DL(dl_tree_query(tree, &total, &nseg, &nbkt, &nch));
  int64_t seg_off[NT + 1];
  DL(dl_tree_seg_off(tree, seg_off));

  /* host: θ_0 and the oracle's copies */
  float *h_theta[NT], *h_buf[NT], *h_in[NT], *h_g[NT];
  float *d_in[NT];
  uint64_t ptrs[NT];
  for (int t = 0; t < NT; ++t) {
    const int64_t n = NUMEL[t] ? NUMEL[t] : 1;
    h_theta[t] = malloc(n * 4);
    h_buf[t] = malloc(n * 4);
    h_in[t] = malloc(n * 4);
    h_g[t] = malloc(n * 4);
    or_fill_synth(h_theta[t], NUMEL[t], 42, (uint64_t)t, 0.0f, 0.02f, NULL);
    HIP(hipMalloc((void**)&d_in[t], n * 4));
    ptrs[t] = (uint64_t)(uintptr_t)d_in[t];
  }
  float *d_theta, *d_wire, *d_mom;
  HIP(hipMalloc((void**)&d_theta, total * 4));
  HIP(hipMalloc((void**)&d_wire, total * 4));
  HIP(hipMalloc((void**)&d_mom, total * 4));
  HIP(hipMemset(d_theta, 0, total * 4));
  HIP(hipMemset(d_wire, 0, total * 4));
  HIP(hipMemset(d_mom, 0, total * 4));
  for (int t = 0; t < NT; ++t)
    HIP(hipMemcpy(d_theta + seg_off[t], h_theta[t], NUMEL[t] * 4, hipMemcpyHostToDevice));

  /* an argument error: the inner slot is not bound yet */
  int rc = dl_delta_pack(tree, DL_ALL_BUCKETS, 0, d_theta, d_wire, DL_F32, NULL);
  if (rc == DL_OK || strstr(dl_last_error(), "not bound") == NULL) {
    fprintf(stderr, "expected an unbound-slot error, got %d (%s)\n", rc, dl_last_error());
    return 4;
  }
  DL(dl_tree_bind(tree, 0, ptrs, NT, NULL));

  float* got = malloc(total * 4);
  float* gotm = malloc(total * 4);
  float* gotw = malloc(total * 4);
  /* steps 3-4: RCCL through the library, one rank (src/comm.py:122 with one peer) */
  DL(dl_rccl_load(NULL));
  char id[128];
  dl_comm_t comm = NULL;
  DL(dl_comm_unique_id(id));
  DL(dl_comm_init(&comm, 1, id, 0));
  float *d_gshard, *d_thshard, *d_momshard; /* this rank's shards: the whole bucket at n = 1 */
  HIP(hipMalloc((void**)&d_gshard, total * 4));
  HIP(hipMalloc((void**)&d_thshard, total * 4));
  HIP(hipMalloc((void**)&d_momshard, total * 4));
  int ok = 1;
  for (int step = 1; step <= 5; ++step) {
    /* inner = θ + noise (the synthetic stand-in for H inner steps) */
    for (int t = 0; t < NT; ++t) {
      or_fill_synth(h_in[t], NUMEL[t], (uint64_t)(1000 * step), (uint64_t)t, 0.0f, 1e-3f,
                    h_theta[t]);
      HIP(hipMemcpy(d_in[t], h_in[t], NUMEL[t] * 4, hipMemcpyHostToDevice));
    }
    if (step == 1) {
      DL(dl_delta_pack_sgd(tree, DL_ALL_BUCKETS, 0, d_theta, d_wire, DL_F32, d_mom, lr, mom, 1, 1,
                           NULL));
    } else if (step == 2) {
      for (int32_t b = 0; b < nbkt; ++b) {
        DL(dl_delta_pack(tree, b, 0, d_theta, d_wire, DL_F32, NULL));
        DL(dl_unpack_sgd(tree, b, d_wire, DL_F32, 1, d_theta, d_mom, lr, mom, 1, 0, 0, NULL));
      }
    } else if (step == 3) {
      for (int32_t b = 0; b < nbkt; ++b) {
        int64_t lo = 0, hi = 0;
        DL(dl_tree_bucket_range(tree, b, &lo, &hi));
        DL(dl_delta_pack(tree, b, 0, d_theta, d_wire, DL_F32, NULL));
        DL(dl_allreduce(d_wire + lo, hi - lo, DL_F32, comm, NULL));
        DL(dl_unpack_sgd(tree, b, d_wire, DL_F32, 1, d_theta, d_mom, lr, mom, 1, 0, 0, NULL));
      }
    } else if (step == 5) {
      HIP(hipMemcpy(d_thshard, d_theta, total * 4, hipMemcpyDeviceToDevice));
      HIP(hipMemcpy(d_momshard, d_mom, total * 4, hipMemcpyDeviceToDevice));
      for (int32_t b = 0; b < nbkt; ++b) {
        int64_t lo = 0, hi = 0;
        DL(dl_tree_bucket_range(tree, b, &lo, &hi));
        DL(dl_delta_pack(tree, b, 0, d_theta, d_wire, DL_F32, NULL));
        DL(dl_group_start());
        DL(dl_send(d_wire + lo, hi - lo, DL_F32, 0, comm, NULL));
        DL(dl_recv(d_gshard + lo, hi - lo, DL_F32, 0, comm, NULL));
        DL(dl_group_end());
        DL(dl_shard_reduce_sgd(d_gshard + lo, DL_F32, 1, hi - lo, d_thshard + lo, d_momshard + lo,
                               lr, mom, 1, 0, NULL));
        DL(dl_all_gather(d_thshard + lo, d_theta + lo, hi - lo, DL_F32, comm, NULL));
        DL(dl_scatter(tree, b, d_theta, 0, NULL));
      }
      HIP(hipMemcpy(d_mom, d_momshard, total * 4, hipMemcpyDeviceToDevice));
    } else {
      HIP(hipMemcpy(d_thshard, d_theta, total * 4, hipMemcpyDeviceToDevice));
      HIP(hipMemcpy(d_momshard, d_mom, total * 4, hipMemcpyDeviceToDevice));
      for (int32_t b = 0; b < nbkt; ++b) {
        int64_t lo = 0, hi = 0;
        DL(dl_tree_bucket_range(tree, b, &lo, &hi));
        DL(dl_delta_pack(tree, b, 0, d_theta, d_wire, DL_F32, NULL));
        DL(dl_reduce_scatter(d_wire + lo, d_gshard + lo, hi - lo, DL_F32, comm, NULL));
        DL(dl_shard_sgd(d_gshard + lo, DL_F32, 1, d_thshard + lo, d_momshard + lo, hi - lo, lr,
                        mom, 1, 0, NULL));
        DL(dl_all_gather(d_thshard + lo, d_theta + lo, hi - lo, DL_F32, comm, NULL));
        DL(dl_scatter(tree, b, d_theta, 0, NULL));
      }
      HIP(hipMemcpy(d_mom, d_momshard, total * 4, hipMemcpyDeviceToDevice));
    }
    HIP(hipDeviceSynchronize());
    for (int t = 0; t < NT; ++t) { /* the oracle's step */
      or_delta(h_theta[t], h_in[t], h_g[t], NUMEL[t]);
      or_sgd(h_theta[t], h_buf[t], h_g[t], NUMEL[t], lr, mom, 1, step == 1);
    }
    HIP(hipMemcpy(got, d_theta, total * 4, hipMemcpyDeviceToHost));
    HIP(hipMemcpy(gotm, d_mom, total * 4, hipMemcpyDeviceToHost));
    HIP(hipMemcpy(gotw, d_wire, total * 4, hipMemcpyDeviceToHost));
    for (int t = 0; t < NT; ++t) {
      ok &= same("theta", t, got + seg_off[t], h_theta[t], NUMEL[t]);
      ok &= same("momentum", t, gotm + seg_off[t], h_buf[t], NUMEL[t]);
      ok &= same("wire (outer.grad)", t, gotw + seg_off[t], h_g[t], NUMEL[t]);
      HIP(hipMemcpy(h_in[t], d_in[t], NUMEL[t] * 4, hipMemcpyDeviceToHost));
      ok &= same("inner (sync_inner_model)", t, h_in[t], h_theta[t], NUMEL[t]);
    }
  }
  DL(dl_comm_destroy(comm));
  DL(dl_tree_destroy(tree));
  printf("cabi host: %d tensors, %lld packed elements, %d buckets, %d chunks: %s\n", NT,
         (long long)total, nbkt, nch, ok ? "bit-exact vs oracle" : "MISMATCH");
  return ok ? 0 : 1;
}
