/*
 * diloco_oracle.c -- CPU restatement of the reference's DiLoCo outer step (checker only).
 *
 * TEST INFRASTRUCTURE. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may
 * load this library, and only as the checker; the product path (libdiloco_hip.so) never
 * links or calls it. Pinned against outputs of the reference itself, imported in the build
 * container (tests/golden/make_golden.py -> tests/golden/*), see DESIGN.md "Oracle".
 *
 * Reference semantics restated (paths relative to the reference repo root):
 *   or_delta      src/utils.py:218-221   grad = outer - inner                  (1 rounding)
 *   or_sum_avg    src/comm.py:117-123    all_reduce(SUM) then grad /= num_peers (true div);
 *                                        num_peers == 1 returns early (no division)
 *   or_sgd        torch.optim.SGD._single_tensor_sgd as built by src/utils.py:62-63
 *                 (weight_decay 0, dampening 0, maximize False), stepped at src/train.py:267:
 *                   first step: buf = clone(g)    else: buf = buf*m (mul_) then + g (add_)
 *                   nesterov:   u = g + m*buf  -> torch CPU `add(alpha)` is fmadd: fmaf(buf,m,g)
 *                   param.add_(u, alpha=-lr)   -> fmaf(u, -lr, θ)
 *                 momentum == 0: θ = fmaf(g, -lr, θ) (no buffer)
 *   or_copy       src/utils.py:223-226   inner = outer
 *   or_plan_tables(_ex)  the build's packed layout (no reference counterpart: the reference
 *                 walks model.parameters() in order, src/comm.py:120); rule frozen in DESIGN.md.
 * Build: make -C oracle  (gcc, -O2 -ffp-contract=off so only the fmaf calls fuse).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define OR_API __attribute__((visibility("default")))

/* Placement rule restated from DESIGN.md §2: tensor i goes at the next align boundary; if
 * that pushes the current bucket's padded size past cap (and i is not the bucket's first
 * tensor) i opens a new bucket, which starts at the next bucket_align boundary. */
OR_API int or_plan_tables_ex(const int64_t* numel, int32_t n, int64_t cap, int32_t align,
                             int64_t bucket_align, int64_t* seg_off, int64_t* bounds,
                             int32_t* n_bkt) {
  if (n < 0 || align <= 0 || bucket_align <= 0 || bucket_align % align) return -1;
  bounds[0] = 0;
  if (n == 0) {
    seg_off[0] = 0;
    *n_bkt = 0;
    return 0;
  }
  int32_t nb = 0;
  int64_t next = 0, bucket_begin = 0;
  for (int32_t i = 0; i < n; ++i) {
    if (numel[i] < 0) return -1;
    int64_t at = next;
    int64_t end = (at + numel[i] + align - 1) / align * align;
    if (cap > 0 && i > bounds[nb] && end - bucket_begin > cap) {
      at = (next + bucket_align - 1) / bucket_align * bucket_align;
      bucket_begin = at;
      end = (at + numel[i] + align - 1) / align * align;
      bounds[++nb] = i;
    }
    seg_off[i] = at;
    next = end;
  }
  seg_off[n] = (next + bucket_align - 1) / bucket_align * bucket_align;
  bounds[++nb] = n;
  *n_bkt = nb;
  return 0;
}

OR_API int or_plan_tables(const int64_t* numel, int32_t n, int64_t cap, int32_t align,
                          int64_t* seg_off, int64_t* bounds, int32_t* n_bkt) {
  if (align <= 0) return -1;
  return or_plan_tables_ex(numel, n, cap, align, align, seg_off, bounds, n_bkt);
}

OR_API void or_delta(const float* outer, const float* inner, float* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = outer[i] - inner[i];
}

/* out = (((g0 + g1) + g2) + ...) / nranks  (rank-order sum; gloo's order is an
 * implementation detail of gloo, bit-identical to this only for nranks <= 2). */
OR_API void or_sum_avg(const float* const* grads, int32_t nranks, float* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    float s = grads[0][i];
    for (int32_t r = 1; r < nranks; ++r) s = s + grads[r][i];
    out[i] = nranks == 1 ? s : s / (float)nranks;
  }
}

OR_API void or_sgd(float* theta, float* buf, const float* g, int64_t n, float lr, float momentum,
                   int32_t nesterov, int32_t first) {
  const float neg_lr = -lr;
  for (int64_t i = 0; i < n; ++i) {
    if (momentum == 0.0f) {
      theta[i] = fmaf(g[i], neg_lr, theta[i]);
      continue;
    }
    float b = first ? g[i] : (buf[i] * momentum) + g[i];
    buf[i] = b;
    float u = nesterov ? fmaf(b, momentum, g[i]) : b;
    theta[i] = fmaf(u, neg_lr, theta[i]);
  }
}

OR_API void or_copy(const float* src, float* dst, int64_t n) { memcpy(dst, src, (size_t)n * 4); }

/* fp32 -> bf16 (round to nearest even, NaN kept NaN) -> fp32: the bf16 wire codec. */
OR_API void or_bf16_round(const float* x, float* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    uint32_t u;
    memcpy(&u, &x[i], 4);
    uint32_t r;
    if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu))
      r = (u | 0x00400000u) & 0xffff0000u;
    else
      r = (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
    memcpy(&out[i], &r, 4);
  }
}

static uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* Same generator as diloco_amd.synth / dl_fill_synth (cross-checks both). */
OR_API void or_fill_synth(float* dst, int64_t n, uint64_t seed, uint64_t stream, float base,
                          float scale, const float* add) {
  const uint64_t key0 = seed * 0xD1B54A32D192ED03ull + (stream << 40);
  for (int64_t i = 0; i < n; ++i) {
    uint64_t z = splitmix64(key0 + (uint64_t)i);
    float u = (float)((int32_t)(z >> 40) - 8388608) * 1.1920928955078125e-07f;
    float x = base + u * scale;
    if (add) x = x + add[i];
    dst[i] = x;
  }
}

/* ---- int8 wire codec (the build's own codec; restates dl_q8.hip) ------
 * Slot = 64-B header (fp32 scale at byte 0) + 4096 int8 values; s = amax/127,
 * q = s == 0 ? 0 : clamp(rint(x/s), -127, 127); dequantised value q*s. */
#define OR_Q8_HDR 64
#define OR_Q8_SLOT 4160
#define OR_CHUNK 4096

static int8_t or_q8(float x, float s) {
  if (s == 0.0f) return 0;
  return (int8_t)(int)fminf(fmaxf(rintf(x / s), -127.0f), 127.0f);
}

static void or_quantize(const float* x, int64_t len, uint8_t* slot) {
  float am = 0.0f;
  for (int64_t i = 0; i < len; ++i) am = fmaxf(am, fabsf(x[i]));
  const float s = am / 127.0f;
  memcpy(slot, &s, 4);
  for (int64_t i = 0; i < len; ++i) slot[OR_Q8_HDR + i] = (uint8_t)or_q8(x[i], s);
}

/* one chunk: slot <- quantise(outer - inner); bytes past len untouched */
OR_API void or_delta_q8(const float* outer, const float* inner, int64_t len, uint8_t* slot) {
  float d[OR_CHUNK];
  for (int64_t i = 0; i < len; ++i) d[i] = outer[i] - inner[i];
  or_quantize(d, len, slot);
}

OR_API void or_q8_deq(const uint8_t* slot, int64_t len, float* out) {
  float s;
  memcpy(&s, slot, 4);
  for (int64_t i = 0; i < len; ++i) out[i] = (float)(int8_t)slot[OR_Q8_HDR + i] * s;
}

/* out[j] <- quantise((sum_{r<n} deq(recv[r*m + j])) / divisor), over all 4096 values */
OR_API void or_q8_reduce(const uint8_t* recv, int32_t n, int32_t m, int32_t divisor,
                         uint8_t* out) {
  float acc[OR_CHUNK], x[OR_CHUNK];
  for (int32_t j = 0; j < m; ++j) {
    for (int i = 0; i < OR_CHUNK; ++i) acc[i] = 0.0f;
    for (int32_t r = 0; r < n; ++r) {
      or_q8_deq(recv + ((int64_t)r * m + j) * OR_Q8_SLOT, OR_CHUNK, x);
      for (int i = 0; i < OR_CHUNK; ++i) acc[i] = acc[i] + x[i];
    }
    if (divisor > 1)
      for (int i = 0; i < OR_CHUNK; ++i) acc[i] = acc[i] / (float)divisor;
    or_quantize(acc, OR_CHUNK, out + (int64_t)j * OR_Q8_SLOT);
  }
}
