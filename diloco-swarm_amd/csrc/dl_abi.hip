// C-ABI of libdiloco_hip.so (include/diloco_hip.h): argument checking, the layout planner,
// tree handles (chunk table + device pointer tables) and kernel dispatch.
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "dl_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int hip_fail(hipError_t e, const char* where) {
  return fail(int(e), "%s: %s (%s)", where, hipGetErrorName(e), hipGetErrorString(e));
}

#define DL_HIP(call, where)                          \
  do {                                               \
    hipError_t e_ = (call);                          \
    if (e_ != hipSuccess) return hip_fail(e_, where); \
  } while (0)

int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

// The planner rule (frozen; bit-exact contract with oracle/diloco_oracle.c:or_plan_tables and
// diloco_amd/plan.py). Tensors are placed in order at align-element boundaries; a tensor that
// would push the current bucket's padded size past cap starts a new bucket (never the first
// tensor of a bucket), and a bucket starts at a bucket_align boundary (bucket_align == align:
// no gap). seg_off[n] = end of the tree, rounded up to bucket_align. Returns number of buckets.
int plan(const int64_t* numel, int32_t n, int64_t cap, int32_t align, int64_t bucket_align,
         int64_t* seg_off, int64_t* bounds) {
  bounds[0] = 0;
  if (n == 0) {
    seg_off[0] = 0;
    return 0;
  }
  int nb = 0;
  int64_t pos = 0, bstart = 0;
  for (int32_t i = 0; i < n; ++i) {
    int64_t s = pos, e = align_up(s + numel[i], align);
    if (cap > 0 && i > bounds[nb] && e - bstart > cap) {
      s = bstart = align_up(pos, bucket_align);
      e = align_up(s + numel[i], align);
      bounds[++nb] = i;
    }
    seg_off[i] = s;
    pos = e;
  }
  seg_off[n] = align_up(pos, bucket_align);
  bounds[++nb] = n;
  return nb;
}

}  // namespace

namespace dl {
int set_error(int code, const char* msg) { return fail(code, "%s", msg); }
}  // namespace dl

struct dl_tree_s;
namespace {
int slot_begin(dl_tree_s* t, int32_t slot, hipStream_t s, const char* who);
int slot_end(dl_tree_s* t, int32_t slot, hipStream_t s, const char* who);
}  // namespace

// Pointer-table uploads go through a small ring of pinned staging slots, each guarded by the
// event of the copy that last read it, so dl_tree_bind never synchronises the host with the
// stream (a DP sync rebinding reallocated .grad tensors every inner step stays asynchronous).
constexpr int kStageRing = 4;

struct dl_tree_s {
  int device = 0;
  int32_t nseg = 0;
  int64_t total = 0;
  std::vector<int64_t> numel, seg_off, bounds;
  std::vector<int32_t> bkt_chunk;  // first chunk of each bucket, + sentinel
  std::vector<dl::Chunk> chunks;
  std::vector<int64_t> chunk_loff;  // offset of each chunk inside its tensor (host copy)
  dl::Chunk* d_chunks = nullptr;
  int64_t* d_loff = nullptr;    // chunk_loff on the device (the resolve kernel's input)
  void** d_caddr = nullptr;     // [DL_MAX_SLOTS][nchunk] resolved chunk addresses
  uint64_t* d_segptr = nullptr; // [DL_MAX_SLOTS][nseg] tensor base addresses
  uint64_t* h_stage = nullptr;  // pinned staging ring: kStageRing x nseg addresses
  hipEvent_t stage_ev[kStageRing] = {};
  bool stage_used[kStageRing] = {};
  int stage_next = 0;
  std::vector<uint8_t> bound;   // slot bound?
  std::vector<uint8_t> slot_aligned;
  int32_t grid = 0;                 // 0 = one workgroup per chunk
  int32_t flags = DL_TUNE_AUTO;
  // Per slot: the event recorded after its last bind or launch and that call's stream. A bind
  // or launch on another stream waits for it first, so the slot's address table is never
  // rewritten under (or read before) work queued on a stream the caller did not order.
  hipEvent_t slot_ev[DL_MAX_SLOTS] = {};
  hipStream_t slot_stream[DL_MAX_SLOTS] = {};
  bool slot_used[DL_MAX_SLOTS] = {};
};

namespace {
// Cross-stream ordering of a slot (dl_tree_s::slot_ev): a bind or launch that uses `slot` on a
// stream other than the slot's last one first waits for the event recorded after that use;
// every use records the event again afterwards. One stream (the usual case) costs one event
// record per call and no wait.
int slot_begin(dl_tree_s* t, int32_t slot, hipStream_t s, const char* who) {
  if (slot < 0) return DL_OK;
  if (t->slot_used[slot] && t->slot_stream[slot] != s)
    DL_HIP(hipStreamWaitEvent(s, t->slot_ev[slot], 0), who);
  return DL_OK;
}
int slot_end(dl_tree_s* t, int32_t slot, hipStream_t s, const char* who) {
  if (slot < 0) return DL_OK;
  DL_HIP(hipEventRecord(t->slot_ev[slot], s), who);
  t->slot_stream[slot] = s;
  t->slot_used[slot] = true;
  return DL_OK;
}
}  // namespace

extern "C" {

DL_API const char* dl_last_error(void) { return g_err.c_str(); }
DL_API int dl_abi_version(void) { return DL_ABI_VERSION; }

DL_API int dl_plan_tables_ex(const int64_t* numel, int32_t n, int64_t cap_elems,
                             int32_t align_elems, int64_t bucket_align_elems, int64_t* seg_off,
                             int64_t* bkt_bounds, int32_t* n_bkt) {
  if (n < 0 || (n > 0 && !numel) || !seg_off || !bkt_bounds || !n_bkt)
    return fail(DL_E_ARG, "dl_plan_tables: null pointer or n < 0");
  if (align_elems <= 0) return fail(DL_E_ARG, "dl_plan_tables: align_elems must be > 0");
  if (bucket_align_elems <= 0 || bucket_align_elems % align_elems)
    return fail(DL_E_ARG, "dl_plan_tables: bucket_align %lld is not a positive multiple of %d",
                (long long)bucket_align_elems, align_elems);
  for (int32_t i = 0; i < n; ++i)
    if (numel[i] < 0) return fail(DL_E_ARG, "dl_plan_tables: numel[%d] < 0", i);
  *n_bkt = plan(numel, n, cap_elems, align_elems, bucket_align_elems, seg_off, bkt_bounds);
  return DL_OK;
}

DL_API int dl_plan_tables(const int64_t* numel, int32_t n, int64_t cap_elems, int32_t align_elems,
                          int64_t* seg_off, int64_t* bkt_bounds, int32_t* n_bkt) {
  return dl_plan_tables_ex(numel, n, cap_elems, align_elems, align_elems, seg_off, bkt_bounds,
                           n_bkt);
}

DL_API int dl_tree_create(const int64_t* numel, int32_t n, int64_t cap_elems, dl_tree_t* out) {
  return dl_tree_create_ex(numel, n, cap_elems, DL_ALIGN_ELEMS, out);
}

DL_API int dl_tree_create_ex(const int64_t* numel, int32_t n, int64_t cap_elems,
                             int64_t bucket_align_elems, dl_tree_t* out) {
  if (!out) return fail(DL_E_ARG, "dl_tree_create: out is null");
  *out = nullptr;
  if (n < 0 || (n > 0 && !numel)) return fail(DL_E_ARG, "dl_tree_create: bad numel/n");
  dl_tree_s* t = new (std::nothrow) dl_tree_s;
  if (!t) return fail(DL_E_STATE, "dl_tree_create: out of host memory");
  t->nseg = n;
  t->numel.assign(numel, numel + n);
  t->seg_off.resize(size_t(n) + 1);
  t->bounds.resize(size_t(n) + 1);
  int32_t nb = 0;
  int rc = dl_plan_tables_ex(numel, n, cap_elems, DL_ALIGN_ELEMS, bucket_align_elems,
                             t->seg_off.data(), t->bounds.data(), &nb);
  if (rc) {
    delete t;
    return rc;
  }
  t->bounds.resize(size_t(nb) + 1);
  t->total = t->seg_off[t->nseg];
  // chunk table, bucket-major (buckets are contiguous runs of segments)
  t->bkt_chunk.resize(size_t(nb) + 1);
  for (int32_t b = 0; b < nb; ++b) {
    t->bkt_chunk[b] = int32_t(t->chunks.size());
    for (int64_t s = t->bounds[b]; s < t->bounds[b + 1]; ++s) {
      for (int64_t off = 0; off < t->numel[s]; off += DL_CHUNK_ELEMS) {
        dl::Chunk c{};
        c.poff = t->seg_off[s] + off;
        c.seg = int32_t(s);
        const int64_t rem = t->numel[s] - off;
        c.len = int32_t(rem < DL_CHUNK_ELEMS ? rem : DL_CHUNK_ELEMS);
        t->chunks.push_back(c);
        t->chunk_loff.push_back(off);
      }
    }
    if (t->chunks.size() > size_t(INT32_MAX)) {
      delete t;
      return fail(DL_E_ARG, "dl_tree_create: tree too large for int32 chunk indices");
    }
  }
  t->bkt_chunk[nb] = int32_t(t->chunks.size());
  t->bound.assign(DL_MAX_SLOTS, 0);
  t->slot_aligned.assign(DL_MAX_SLOTS, 1);

  hipError_t e = hipGetDevice(&t->device);
  const size_t nch = t->chunks.empty() ? 1 : t->chunks.size();
  const size_t nsg = n > 0 ? size_t(n) : 1;
  const size_t cbytes = nch * sizeof(dl::Chunk);
  const size_t abytes = size_t(DL_MAX_SLOTS) * nch * sizeof(void*);
  if (e == hipSuccess) e = hipMalloc(&t->d_chunks, cbytes);
  if (e == hipSuccess) e = hipMalloc(&t->d_loff, nch * sizeof(int64_t));
  if (e == hipSuccess) e = hipMalloc(&t->d_caddr, abytes);
  if (e == hipSuccess) e = hipMemset(t->d_caddr, 0, abytes);
  if (e == hipSuccess) e = hipMalloc(&t->d_segptr, size_t(DL_MAX_SLOTS) * nsg * sizeof(uint64_t));
  if (e == hipSuccess && !t->chunks.empty())
    e = hipMemcpy(t->d_chunks, t->chunks.data(), t->chunks.size() * sizeof(dl::Chunk),
                  hipMemcpyHostToDevice);
  if (e == hipSuccess && !t->chunks.empty())
    e = hipMemcpy(t->d_loff, t->chunk_loff.data(), t->chunks.size() * sizeof(int64_t),
                  hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipHostMalloc(reinterpret_cast<void**>(&t->h_stage), kStageRing * nsg * sizeof(uint64_t),
                      hipHostMallocDefault);
  for (int i = 0; i < kStageRing && e == hipSuccess; ++i)
    e = hipEventCreateWithFlags(&t->stage_ev[i], hipEventDisableTiming);
  for (int i = 0; i < DL_MAX_SLOTS && e == hipSuccess; ++i)
    e = hipEventCreateWithFlags(&t->slot_ev[i], hipEventDisableTiming);
  if (e != hipSuccess) {
    int rc2 = hip_fail(e, "dl_tree_create");
    dl_tree_destroy(t);
    return rc2;
  }
  *out = t;
  return DL_OK;
}

DL_API int dl_tree_destroy(dl_tree_t t) {
  if (!t) return DL_OK;
  // uploads still in flight read the staging ring: let them land before freeing it
  for (int i = 0; i < kStageRing; ++i)
    if (t->stage_ev[i]) {
      if (t->stage_used[i]) (void)hipEventSynchronize(t->stage_ev[i]);
      (void)hipEventDestroy(t->stage_ev[i]);
    }
  for (int i = 0; i < DL_MAX_SLOTS; ++i)
    if (t->slot_ev[i]) (void)hipEventDestroy(t->slot_ev[i]);
  if (t->d_chunks) (void)hipFree(t->d_chunks);
  if (t->d_loff) (void)hipFree(t->d_loff);
  if (t->d_caddr) (void)hipFree(t->d_caddr);
  if (t->d_segptr) (void)hipFree(t->d_segptr);
  if (t->h_stage) (void)hipHostFree(t->h_stage);
  delete t;
  return DL_OK;
}

DL_API int dl_tree_query(dl_tree_t t, int64_t* total, int32_t* nseg, int32_t* nbkt,
                         int32_t* nchunk) {
  if (!t) return fail(DL_E_ARG, "dl_tree_query: null tree");
  if (total) *total = t->total;
  if (nseg) *nseg = t->nseg;
  if (nbkt) *nbkt = int32_t(t->bounds.size()) - 1;
  if (nchunk) *nchunk = int32_t(t->chunks.size());
  return DL_OK;
}

DL_API int dl_tree_seg_off(dl_tree_t t, int64_t* seg_off) {
  if (!t || !seg_off) return fail(DL_E_ARG, "dl_tree_seg_off: null argument");
  std::memcpy(seg_off, t->seg_off.data(), t->seg_off.size() * sizeof(int64_t));
  return DL_OK;
}

DL_API int dl_tree_bucket_range(dl_tree_t t, int32_t b, int64_t* begin, int64_t* end) {
  if (!t || !begin || !end) return fail(DL_E_ARG, "dl_tree_bucket_range: null argument");
  const int32_t nb = int32_t(t->bounds.size()) - 1;
  if (b == DL_ALL_BUCKETS) {
    *begin = 0;
    *end = t->total;
    return DL_OK;
  }
  if (b < 0 || b >= nb) return fail(DL_E_ARG, "dl_tree_bucket_range: bucket %d of %d", b, nb);
  *begin = t->seg_off[t->bounds[b]];
  *end = t->seg_off[t->bounds[b + 1]];  // next bucket's start, or seg_off[n] = the tree's end
  return DL_OK;
}

DL_API int dl_tree_bucket_chunks(dl_tree_t t, int32_t b, int32_t* c0, int32_t* c1) {
  if (!t || !c0 || !c1) return fail(DL_E_ARG, "dl_tree_bucket_chunks: null argument");
  const int32_t nb = int32_t(t->bounds.size()) - 1;
  if (b == DL_ALL_BUCKETS) {
    *c0 = 0;
    *c1 = int32_t(t->chunks.size());
    return DL_OK;
  }
  if (b < 0 || b >= nb) return fail(DL_E_ARG, "dl_tree_bucket_chunks: bucket %d of %d", b, nb);
  *c0 = t->bkt_chunk[b];
  *c1 = t->bkt_chunk[b + 1];
  return DL_OK;
}

DL_API int dl_tree_tune(dl_tree_t t, int32_t max_blocks, int32_t flags) {
  if (!t || max_blocks < 0) return fail(DL_E_ARG, "dl_tree_tune: bad argument");
  if (flags != DL_TUNE_AUTO &&
      (flags & ~(DL_TUNE_NT_LOADS | DL_TUNE_NT_STORES | DL_TUNE_WT_STORES | DL_TUNE_PAIRS)))
    return fail(DL_E_ARG, "dl_tree_tune: unknown flags 0x%x", flags);
#ifndef DL_TUNING
  // the product build instantiates the AUTO policies only: NT loads, plain or NT stores
  if (flags != DL_TUNE_AUTO &&
      (!(flags & DL_TUNE_NT_LOADS) || (flags & (DL_TUNE_WT_STORES | DL_TUNE_PAIRS))))
    return fail(DL_E_ARG,
                "dl_tree_tune: flags 0x%x need the tuning build (make TUNING=1): the product "
                "library has NT loads with plain or NT stores only", flags);
#endif
  t->grid = max_blocks;
  t->flags = flags;
  return DL_OK;
}

DL_API int dl_tuning_build(void) {
#ifdef DL_TUNING
  return 1;
#else
  return 0;
#endif
}

DL_API int dl_tree_bind(dl_tree_t t, int32_t slot, const uint64_t* ptrs, int32_t n,
                        dl_stream_t stream) {
  if (!t) return fail(DL_E_ARG, "dl_tree_bind: null tree");
  if (slot < 0 || slot >= DL_MAX_SLOTS) return fail(DL_E_ARG, "dl_tree_bind: slot %d", slot);
  if (n != t->nseg) return fail(DL_E_ARG, "dl_tree_bind: %d pointers for %d tensors", n, t->nseg);
  if (n > 0 && !ptrs) return fail(DL_E_ARG, "dl_tree_bind: null pointer array");
  for (int32_t i = 0; i < n; ++i) {
    if (ptrs[i] == 0 && t->numel[i] > 0)
      return fail(DL_E_ARG, "dl_tree_bind: null address for tensor %d", i);
    if (ptrs[i] & 3u) return fail(DL_E_ALIGN, "dl_tree_bind: tensor %d not 4-B aligned", i);
  }
  const size_t nch = t->chunks.size();
  if (nch == 0) {
    t->bound[slot] = 1;
    return DL_OK;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  // Stream-ordered and host-asynchronous: the n tensor addresses go into the next staging
  // slot of the ring (waiting only if that slot's previous upload -- kStageRing binds ago --
  // has not landed), one n-entry copy to the device, then dl_resolve_chunks expands them into
  // the slot's per-chunk address table. Kernels queued earlier on `s` still read the previous
  // table; the rewrite is ordered behind them.
  const int rc0 = slot_begin(t, slot, s, "dl_tree_bind");
  if (rc0) return rc0;
  const int k = t->stage_next;
  t->stage_next = (k + 1) % kStageRing;
  if (t->stage_used[k]) {  // normally long landed: a query, a wait only if it has not
    hipError_t q = hipEventQuery(t->stage_ev[k]);
    if (q == hipErrorNotReady)
      DL_HIP(hipEventSynchronize(t->stage_ev[k]), "dl_tree_bind(stage slot)");
    else if (q != hipSuccess)
      return hip_fail(q, "dl_tree_bind(stage slot)");
  }
  uint64_t* stage = t->h_stage + size_t(k) * size_t(n);
  for (int32_t i = 0; i < n; ++i) stage[i] = ptrs[i];
  uint64_t* segptr = t->d_segptr + size_t(slot) * size_t(n);
  DL_HIP(hipMemcpyAsync(segptr, stage, size_t(n) * sizeof(uint64_t), hipMemcpyHostToDevice, s),
         "dl_tree_bind(upload)");
  DL_HIP(hipEventRecord(t->stage_ev[k], s), "dl_tree_bind(event)");
  t->stage_used[k] = true;
  DL_HIP(dl::launch_resolve_chunks(t->d_chunks, t->d_loff, segptr, int32_t(nch),
                                   t->d_caddr + size_t(slot) * nch, s),
         "dl_tree_bind(resolve)");
  t->bound[slot] = 1;
  return slot_end(t, slot, s, "dl_tree_bind");
}

}  // extern "C"

namespace {

// per-kernel launch policy under DL_TUNE_AUTO (tools/sweep.py on T125 / T1.3B)
constexpr int32_t kAutoDelta = DL_TUNE_NT_LOADS;
constexpr int32_t kAutoOther = DL_TUNE_NT_LOADS;
// int8 encoder: its one 16-B payload store per lane non-temporal (tools/q8_layout.hip)
constexpr int32_t kAutoDeltaQ8 = DL_TUNE_NT_LOADS | DL_TUNE_NT_STORES;
// The two producers (dl_delta_pack, dl_gather) store plainly below 2^28 elements: the bucket
// they write is read next by RCCL or the unpack, from the Infinity Cache -- timed together with
// the consumer and charged with the write-back, plain is 4.5-7 % faster than NT on T125
// (tools/cold_sweep.py --what pipe --flushed, profiles/r03_pipe_flushed_t125.json). Over more
// than 2^28 elements (1 GiB of fp32, four times the Infinity Cache) the output cannot stay
// cached, so they store non-temporally (dl_scatter and dl_unpack_avg also take two chunks per
// workgroup there: 6 % faster flushed, profiles/r03_cold_sweep_flushed_t13b.json).
constexpr int32_t kBigLaunchChunks = (1 << 28) / DL_CHUNK_ELEMS;
constexpr int32_t kAutoUnpackSgd = DL_TUNE_NT_LOADS | DL_TUNE_NT_STORES;
// Kernels whose output no kernel re-reads next (dl_scatter: the inner params; dl_unpack_avg:
// gradients; dl_unpack_sgd_q8: θ, momentum, inner) store non-temporally at every size. Round 2
// chose plain stores below 2^28 elements for the first two and write-through (sc1) for the int8
// unpack from a cold timing whose end event did not wait for the lines a launch leaves dirty in
// the Infinity Cache. Charged with that write-back (tools/cold_sweep.py --flushed,
// profiles/r03_cold_sweep_flushed_t125.json): NT stores are 8 % faster than plain for dl_scatter
// and dl_unpack_avg and 2.5 % faster than write-through for dl_unpack_sgd_q8 on T125-size
// launches, equal over a whole T1.3B tree. The product library has no write-through stores.
constexpr int32_t kAutoNT = DL_TUNE_NT_LOADS | DL_TUNE_NT_STORES;
enum class Big { keep, nt_stores, nt_stores_2, two_chunks };
// dl_delta_pack / dl_gather with two chunks per workgroup (DL_TUNE_PAIRS, tuning build only):
// measured slower (dl_kernels.hip), so never part of AUTO
constexpr bool kAutoPairs = false;

int make_launch(dl_tree_t t, int32_t b, dl_stream_t s, dl::Launch* L, const char* who,
                int32_t auto_flags = kAutoOther, Big big = Big::keep) {
  if (!t) return fail(DL_E_ARG, "%s: null tree", who);
  const int32_t nb = int32_t(t->bounds.size()) - 1;
  if (b == DL_ALL_BUCKETS) {
    L->c0 = 0;
    L->c1 = int32_t(t->chunks.size());
  } else if (b >= 0 && b < nb) {
    L->c0 = t->bkt_chunk[b];
    L->c1 = t->bkt_chunk[b + 1];
  } else {
    return fail(DL_E_ARG, "%s: bucket %d of %d", who, b, nb);
  }
  L->chunks = t->d_chunks;
  L->caddr = t->d_caddr;
  L->nchunk = int32_t(t->chunks.size());
  L->grid = t->grid;
  L->flags = t->flags == DL_TUNE_AUTO ? auto_flags : t->flags;
  L->pairs = (L->flags & DL_TUNE_PAIRS) != 0;
#ifdef DL_XCD_XLOG  // A/B builds (tools/store_order_ab.py): one mapping for every launch
  L->xlog = DL_XCD_XLOG;
#else
  // the dispatcher's interleave: runs of B chunks per XCD change the headline kernel's time by
  // -3.4 ... +2.0 % depending on the box (profiles/r06_store_order_ab_*)
  L->xlog = 0;
#endif
  if (t->flags == DL_TUNE_AUTO && big != Big::keep && L->c1 - L->c0 >= kBigLaunchChunks) {
    L->flags |= DL_TUNE_NT_STORES;
    if ((big == Big::nt_stores_2 || big == Big::two_chunks) && L->grid == 0)
      L->grid = (L->c1 - L->c0 + 1) / 2;
  }
  L->stream = static_cast<hipStream_t>(s);
  return DL_OK;
}

int check_slot(dl_tree_t t, int32_t slot, const char* who, bool optional = false) {
  if (optional && slot < 0) return DL_OK;
  if (slot < 0 || slot >= DL_MAX_SLOTS) return fail(DL_E_ARG, "%s: slot %d", who, slot);
  if (!t->bound[slot]) return fail(DL_E_STATE, "%s: slot %d not bound", who, slot);
  return DL_OK;
}

int check_packed(const void* p, const char* who, const char* what) {
  if (!p) return fail(DL_E_ARG, "%s: %s is null", who, what);
  if (!dl::aligned16_host(p)) return fail(DL_E_ALIGN, "%s: %s not 16-B aligned", who, what);
  return DL_OK;
}

int check_dtype(int32_t d, const char* who) {
  if (d != DL_F32 && d != DL_BF16) return fail(DL_E_ARG, "%s: wire dtype %d", who, d);
  return DL_OK;
}

#define DL_TRY(x)         \
  do {                    \
    int rc_ = (x);        \
    if (rc_) return rc_;  \
  } while (0)

}  // namespace

extern "C" {

DL_API int dl_delta_pack(dl_tree_t t, int32_t b, int32_t inner_slot, const float* outer,
                         void* wire, int32_t wire_dtype, dl_stream_t s) {
  dl::Launch L;
  DL_TRY(make_launch(t, b, s, &L, "dl_delta_pack", kAutoDelta | (kAutoPairs ? DL_TUNE_PAIRS : 0),
                     Big::nt_stores));
  DL_TRY(check_slot(t, inner_slot, "dl_delta_pack"));
  DL_TRY(check_packed(outer, "dl_delta_pack", "outer"));
  DL_TRY(check_packed(wire, "dl_delta_pack", "wire"));
  DL_TRY(check_dtype(wire_dtype, "dl_delta_pack"));
  DL_TRY(slot_begin(t, inner_slot, L.stream, "dl_delta_pack"));
  hipError_t e = dl::launch_delta_pack(L, inner_slot, outer, wire, wire_dtype);
  return e == hipSuccess ? slot_end(t, inner_slot, L.stream, "dl_delta_pack") : hip_fail(e, "dl_delta_pack");
}

DL_API int dl_unpack_avg(dl_tree_t t, int32_t b, const void* wire, int32_t wire_dtype,
                         int32_t divisor, int32_t dst_slot, float* dst_packed, dl_stream_t s) {
  dl::Launch L;
  DL_TRY(make_launch(t, b, s, &L, "dl_unpack_avg", kAutoNT, Big::two_chunks));
  DL_TRY(check_packed(wire, "dl_unpack_avg", "wire"));
  DL_TRY(check_dtype(wire_dtype, "dl_unpack_avg"));
  if (divisor < 1) return fail(DL_E_ARG, "dl_unpack_avg: divisor %d", divisor);
  if (dst_slot >= 0)
    DL_TRY(check_slot(t, dst_slot, "dl_unpack_avg"));
  else
    DL_TRY(check_packed(dst_packed, "dl_unpack_avg", "dst_packed"));
  DL_TRY(slot_begin(t, dst_slot, L.stream, "dl_unpack_avg"));
  hipError_t e = dl::launch_unpack_avg(L, wire, wire_dtype, divisor, dst_slot, dst_packed);
  return e == hipSuccess ? slot_end(t, dst_slot, L.stream, "dl_unpack_avg") : hip_fail(e, "dl_unpack_avg");
}

DL_API int dl_unpack_sgd(dl_tree_t t, int32_t b, const void* wire, int32_t wire_dtype,
                         int32_t divisor, float* outer, float* mom, float lr, float momentum,
                         int32_t nesterov, int32_t first_step, int32_t inner_slot,
                         dl_stream_t s) {
  dl::Launch L;
  DL_TRY(make_launch(t, b, s, &L, "dl_unpack_sgd", kAutoUnpackSgd));
  DL_TRY(check_packed(wire, "dl_unpack_sgd", "wire"));
  DL_TRY(check_dtype(wire_dtype, "dl_unpack_sgd"));
  DL_TRY(check_packed(outer, "dl_unpack_sgd", "outer"));
  if (momentum != 0.f) DL_TRY(check_packed(mom, "dl_unpack_sgd", "momentum"));
  DL_TRY(check_slot(t, inner_slot, "dl_unpack_sgd", true));
  if (divisor < 1) return fail(DL_E_ARG, "dl_unpack_sgd: divisor %d", divisor);
  if (nesterov && momentum == 0.f)
    return fail(DL_E_ARG, "dl_unpack_sgd: Nesterov momentum requires a momentum");
  dl::SgdArgs a{-lr, momentum, nesterov ? 1 : 0, first_step ? 1 : 0};
  DL_TRY(slot_begin(t, inner_slot, L.stream, "dl_unpack_sgd"));
  hipError_t e = dl::launch_unpack_sgd(L, wire, wire_dtype, divisor, outer, mom, a, inner_slot);
  return e == hipSuccess ? slot_end(t, inner_slot, L.stream, "dl_unpack_sgd") : hip_fail(e, "dl_unpack_sgd");
}

DL_API int dl_delta_sgd(dl_tree_t t, int32_t b, int32_t inner_slot, float* outer, float* mom,
                        float lr, float momentum, int32_t nesterov, int32_t first_step,
                        dl_stream_t s) {
  dl::Launch L;
  DL_TRY(make_launch(t, b, s, &L, "dl_delta_sgd", kAutoUnpackSgd));
  DL_TRY(check_slot(t, inner_slot, "dl_delta_sgd"));
  DL_TRY(check_packed(outer, "dl_delta_sgd", "outer"));
  if (momentum != 0.f) DL_TRY(check_packed(mom, "dl_delta_sgd", "momentum"));
  if (nesterov && momentum == 0.f)
    return fail(DL_E_ARG, "dl_delta_sgd: Nesterov momentum requires a momentum");
  dl::SgdArgs a{-lr, momentum, nesterov ? 1 : 0, first_step ? 1 : 0};
  DL_TRY(slot_begin(t, inner_slot, L.stream, "dl_delta_sgd"));
  hipError_t e = dl::launch_delta_sgd(L, inner_slot, outer, mom, a);
  return e == hipSuccess ? slot_end(t, inner_slot, L.stream, "dl_delta_sgd") : hip_fail(e, "dl_delta_sgd");
}

DL_API int dl_delta_pack_sgd(dl_tree_t t, int32_t b, int32_t inner_slot, float* outer, void* wire,
                             int32_t wire_dtype, float* mom, float lr, float momentum,
                             int32_t nesterov, int32_t first_step, dl_stream_t s) {
  dl::Launch L;
  DL_TRY(make_launch(t, b, s, &L, "dl_delta_pack_sgd", kAutoUnpackSgd));
  DL_TRY(check_slot(t, inner_slot, "dl_delta_pack_sgd"));
  DL_TRY(check_packed(outer, "dl_delta_pack_sgd", "outer"));
  DL_TRY(check_packed(wire, "dl_delta_pack_sgd", "wire"));
  DL_TRY(check_dtype(wire_dtype, "dl_delta_pack_sgd"));
  if (momentum != 0.f) DL_TRY(check_packed(mom, "dl_delta_pack_sgd", "momentum"));
  if (nesterov && momentum == 0.f)
    return fail(DL_E_ARG, "dl_delta_pack_sgd: Nesterov momentum requires a momentum");
  dl::SgdArgs a{-lr, momentum, nesterov ? 1 : 0, first_step ? 1 : 0};
  DL_TRY(slot_begin(t, inner_slot, L.stream, "dl_delta_pack_sgd"));
  hipError_t e = dl::launch_delta_pack_sgd(L, inner_slot, outer, wire, wire_dtype, mom, a);
  return e == hipSuccess ? slot_end(t, inner_slot, L.stream, "dl_delta_pack_sgd") : hip_fail(e, "dl_delta_pack_sgd");
}

// a2 -> (one peer: the exchange is the identity, src/comm.py:118-119) -> a3-a5, cache-blocked:
// the tree is walked in tiles of tile_chunks chunks and each tile runs dl_delta_pack then
// dl_unpack_sgd, so the wire and θ bytes the pack just touched are re-read by the unpack from
// the 256 MiB Infinity Cache instead of HBM. Elementwise work: bit-identical to the two
// whole-range launches for every tile size.
DL_API int dl_pack_sgd_tiled(dl_tree_t t, int32_t b, int32_t inner_slot, float* outer, void* wire,
                             int32_t wire_dtype, float* mom, float lr, float momentum,
                             int32_t nesterov, int32_t first_step, int32_t tile_chunks,
                             dl_stream_t s) {
  dl::Launch P, U;
  DL_TRY(make_launch(t, b, s, &P, "dl_pack_sgd_tiled", kAutoDelta));
  DL_TRY(make_launch(t, b, s, &U, "dl_pack_sgd_tiled", kAutoUnpackSgd));
  DL_TRY(check_slot(t, inner_slot, "dl_pack_sgd_tiled"));
  DL_TRY(check_packed(outer, "dl_pack_sgd_tiled", "outer"));
  DL_TRY(check_packed(wire, "dl_pack_sgd_tiled", "wire"));
  DL_TRY(check_dtype(wire_dtype, "dl_pack_sgd_tiled"));
  if (momentum != 0.f) DL_TRY(check_packed(mom, "dl_pack_sgd_tiled", "momentum"));
  if (nesterov && momentum == 0.f)
    return fail(DL_E_ARG, "dl_pack_sgd_tiled: Nesterov momentum requires a momentum");
  if (tile_chunks < 0) return fail(DL_E_ARG, "dl_pack_sgd_tiled: tile_chunks %d", tile_chunks);
  const dl::SgdArgs a{-lr, momentum, nesterov ? 1 : 0, first_step ? 1 : 0};
  DL_TRY(slot_begin(t, inner_slot, P.stream, "dl_pack_sgd_tiled"));
  const int32_t c0 = P.c0, c1 = P.c1;
  const int32_t step = tile_chunks > 0 ? tile_chunks : (c1 - c0 > 0 ? c1 - c0 : 1);
  for (int32_t c = c0; c < c1; c += step) {
    const int32_t e = c1 - c < step ? c1 : c + step;
    P.c0 = U.c0 = c;
    P.c1 = U.c1 = e;
    hipError_t err = dl::launch_delta_pack(P, inner_slot, outer, wire, wire_dtype);
    if (err == hipSuccess)
      err = dl::launch_unpack_sgd(U, wire, wire_dtype, 1, outer, mom, a, inner_slot);
    if (err != hipSuccess) return hip_fail(err, "dl_pack_sgd_tiled");
  }
  return slot_end(t, inner_slot, P.stream, "dl_pack_sgd_tiled");
}

DL_API int dl_shard_sgd(const void* wire, int32_t wire_dtype, int32_t divisor, float* outer,
                        float* mom, int64_t n, float lr, float momentum, int32_t nesterov,
                        int32_t first_step, dl_stream_t s) {
  if (n < 0) return fail(DL_E_ARG, "dl_shard_sgd: n %lld", (long long)n);
  if (n == 0) return DL_OK;
  DL_TRY(check_packed(wire, "dl_shard_sgd", "wire"));
  DL_TRY(check_dtype(wire_dtype, "dl_shard_sgd"));
  DL_TRY(check_packed(outer, "dl_shard_sgd", "outer"));
  if (momentum != 0.f) DL_TRY(check_packed(mom, "dl_shard_sgd", "momentum"));
  if (divisor < 1) return fail(DL_E_ARG, "dl_shard_sgd: divisor %d", divisor);
  if (nesterov && momentum == 0.f)
    return fail(DL_E_ARG, "dl_shard_sgd: Nesterov momentum requires a momentum");
  if ((n + DL_CHUNK_ELEMS - 1) / DL_CHUNK_ELEMS > INT32_MAX)
    return fail(DL_E_ARG, "dl_shard_sgd: shard too large");
  dl::SgdArgs a{-lr, momentum, nesterov ? 1 : 0, first_step ? 1 : 0};
  hipError_t e = dl::launch_shard_sgd(wire, wire_dtype, divisor, outer, mom, n, a,
                                      static_cast<hipStream_t>(s));
  return e == hipSuccess ? DL_OK : hip_fail(e, "dl_shard_sgd");
}

DL_API int dl_shard_reduce_sgd(const void* slices, int32_t wire_dtype, int32_t n_slices,
                               int64_t len, float* outer, float* mom, float lr, float momentum,
                               int32_t nesterov, int32_t first_step, dl_stream_t s) {
  if (len < 0 || len % 4 != 0)
    return fail(DL_E_ARG, "dl_shard_reduce_sgd: len %lld (a multiple of 4)", (long long)len);
  if (n_slices < 1) return fail(DL_E_ARG, "dl_shard_reduce_sgd: n_slices %d", n_slices);
  if (len == 0) return DL_OK;
  DL_TRY(check_packed(slices, "dl_shard_reduce_sgd", "slices"));
  DL_TRY(check_dtype(wire_dtype, "dl_shard_reduce_sgd"));
  DL_TRY(check_packed(outer, "dl_shard_reduce_sgd", "outer"));
  if (momentum != 0.f) DL_TRY(check_packed(mom, "dl_shard_reduce_sgd", "momentum"));
  if (nesterov && momentum == 0.f)
    return fail(DL_E_ARG, "dl_shard_reduce_sgd: Nesterov momentum requires a momentum");
  dl::SgdArgs a{-lr, momentum, nesterov ? 1 : 0, first_step ? 1 : 0};
  hipError_t e = dl::launch_slices_sgd(slices, wire_dtype, n_slices, len, outer, mom, a,
                                       static_cast<hipStream_t>(s));
  return e == hipSuccess ? DL_OK : hip_fail(e, "dl_shard_reduce_sgd");
}

DL_API int dl_shard_reduce_avg(const void* slices, int32_t wire_dtype, int32_t n_slices,
                               int64_t len, float* out, dl_stream_t s) {
  if (len < 0 || len % 4 != 0)
    return fail(DL_E_ARG, "dl_shard_reduce_avg: len %lld (a multiple of 4)", (long long)len);
  if (n_slices < 1) return fail(DL_E_ARG, "dl_shard_reduce_avg: n_slices %d", n_slices);
  if (len == 0) return DL_OK;
  DL_TRY(check_packed(slices, "dl_shard_reduce_avg", "slices"));
  DL_TRY(check_dtype(wire_dtype, "dl_shard_reduce_avg"));
  DL_TRY(check_packed(out, "dl_shard_reduce_avg", "out"));
  dl::SgdArgs a{0.f, 0.f, 0, 0};
  hipError_t e = dl::launch_slices_sgd(slices, wire_dtype, n_slices, len, out, nullptr, a,
                                       static_cast<hipStream_t>(s), true);
  return e == hipSuccess ? DL_OK : hip_fail(e, "dl_shard_reduce_avg");
}

DL_API int dl_ipc_handle(const void* ptr, void* handle, int64_t* offset) {
  if (!ptr || !handle || !offset) return fail(DL_E_ARG, "dl_ipc_handle: null argument");
  void* base = nullptr;
  size_t size = 0;
  DL_HIP(hipMemGetAddressRange(&base, &size, const_cast<void*>(ptr)), "dl_ipc_handle");
  hipIpcMemHandle_t h;
  DL_HIP(hipIpcGetMemHandle(&h, base), "dl_ipc_handle");
  static_assert(sizeof(h) <= DL_IPC_HANDLE_BYTES, "IPC handle size");
  std::memset(handle, 0, DL_IPC_HANDLE_BYTES);
  std::memcpy(handle, &h, sizeof h);
  *offset = static_cast<const char*>(ptr) - static_cast<const char*>(base);
  return DL_OK;
}

DL_API int dl_ipc_open(const void* handle, void** base) {
  if (!handle || !base) return fail(DL_E_ARG, "dl_ipc_open: null argument");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof h);
  DL_HIP(hipIpcOpenMemHandle(base, h, hipIpcMemLazyEnablePeerAccess), "dl_ipc_open");
  return DL_OK;
}

DL_API int dl_ipc_close(void* base) {
  if (!base) return DL_OK;
  DL_HIP(hipIpcCloseMemHandle(base), "dl_ipc_close");
  return DL_OK;
}

DL_API int dl_can_access_peer(int32_t device, int32_t peer, int32_t* can) {
  if (!can) return fail(DL_E_ARG, "dl_can_access_peer: null argument");
  if (device == peer) {
    *can = 1;
    return DL_OK;
  }
  int c = 0;
  DL_HIP(hipDeviceCanAccessPeer(&c, device, peer), "dl_can_access_peer");
  *can = c;
  return DL_OK;
}

DL_API int dl_enable_peer_access(int32_t peer) {
  hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();  // clear the sticky "already enabled"
    return DL_OK;
  }
  return e == hipSuccess ? DL_OK : hip_fail(e, "dl_enable_peer_access");
}

DL_API int dl_sys_fence(dl_stream_t s) {
  hipError_t e = dl::launch_sys_fence(nullptr, nullptr, static_cast<hipStream_t>(s));
  return e == hipSuccess ? DL_OK : hip_fail(e, "dl_sys_fence");
}

DL_API int dl_sys_fence_census(uint32_t* xcc, int32_t cap, int32_t* grid, dl_stream_t s) {
  if (!xcc || !grid) return fail(DL_E_ARG, "dl_sys_fence_census: null argument");
  int dev = 0, n = 0;
  DL_HIP(hipGetDevice(&dev), "dl_sys_fence_census");
  DL_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev),
         "dl_sys_fence_census");
  if (cap < n)
    return fail(DL_E_ARG, "dl_sys_fence_census: %d entries for %d workgroups", cap, n);
  hipError_t e = dl::launch_sys_fence(xcc, grid, static_cast<hipStream_t>(s));
  return e == hipSuccess ? DL_OK : hip_fail(e, "dl_sys_fence_census");
}

DL_API int dl_copy(const void* src, void* dst, int64_t bytes, int32_t flags, dl_stream_t s) {
  if (bytes < 0 || bytes % 16) return fail(DL_E_ARG, "dl_copy: bytes %lld (multiple of 16)",
                                           (long long)bytes);
  if (flags & ~(DL_TUNE_NT_LOADS | DL_COPY_WIDE | DL_COPY_READ | DL_COPY_WRITE | (3 << 8)))
    return fail(DL_E_ARG, "dl_copy: flags 0x%x", flags);
  const bool rd = (flags & DL_COPY_READ) != 0, wr = (flags & DL_COPY_WRITE) != 0;
  const bool nt = (flags & DL_TUNE_NT_LOADS) != 0;
  if (rd && wr) return fail(DL_E_ARG, "dl_copy: DL_COPY_READ and DL_COPY_WRITE together");
  if (rd || wr) {
    if (flags & DL_COPY_WIDE) return fail(DL_E_ARG, "dl_copy: DL_COPY_WIDE with a probe");
    const int streams = ((flags >> 8) & 3) + 1;
    if (bytes % (16 * streams))
      return fail(DL_E_ARG, "dl_copy: bytes %lld not a multiple of 16 x %d streams",
                  (long long)bytes, streams);
    if (bytes == 0) return DL_OK;
    if (rd) DL_TRY(check_packed(src, "dl_copy", "src"));
    else DL_TRY(check_packed(dst, "dl_copy", "dst"));
    hipError_t e = dl::launch_probe(wr, streams, src, dst, bytes / 16 / streams, nt,
                                    static_cast<hipStream_t>(s));
    return e == hipSuccess ? DL_OK : hip_fail(e, "dl_copy");
  }
  if (flags & (3 << 8)) return fail(DL_E_ARG, "dl_copy: DL_COPY_STREAMS needs a probe");
  if (bytes == 0) return DL_OK;
  DL_TRY(check_packed(src, "dl_copy", "src"));
  DL_TRY(check_packed(dst, "dl_copy", "dst"));
  hipError_t e = dl::launch_copy(src, dst, bytes / 16, nt, (flags & DL_COPY_WIDE) != 0,
                                 static_cast<hipStream_t>(s));
  return e == hipSuccess ? DL_OK : hip_fail(e, "dl_copy");
}

DL_API int dl_peer_gather(const uint64_t* srcs, int32_t nsrc, int64_t bytes_each, void* dst,
                          dl_stream_t s) {
  if (!srcs || !dst) return fail(DL_E_ARG, "dl_peer_gather: null argument");
  if (nsrc < 1 || nsrc > dl::kMaxPeers)
    return fail(DL_E_ARG, "dl_peer_gather: %d sources (1..%d)", nsrc, dl::kMaxPeers);
  if (bytes_each < 0 || bytes_each % 16 || bytes_each / 16 > INT32_MAX - (1 << 24))
    return fail(DL_E_ARG, "dl_peer_gather: bytes_each %lld (multiple of 16, < 32 GiB)",
                (long long)bytes_each);
  DL_TRY(check_packed(dst, "dl_peer_gather", "dst"));
  dl::XgmiPeers p{};
  for (int32_t i = 0; i < nsrc; ++i) {
    p.wire[i] = reinterpret_cast<const float*>(srcs[i]);
    DL_TRY(check_packed(p.wire[i], "dl_peer_gather", "source"));
  }
  hipError_t e = dl::launch_peer_gather(p, nsrc, int32_t(bytes_each / 16),
                                        static_cast<float*>(dst), static_cast<hipStream_t>(s));
  return e == hipSuccess ? DL_OK : hip_fail(e, "dl_peer_gather");
}

}  // extern "C"

namespace {
int xgmi_step(const char* who, bool delta, const uint64_t* srcs, const uint64_t* thetas,
              int32_t n, int32_t rank, int64_t lo, int64_t len, float* mom, float lr,
              float momentum, int32_t nesterov, int32_t first_step, dl_stream_t s) {
  if (!srcs || !thetas) return fail(DL_E_ARG, "%s: null peer table", who);
  if (n < 1 || n > dl::kMaxPeers || rank < 0 || rank >= n)
    return fail(DL_E_ARG, "%s: rank %d of %d (1..%d peers)", who, rank, n, dl::kMaxPeers);
  if (lo < 0 || len < 0 || lo % 4 || len % 4)
    return fail(DL_E_ARG, "%s: shard [%lld, +%lld) not a multiple of 4", who, (long long)lo,
                (long long)len);
  if (momentum != 0.f) DL_TRY(check_packed(mom, who, "momentum"));
  if (nesterov && momentum == 0.f)
    return fail(DL_E_ARG, "%s: Nesterov momentum requires a momentum", who);
  dl::XgmiPeers p{};
  for (int32_t q = 0; q < n; ++q) {
    p.wire[q] = reinterpret_cast<const float*>(srcs[q]);
    p.theta[q] = reinterpret_cast<float*>(thetas[q]);
    DL_TRY(check_packed(p.wire[q], who, delta ? "inner" : "wire"));
    DL_TRY(check_packed(p.theta[q], who, "theta"));
  }
  dl::SgdArgs a{-lr, momentum, nesterov ? 1 : 0, first_step ? 1 : 0};
  hipError_t e = dl::launch_xgmi_reduce_sgd(p, n, rank, lo, len, mom, a, delta,
                                            static_cast<hipStream_t>(s));
  return e == hipSuccess ? DL_OK : hip_fail(e, who);
}
}  // namespace

extern "C" {

DL_API int dl_xgmi_reduce_sgd(const uint64_t* wires, const uint64_t* thetas, int32_t n,
                              int32_t rank, int64_t lo, int64_t len, float* mom, float lr,
                              float momentum, int32_t nesterov, int32_t first_step,
                              dl_stream_t s) {
  return xgmi_step("dl_xgmi_reduce_sgd", false, wires, thetas, n, rank, lo, len, mom, lr,
                   momentum, nesterov, first_step, s);
}

DL_API int dl_xgmi_delta_sgd(const uint64_t* inners, const uint64_t* thetas, int32_t n,
                             int32_t rank, int64_t lo, int64_t len, float* mom, float lr,
                             float momentum, int32_t nesterov, int32_t first_step,
                             dl_stream_t s) {
  return xgmi_step("dl_xgmi_delta_sgd", true, inners, thetas, n, rank, lo, len, mom, lr,
                   momentum, nesterov, first_step, s);
}

DL_API int dl_delta_q8(dl_tree_t t, int32_t b, int32_t inner_slot, const float* outer,
                       void* slots, dl_stream_t s) {
  dl::Launch L;
  DL_TRY(make_launch(t, b, s, &L, "dl_delta_q8", kAutoDeltaQ8));
  DL_TRY(check_slot(t, inner_slot, "dl_delta_q8"));
  DL_TRY(check_packed(outer, "dl_delta_q8", "outer"));
  DL_TRY(check_packed(slots, "dl_delta_q8", "slots"));
  DL_TRY(slot_begin(t, inner_slot, L.stream, "dl_delta_q8"));
  hipError_t e = dl::launch_delta_q8(L, inner_slot, outer, static_cast<uint8_t*>(slots));
  return e == hipSuccess ? slot_end(t, inner_slot, L.stream, "dl_delta_q8") : hip_fail(e, "dl_delta_q8");
}

DL_API int dl_q8_reduce(const void* recv, int32_t n, int32_t m, int32_t divisor, void* out,
                        dl_stream_t s) {
  if (n < 1 || m < 0 || divisor < 1) return fail(DL_E_ARG, "dl_q8_reduce: n %d m %d div %d", n, m, divisor);
  DL_TRY(check_packed(recv, "dl_q8_reduce", "recv"));
  DL_TRY(check_packed(out, "dl_q8_reduce", "out"));
  if (recv == out && n != 1) return fail(DL_E_ARG, "dl_q8_reduce: in place needs n_peers == 1");
  hipError_t e = dl::launch_q8_reduce(static_cast<const uint8_t*>(recv), n, m, divisor,
                                      static_cast<uint8_t*>(out), static_cast<hipStream_t>(s));
  return e == hipSuccess ? DL_OK : hip_fail(e, "dl_q8_reduce");
}

DL_API int dl_unpack_sgd_q8(dl_tree_t t, int32_t b, const void* slots, float* outer, float* mom,
                            float lr, float momentum, int32_t nesterov, int32_t first_step,
                            int32_t inner_slot, dl_stream_t s) {
  dl::Launch L;
  DL_TRY(make_launch(t, b, s, &L, "dl_unpack_sgd_q8", kAutoNT));
  DL_TRY(check_packed(slots, "dl_unpack_sgd_q8", "slots"));
  DL_TRY(check_packed(outer, "dl_unpack_sgd_q8", "outer"));
  if (momentum != 0.f) DL_TRY(check_packed(mom, "dl_unpack_sgd_q8", "momentum"));
  DL_TRY(check_slot(t, inner_slot, "dl_unpack_sgd_q8", true));
  if (nesterov && momentum == 0.f)
    return fail(DL_E_ARG, "dl_unpack_sgd_q8: Nesterov momentum requires a momentum");
  dl::SgdArgs a{-lr, momentum, nesterov ? 1 : 0, first_step ? 1 : 0};
  DL_TRY(slot_begin(t, inner_slot, L.stream, "dl_unpack_sgd_q8"));
  hipError_t e = dl::launch_unpack_sgd_q8(L, static_cast<const uint8_t*>(slots), outer, mom, a,
                                          inner_slot);
  return e == hipSuccess ? slot_end(t, inner_slot, L.stream, "dl_unpack_sgd_q8")
                         : hip_fail(e, "dl_unpack_sgd_q8");
}

DL_API int dl_gather(dl_tree_t t, int32_t b, int32_t src_slot, void* packed, int32_t dtype,
                     dl_stream_t s) {
  dl::Launch L;
  DL_TRY(make_launch(t, b, s, &L, "dl_gather", kAutoOther | (kAutoPairs ? DL_TUNE_PAIRS : 0),
                     Big::nt_stores));
  DL_TRY(check_slot(t, src_slot, "dl_gather"));
  DL_TRY(check_packed(packed, "dl_gather", "packed"));
  DL_TRY(check_dtype(dtype, "dl_gather"));
  DL_TRY(slot_begin(t, src_slot, L.stream, "dl_gather"));
  hipError_t e = dl::launch_gather(L, src_slot, packed, dtype);
  return e == hipSuccess ? slot_end(t, src_slot, L.stream, "dl_gather") : hip_fail(e, "dl_gather");
}

DL_API int dl_scatter(dl_tree_t t, int32_t b, const float* packed, int32_t dst_slot,
                      dl_stream_t s) {
  dl::Launch L;
  DL_TRY(make_launch(t, b, s, &L, "dl_scatter", kAutoNT, Big::two_chunks));
  DL_TRY(check_slot(t, dst_slot, "dl_scatter"));
  DL_TRY(check_packed(packed, "dl_scatter", "packed"));
  DL_TRY(slot_begin(t, dst_slot, L.stream, "dl_scatter"));
  hipError_t e = dl::launch_scatter(L, packed, dst_slot);
  return e == hipSuccess ? slot_end(t, dst_slot, L.stream, "dl_scatter") : hip_fail(e, "dl_scatter");
}

DL_API int dl_serialize(const void* src, int32_t src_dtype, int64_t numel, float meta0,
                        float meta1, float* out, dl_stream_t s) {
  if (!src || !out) return fail(DL_E_ARG, "dl_serialize: null pointer");
  if (numel < 2) return fail(DL_E_ARG, "dl_serialize: numel %lld < 2", (long long)numel);
  if (src_dtype != DL_F32 && src_dtype != DL_BF16 && src_dtype != DL_F16)
    return fail(DL_E_ARG, "dl_serialize: dtype %d", src_dtype);
  hipError_t e = dl::launch_serialize(src, src_dtype, numel, meta0, meta1, out,
                                      static_cast<hipStream_t>(s));
  return e == hipSuccess ? DL_OK : hip_fail(e, "dl_serialize");
}

DL_API int dl_serialize_f64(const double* src, int64_t numel, float meta0, float meta1,
                            double* out, dl_stream_t s) {
  if (!src || !out) return fail(DL_E_ARG, "dl_serialize_f64: null pointer");
  if (numel < 2) return fail(DL_E_ARG, "dl_serialize_f64: numel %lld < 2", (long long)numel);
  hipError_t e = dl::launch_serialize_f64(src, numel, meta0, meta1, out,
                                          static_cast<hipStream_t>(s));
  return e == hipSuccess ? DL_OK : hip_fail(e, "dl_serialize_f64");
}

DL_API int dl_fill_synth(float* dst, int64_t n, uint64_t seed, uint64_t stream_id, float base,
                         float scale, const float* add, dl_stream_t s) {
  if (n < 0 || (n > 0 && !dst)) return fail(DL_E_ARG, "dl_fill_synth: bad dst/n");
  if (stream_id >= (1ull << 24)) return fail(DL_E_ARG, "dl_fill_synth: stream_id >= 2^24");
  if (n >= (1ll << 40)) return fail(DL_E_ARG, "dl_fill_synth: n >= 2^40");
  hipError_t e = dl::launch_fill_synth(dst, n, seed, stream_id, base, scale, add,
                                       static_cast<hipStream_t>(s));
  return e == hipSuccess ? DL_OK : hip_fail(e, "dl_fill_synth");
}

DL_API int dl_spin(uint64_t ns, dl_stream_t s) {
  if (ns > 10000000000ull) return fail(DL_E_ARG, "dl_spin: %llu ns > 10 s", (unsigned long long)ns);
  hipError_t e = dl::launch_spin(ns, static_cast<hipStream_t>(s));
  return e == hipSuccess ? DL_OK : hip_fail(e, "dl_spin");
}

}  // extern "C"
