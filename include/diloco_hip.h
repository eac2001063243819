/*
 * diloco_hip.h — C-ABI of libdiloco_hip.so, the MI355X (gfx950) implementation of the DiLoCo
 * outer-step pseudo-gradient sync of mikasenghaas/diloco-swarm.
 *
 * The reference has no native code and no FFI: its hot path is per-parameter torch CPU ops
 * plus one gloo all_reduce per tensor. Each entry point below names the reference code it
 * replaces (paths relative to the reference repository root). The Python host layer
 * (diloco-swarm_amd/diloco_amd) binds these symbols with ctypes; see INTEGRATION.md.
 *
 * Conventions
 *   - Every function returns int: 0 = ok, <0 = DL_E_* argument/state error,
 *     >0 = the hipError_t passed through. dl_last_error() returns a thread-local message.
 *   - Pointers are plain device (or pinned host, where stated) addresses; no torch types.
 *   - Memory handed in is owned by the caller; the library owns only the tree handle's
 *     device tables (freed by dl_tree_destroy).
 *   - A "packed" buffer holds the tree's tensors back to back in parameters() order, each
 *     segment starting at a multiple of DL_ALIGN_ELEMS elements; padding is never written.
 *   - "bucket" selects one bucket of the plan; DL_ALL_BUCKETS (-1) selects the whole tree.
 *   - All kernels are stream-ordered on the hipStream_t passed in; no entry point
 *     synchronises the host with a stream (dl_tree_bind is asynchronous too).
 */
#ifndef DILOCO_HIP_H
#define DILOCO_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DL_API __attribute__((visibility("default")))

#define DL_ABI_VERSION 2
#define DL_ALIGN_ELEMS 64      /* segment start alignment in the packed space: 256 B of fp32 */
#define DL_CHUNK_ELEMS 4096    /* work unit of every segment walker: 16 KiB of fp32 */
#define DL_ALL_BUCKETS (-1)
#define DL_MAX_SLOTS 4         /* per-tensor pointer tables per tree */
#define DL_Q8_SLOT_BYTES 4160  /* int8 wire: 64-B header (fp32 scale) + DL_CHUNK_ELEMS int8 */

/* wire / packed dtypes */
#define DL_F32 0
#define DL_BF16 1
#define DL_F16 2
#define DL_U8 3 /* bytes (int8 wire slots); collectives only */

/* errors (negative); positive codes are hipError_t */
#define DL_OK 0
#define DL_E_ARG (-1)
#define DL_E_STATE (-2)
#define DL_E_ALIGN (-3)
#define DL_E_RCCL (-4) /* an RCCL call failed; dl_last_error() has its message */

typedef struct dl_tree_s* dl_tree_t;
typedef void* dl_stream_t; /* hipStream_t */
typedef void* dl_comm_t;   /* ncclComm_t of the RCCL selected by dl_rccl_load */

/* ---- planner (host only; needs no GPU) -------------------------------------------------
 * Replaces the reference's implicit layout: the per-tensor loop over model.parameters()
 * in src/comm.py:120-123 and src/utils.py:220,225. Input: numel of each tensor in
 * parameters() order. Output: seg_off[n+1] (element offsets, each start aligned to
 * align_elems), bkt_bounds[n_bkt+1] (segment indices; greedy split at tensor boundaries so
 * a bucket's padded size stays <= cap_elems unless a single tensor exceeds it; cap_elems<=0
 * = one bucket). bkt_bounds must hold n+1 entries. Bit-exact contract with
 * oracle/diloco_oracle.c:or_plan_tables. */
DL_API int dl_plan_tables(const int64_t* numel, int32_t n, int64_t cap_elems, int32_t align_elems,
                          int64_t* seg_off, int64_t* bkt_bounds, int32_t* n_bkt);
/* Same rule with every bucket starting at a multiple of bucket_align_elems (a positive
 * multiple of align_elems) and seg_off[n] rounded up to it, so each bucket's range
 * [seg_off[bkt_bounds[b]], seg_off[bkt_bounds[b+1]]) splits into equal, aligned shards for a
 * reduce-scatter over n peers (bucket_align = DL_ALIGN_ELEMS * n). bucket_align ==
 * align_elems is dl_plan_tables. */
DL_API int dl_plan_tables_ex(const int64_t* numel, int32_t n, int64_t cap_elems,
                             int32_t align_elems, int64_t bucket_align_elems, int64_t* seg_off,
                             int64_t* bkt_bounds, int32_t* n_bkt);

/* ---- tree handle ------------------------------------------------------------------------
 * One parameter tree on the current device: planner tables + the chunk table + DL_MAX_SLOTS
 * per-tensor device pointer tables. Created once per model (src/utils.py:213-216
 * get_outer_model / src/comm.py:81 TrainingComm.__init__ are the natural creation points). */
DL_API int dl_tree_create(const int64_t* numel, int32_t n, int64_t cap_elems, dl_tree_t* out);
/* dl_tree_create with the dl_plan_tables_ex bucket alignment (the sharded outer step). */
DL_API int dl_tree_create_ex(const int64_t* numel, int32_t n, int64_t cap_elems,
                             int64_t bucket_align_elems, dl_tree_t* out);
DL_API int dl_tree_destroy(dl_tree_t tree);
DL_API int dl_tree_query(dl_tree_t tree, int64_t* total_elems, int32_t* n_seg, int32_t* n_bkt,
                         int32_t* n_chunk);
DL_API int dl_tree_bucket_range(dl_tree_t tree, int32_t bucket, int64_t* elem_begin,
                                int64_t* elem_end);
DL_API int dl_tree_seg_off(dl_tree_t tree, int64_t* seg_off /* n_seg+1 */);
/* Chunk index range [chunk_begin, chunk_end) of a bucket (DL_ALL_BUCKETS: the whole tree). */
DL_API int dl_tree_bucket_chunks(dl_tree_t tree, int32_t bucket, int32_t* chunk_begin,
                                 int32_t* chunk_end);
/* Upload the device addresses of the n_seg tensors of one slot (e.g. inner params, grads).
 * fp32 tensors, contiguous; a 16-B-misaligned address takes the scalar path. Stream-ordered
 * on `stream` and asynchronous for the host: the n_seg addresses are staged in a ring of
 * pinned slots and expanded into the slot's per-chunk table by a kernel, so rebinding grads
 * that torch reallocated (zero_grad(set_to_none=True) before every inner step,
 * src/train.py:164) costs no host synchronisation. Kernels queued on `stream` before the
 * call still see the previous table. A bind or kernel that uses a slot on another stream than
 * the slot's previous bind or kernel first waits for that one (an event per slot), so a
 * table is never rewritten under, or read before, work the caller did not order. */
DL_API int dl_tree_bind(dl_tree_t tree, int32_t slot, const uint64_t* dev_ptrs, int32_t n,
                        dl_stream_t stream);
/* Launch shape of every walker kernel on this tree: max_blocks caps the grid (0 = one
 * workgroup per chunk, the default); flags = DL_TUNE_AUTO (the default: the measured
 * per-kernel choice -- NT loads everywhere; NT stores in the SGD kernels, dl_scatter,
 * dl_unpack_avg and dl_unpack_sgd_q8, and in dl_delta_pack / dl_gather over launches of more
 * than 2^28 elements; plain stores for those two producers below that size, where the next
 * kernel or RCCL re-reads their output from the Infinity Cache) or DL_TUNE_NT_LOADS [|
 * DL_TUNE_NT_STORES] for every kernel. Plain loads, DL_TUNE_WT_STORES (write-through, sc1)
 * for every kernel and DL_TUNE_PAIRS exist only in the tuning build (make TUNING=1, dl_tuning_build() == 1);
 * the product library rejects them with DL_E_ARG. Results are identical for every setting;
 * only speed differs. */
#define DL_TUNE_NT_LOADS 1
#define DL_TUNE_NT_STORES 2
#define DL_TUNE_WT_STORES 8 /* write-through (sc1) stores; tuning build only */
/* tuning build only: two chunks per workgroup, both chunks' loads issued before the first
 * store, in the 2-read / 1-write kernels (dl_delta_pack, dl_gather; measured slower) */
#define DL_TUNE_PAIRS 16
#define DL_TUNE_AUTO (-1)
DL_API int dl_tree_tune(dl_tree_t tree, int32_t max_blocks, int32_t flags);
/* 1 in the tuning build (every load / store policy instantiated), 0 in the product library. */
DL_API int dl_tuning_build(void);

/* ---- hot-path kernels ----------------------------------------------------------------- */

/* a2: compute_pseudo_gradient, src/utils.py:218-221:
 *   wire[k] = outer_packed[k] - inner[seg][j]      (fp32 subtract; bf16 wire rounds RNE)
 * outer_packed: fp32 packed θ_outer; inner: slot `inner_slot`. 12 B/param (fp32 wire). */
DL_API int dl_delta_pack(dl_tree_t tree, int32_t bucket, int32_t inner_slot,
                         const float* outer_packed, void* wire, int32_t wire_dtype,
                         dl_stream_t stream);

/* a3 unpack: src/comm.py:122-123 `param.grad /= num_peers` after the SUM all-reduce:
 *   dst[seg][j] = wire[k] / divisor   (IEEE true division; divisor 1 = plain copy)
 * dst is slot `dst_slot` (per-tensor fp32) or, when dst_slot < 0, the packed fp32 buffer
 * dst_packed (may alias an fp32 wire). 8 B/param. */
DL_API int dl_unpack_avg(dl_tree_t tree, int32_t bucket, const void* wire, int32_t wire_dtype,
                         int32_t divisor, int32_t dst_slot, float* dst_packed,
                         dl_stream_t stream);

/* a3+a4+a5 fused: unpack the summed wire, average, outer SGD (torch.optim.SGD
 * _single_tensor_sgd as built by src/utils.py:62-63 and stepped at src/train.py:267),
 * then sync_inner_model (src/utils.py:223-226):
 *   g = wire/divisor; buf = first ? g : (buf*m) + g; u = nesterov ? fma(buf,m,g) : buf
 *   θ = fma(u, -lr, θ); inner[seg][j] = θ      (momentum==0: θ = fma(g,-lr,θ), no buf)
 * inner_slot < 0 skips the inner write. 24 B/param (20 on the first step). */
DL_API int dl_unpack_sgd(dl_tree_t tree, int32_t bucket, const void* wire, int32_t wire_dtype,
                         int32_t divisor, float* outer_packed, float* mom_packed, float lr,
                         float momentum, int32_t nesterov, int32_t first_step,
                         int32_t inner_slot, dl_stream_t stream);

/* a2+a4+a5 at ONE peer (src/comm.py:118-119 skips the all-reduce and the division):
 *   g = θ - inner[seg][j]; SGD as dl_unpack_sgd; θ and inner[seg][j] <- new θ
 * One pass, the delta stays in registers: 24 B/param (20 on the first step) instead of 36
 * for dl_delta_pack + dl_unpack_sgd; bit-identical results. */
DL_API int dl_delta_sgd(dl_tree_t tree, int32_t bucket, int32_t inner_slot, float* outer_packed,
                        float* mom_packed, float lr, float momentum, int32_t nesterov,
                        int32_t first_step, dl_stream_t stream);

/* a2+a3+a4+a5 at ONE peer, keeping the pseudo-gradient: dl_delta_sgd that also writes the
 * packed wire (outer.grad of src/utils.py:221, as dl_delta_pack would):
 *   g = θ - inner[seg][j]; wire[k] = g (bf16 wire: RNE, and the SGD uses the rounded value);
 *   SGD as dl_unpack_sgd (divisor 1); θ and inner[seg][j] <- new θ
 * One pass: 28 B/param (fp32 wire; 24 on the first step) instead of 36 for dl_delta_pack +
 * dl_unpack_sgd, bit-identical to that pair (wire included). */
DL_API int dl_delta_pack_sgd(dl_tree_t tree, int32_t bucket, int32_t inner_slot,
                             float* outer_packed, void* wire, int32_t wire_dtype,
                             float* mom_packed, float lr, float momentum, int32_t nesterov,
                             int32_t first_step, dl_stream_t stream);

/* a2 -> a3 -> a4 -> a5 at ONE peer as the two-kernel pipeline (dl_delta_pack then
 * dl_unpack_sgd with divisor 1; src/utils.py:221, src/comm.py:118-119, src/train.py:267,
 * src/utils.py:226), cache-blocked: the bucket's chunk range is walked in tiles of
 * tile_chunks chunks (0 = one tile), each tile packed then stepped, so the unpack re-reads
 * the wire and θ bytes the pack just touched from the Infinity Cache. wire holds the
 * pseudo-gradient afterwards. Bit-identical to the two whole-range launches. */
DL_API int dl_pack_sgd_tiled(dl_tree_t tree, int32_t bucket, int32_t inner_slot,
                             float* outer_packed, void* wire, int32_t wire_dtype,
                             float* mom_packed, float lr, float momentum, int32_t nesterov,
                             int32_t first_step, int32_t tile_chunks, dl_stream_t stream);

/* Gather per-tensor fp32 (slot) into a packed buffer of dtype `dtype` (fp32 or bf16).
 * Used to pack device gradients (DP sync, src/comm.py:117-123 with device grads, called at
 * src/train.py:251) and to initialise the device θ_outer mirror (src/utils.py:215). */
DL_API int dl_gather(dl_tree_t tree, int32_t bucket, int32_t src_slot, void* packed,
                     int32_t dtype, dl_stream_t stream);

/* a5: sync_inner_model, src/utils.py:223-226: dst[seg][j] = packed[k] (fp32). */
DL_API int dl_scatter(dl_tree_t tree, int32_t bucket, const float* packed, int32_t dst_slot,
                      dl_stream_t stream);

/* a3 /n + a4 on one peer's shard after a reduce-scatter (the sharded variant):
 * flat contiguous arrays of n elements, no tree: g = wire[k] / divisor (divisor 1: untouched),
 * SGD exactly as dl_unpack_sgd on outer[k], mom[k]. The caller all-gathers `outer` and
 * scatters it to the inner params (dl_scatter) afterwards. 20 B/param of the shard. All
 * pointers 16-B aligned. */
DL_API int dl_shard_sgd(const void* wire, int32_t wire_dtype, int32_t divisor, float* outer,
                        float* mom, int64_t n, float lr, float momentum, int32_t nesterov,
                        int32_t first_step, dl_stream_t stream);

/* a3 (Σ, /n) + a4 on one peer's shard after an all_to_all instead of a reduce-scatter
 * (OuterSync(exchange="a2a")): `slices` holds n_slices equal slices of `len` elements
 * (wire dtype), slice q = rank q's copy of this peer's shard of the bucket
 * (src/comm.py:122 `all_reduce(SUM)` + :123 `/= num_peers`, then the SGD of src/train.py:267).
 * g = ((s_0 + s_1) + ... + s_{n-1}) / n in fp32 in rank order -- deterministic and identical
 * on every rank, bit-exact against oracle/or_sum_avg at every n (a bf16 wire is summed in
 * fp32 and never re-rounded) -- then dl_shard_sgd's SGD on outer[k], mom[k]. len a multiple
 * of 4; all pointers 16-B aligned. Reads n·sizeof(wire) + 8 B, writes 8 B per element. */
DL_API int dl_shard_reduce_sgd(const void* slices, int32_t wire_dtype, int32_t n_slices,
                               int64_t len, float* outer, float* mom, float lr, float momentum,
                               int32_t nesterov, int32_t first_step, dl_stream_t stream);

/* The same rank-order average without the SGD, for the ordered per-step DP gradient sync
 * (GradSync(exchange="a2a"), src/comm.py:120-123 on device grads): out[k] =
 * ((s_0[k] + s_1[k]) + ... + s_{n-1}[k]) / n in fp32. len a multiple of 4; 16-B aligned. */
DL_API int dl_shard_reduce_avg(const void* slices, int32_t wire_dtype, int32_t n_slices,
                               int64_t len, float* out, dl_stream_t stream);

/* ---- int8 wire codec (not in the reference) --------------------------
 * One DL_Q8_SLOT_BYTES slot per chunk of the bucket, in chunk order: fp32 scale at byte 0,
 * zeros to byte 64 (the encoder and the reduce write the whole header), int8 values at byte
 * 64 (bytes past the chunk's length stay zero; slots must be zeroed once).
 * Quantiser: s = amax/127, q = s == 0 ? 0 : clamp(rint(x/s), -127, 127), value q*s.
 * dl_delta_q8:      slots <- quantise(outer - inner) per chunk  (a2, 8 B read + 1.02 B written)
 * dl_q8_reduce:     out[j] <- quantise((sum_r deq(recv[r][j])) / divisor), r in rank order;
 *                   recv holds n_peers x n_slots slots; out may alias recv when n_peers == 1
 * dl_unpack_sgd_q8: g = deq(slot); SGD and copy-back exactly as dl_unpack_sgd (divisor 1). */
DL_API int dl_delta_q8(dl_tree_t tree, int32_t bucket, int32_t inner_slot,
                       const float* outer_packed, void* slots, dl_stream_t stream);
DL_API int dl_q8_reduce(const void* recv, int32_t n_peers, int32_t n_slots, int32_t divisor,
                        void* out, dl_stream_t stream);
DL_API int dl_unpack_sgd_q8(dl_tree_t tree, int32_t bucket, const void* slots,
                            float* outer_packed, float* mom_packed, float lr, float momentum,
                            int32_t nesterov, int32_t first_step, int32_t inner_slot,
                            dl_stream_t stream);

/* ---- serializer (src/serializer.py:11-15) ----------------------------------------------
 * out is fp32 of 2*numel elements: out[0] = meta0, out[1] = meta1, out[numel + i] =
 * float(src[i]) for src dtype DL_F32/DL_BF16/DL_F16. out[2..numel) is left unwritten, as
 * the reference leaves it uninitialised (torch.empty, src/serializer.py:12). numel >= 2. */
DL_API int dl_serialize(const void* src, int32_t src_dtype, int64_t numel, float meta0,
                        float meta1, float* out, dl_stream_t stream);
/* The fp64 frame (torch.cat promotes the fp32 metadata plane to the fp64 payload's dtype):
 * out is fp64 of 2*numel elements, out[0] = (double)meta0, out[1] = (double)meta1 (the
 * metadata rounds through fp32 first, as the reference's fp32 metadata tensor does),
 * out[numel + i] = src[i]. */
DL_API int dl_serialize_f64(const double* src, int64_t numel, float meta0, float meta1,
                            double* out, dl_stream_t stream);

/* ---- synthetic parameter trees (bench / tests) ------------------------------------------
 * dst[i] = base + u(seed, stream_id, i) * scale (+ add[i] if add != NULL), with
 * u = ((splitmix64(seed*0xD1B54A32D192ED03 + (stream_id<<40) + i) >> 40) - 2^23) * 2^-23,
 * all fp32 ops correctly rounded: bit-identical to diloco_amd.synth (numpy). */
DL_API int dl_fill_synth(float* dst, int64_t n, uint64_t seed, uint64_t stream_id, float base,
                         float scale, const float* add, dl_stream_t stream);
/* TEST SUPPORT, not part of the outer step: a slow producer for the ordering tests
 * (tests/test_async_order_gpu.py, the slow-producer cases of tests/test_dropin_gpu.py): one
 * workgroup that occupies `stream` for `ns` nanoseconds of the wall clock of the device
 * `stream` belongs to (at most 10 s), touching no memory. */
DL_API int dl_spin(uint64_t ns, dl_stream_t stream);

/* ---- RCCL ------------------------------------------------------------
 * The exchange of src/comm.py:122 for hosts that drive RCCL through this library instead of
 * torch.distributed. RCCL is resolved at run time: a communicator must be used with the
 * RCCL that created it (a PyTorch process carries its own; ProcessGroupNCCL._comm_ptr()
 * returns its ncclComm_t). dl_rccl_load(path): that library; NULL = the RCCL already loaded
 * in the process, else librccl.so.1. The other entry points load it on first use.
 * Collectives are SUM, enqueued on `stream`, dtype DL_F32 / DL_BF16 / DL_F16 / DL_U8. */
DL_API int dl_rccl_load(const char* path);
DL_API int dl_rccl_version(int32_t* version);
DL_API int dl_comm_unique_id(void* id /* 128 B, NCCL_UNIQUE_ID_BYTES */);
DL_API int dl_comm_init(dl_comm_t* comm, int32_t nranks, const void* id, int32_t rank);
DL_API int dl_comm_destroy(dl_comm_t comm);
/* in place: buf[0:count) <- Σ over the communicator's ranks (src/comm.py:122; /n is the
 * caller's, e.g. dl_unpack_sgd's divisor) */
DL_API int dl_allreduce(void* buf, int64_t count, int32_t dtype, dl_comm_t comm,
                        dl_stream_t stream);
/* recv[0:recv_count) <- Σ_ranks send[rank*recv_count : (rank+1)*recv_count) (sharded step) */
DL_API int dl_reduce_scatter(const void* send, void* recv, int64_t recv_count, int32_t dtype,
                             dl_comm_t comm, dl_stream_t stream);
/* recv[r*send_count : (r+1)*send_count) <- rank r's send[0:send_count) */
DL_API int dl_all_gather(const void* send, void* recv, int64_t send_count, int32_t dtype,
                         dl_comm_t comm, dl_stream_t stream);
/* Point-to-point, the payload leg of the device pipeline transport:
 * replaces src/comm.py:38 `dist.send(tensor.to("cpu"), dst)` and src/comm.py:67
 * `dist.recv(tensor, group)` (after the any-source header names the sender) with RCCL over
 * xGMI on device buffers. A send and a receive on the same rank (or several transfers that
 * must progress together) go between dl_group_start() and dl_group_end(). */
DL_API int dl_send(const void* buf, int64_t count, int32_t dtype, int32_t peer, dl_comm_t comm,
                   dl_stream_t stream);
DL_API int dl_recv(void* buf, int64_t count, int32_t dtype, int32_t peer, dl_comm_t comm,
                   dl_stream_t stream);
DL_API int dl_group_start(void);
DL_API int dl_group_end(void);

/* ---- direct peer-access exchange (one node; SURVEY §8e alternative to RCCL) ----------------
 * IPC: dl_ipc_handle(ptr) -> the handle of the allocation holding ptr + ptr's byte offset in
 * it; a peer maps it with dl_ipc_open (base address; add the offset) and unmaps with
 * dl_ipc_close(base). dl_can_access_peer: hipDeviceCanAccessPeer; dl_enable_peer_access:
 * hipDeviceEnablePeerAccess.
 * dl_xgmi_reduce_sgd: on rank `rank` of n (<= 8), for packed elements [lo, lo+len) (this rank's
 * shard; lo, len multiples of 4, buffers 16-B aligned): g = (Σ_q wires[q][k] in rank order)/n,
 * Nesterov SGD on thetas[rank][k] and mom[k - lo], then thetas[q][k] = θ for every q. wires /
 * thetas: host arrays of n device addresses (peers' IPC-mapped buffers). Order it between two
 * barriers of the n ranks: after every rank's wire is written, before any rank reads θ. */
#define DL_IPC_HANDLE_BYTES 64
DL_API int dl_ipc_handle(const void* ptr, void* handle, int64_t* offset);
DL_API int dl_ipc_open(const void* handle, void** base);
DL_API int dl_ipc_close(void* base);
DL_API int dl_can_access_peer(int32_t device, int32_t peer, int32_t* can);
/* hipDeviceEnablePeerAccess(peer) from the current device; already enabled is success */
DL_API int dl_enable_peer_access(int32_t peer);
/* Stream-ordered system-scope fence on every XCD of this GPU (L2 write-back + invalidate):
 * issue it after kernels whose stores peers will read over xGMI (before the barrier that
 * releases the peers), and after that barrier before reading what peers wrote here or
 * re-reading their memory. Coarse-grained (hipMalloc / PyTorch) buffers are otherwise
 * coherent across GPUs only at the runtime's own synchronisation points. */
DL_API int dl_sys_fence(dl_stream_t stream);
/* dl_sys_fence that also records, per workgroup, the XCD it ran on (HW_REG_XCC_ID, 0..7) into
 * the device array xcc[cap]; *grid = the workgroups launched (one per CU: multiProcessorCount).
 * Lets a test prove that the fence reached every XCD. */
DL_API int dl_sys_fence_census(uint32_t* xcc, int32_t cap, int32_t* grid, dl_stream_t stream);
/* link probe: dst[i*bytes_each ...] <- srcs[i][0 .. bytes_each) for i < nsrc (<= 8), all
 * sources streamed at once by one kernel (measures per-link and aggregate peer read rates) */
DL_API int dl_peer_gather(const uint64_t* srcs, int32_t nsrc, int64_t bytes_each, void* dst,
                          dl_stream_t stream);
DL_API int dl_xgmi_reduce_sgd(const uint64_t* wires, const uint64_t* thetas, int32_t n,
                              int32_t rank, int64_t lo, int64_t len, float* mom, float lr,
                              float momentum, int32_t nesterov, int32_t first_step,
                              dl_stream_t stream);

/* dl_xgmi_reduce_sgd without a wire: inners[q] is rank q's INNER parameters laid out in the
 * packed layout (OuterSync(exchange="xgmi_inner") keeps them in one such arena), and the
 * kernel forms g = (Σ_q (thetas[rank][k] - inners[q][k]) in rank order) / n itself -- the
 * subtraction of src/utils.py:221 rank q would have made, θ_outer being identical on every
 * rank -- so no rank runs dl_delta_pack. Bit-identical to dl_delta_pack + dl_xgmi_reduce_sgd;
 * same ordering rules (between two barriers, dl_sys_fence around each). */
DL_API int dl_xgmi_delta_sgd(const uint64_t* inners, const uint64_t* thetas, int32_t n,
                             int32_t rank, int64_t lo, int64_t len, float* mom, float lr,
                             float momentum, int32_t nesterov, int32_t first_step,
                             dl_stream_t stream);

/* ---- calibration ------------------------------------------------------------------------
 * dst[0:bytes) = src[0:bytes) with the segment walker's access shape (one 256-lane
 * workgroup per 16 KiB, 4 float4 loads per lane before the stores); flags: DL_TUNE_NT_LOADS =
 * non-temporal loads and stores, DL_COPY_WIDE = 8 float4 loads per lane (32 KiB per
 * workgroup). bench.py times every variant in the same run as the outer step and reads its
 * roofline fractions against the fastest: the copy ceiling (not on the reference's path).
 * Probes: DL_COPY_READ only reads src[0:bytes) (dst is not written, may be NULL);
 * DL_COPY_WRITE only writes dst[0:bytes), each 32-bit word its own index (src unused, may be
 * NULL). DL_COPY_STREAMS(s), s = 1..4, splits the buffer into s equal streams (bytes a
 * multiple of 16 s) and has each workgroup touch one 16 KiB tile of every stream, as a walker
 * kernel with s input (output) buffers does. bench.py combines the rates into the same-run
 * ceiling of a kernel's byte mix: t >= R / BW_read(s_r) + W / BW_write(s_w) (tools/rw_mix.hip). */
#define DL_COPY_WIDE 8
#define DL_COPY_READ 16
#define DL_COPY_WRITE 32
#define DL_COPY_STREAMS(s) ((((s) - 1) & 3) << 8)
DL_API int dl_copy(const void* src, void* dst, int64_t bytes, int32_t flags, dl_stream_t stream);

DL_API const char* dl_last_error(void);
DL_API int dl_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* DILOCO_HIP_H */
