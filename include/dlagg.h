/*
 * dlagg.h — C ABI of libdlagg.so, the MI355X (gfx950) implementation of the
 * accdfl gossip model-aggregation reduce (FedAvg).
 *
 * Reference interface replaced:
 *   accdfl/core/gradient_aggregation/fedavg.py:12-26   FedAvg.aggregate(models, weights)
 *     - :14-17  weight defaulting (falsy -> uniform 1/N) / length assertion
 *     - :20-22  center = deepcopy(models[0]); p.mul_(0)       -> acc = p0 * 0
 *     - :23-25  for m, w: c1.add_(w * p1)                      -> acc = acc + w_k * p_k
 *   accdfl/core/gradient_aggregation/__init__.py:12-17 GradientAggregation.aggregate
 *   accdfl/core/model_manager.py:56-58 aggregate_trained_models (list order = summation order)
 *
 * The reference has no native code; there is no FFI to bind in it.  The Python
 * host package (decentralized-learning_amd/accdfl_amd) binds these entry points
 * with ctypes; INTEGRATION.md shows the binding a maintainer would add to the
 * reference tree.
 *
 * Arithmetic contract ("bit-exact mode", the only mode): for every element j
 *     acc = p_0[j] * 0                       (keeps -0, turns +-Inf/NaN into NaN)
 *     for k = 0 .. n_peers-1 (list order):
 *         acc = R(acc + R(W(w_k) * p_k[j]))
 * with no fused multiply-add.  W(w) is the weight rounded RNE from double to the
 * dtype's op-math type (float for F32/BF16/F16, double for F64).  R() is the
 * op-math result rounded RNE to the storage dtype (identity for F32/F64).  This
 * equals torch-CPU's `c.add_(w * p)` sequence bit for bit; NaN payload bits are
 * not part of the contract (torch-CPU itself emits different NaN payloads
 * depending on vector-lane position).
 *
 * Ownership: the caller owns every buffer (device pointers from hipMalloc / the
 * torch caching allocator).  The library keeps no device allocation across calls.
 * Errors: return 0 on success, a negative DLA_E_* code or a positive hipError_t;
 * dla_last_error() returns a thread-local message.  No C++ exception crosses the ABI.
 * Threading: reentrant; work is enqueued on `stream` (a hipStream_t, NULL = the
 * default stream) and the call does not synchronise.
 *
 * Surface.  The drop-in for the reference path is: dla_wsum, dla_wsum_multi(_table[_acc]),
 * dla_wsum_mixed, dla_wsum_slab(_tiled) + dla_slab_stage, dla_wsum_sharded, dla_host_round_start /
 * _finish, dla_host_reduce / dla_host_reduce_launch / _join, dla_plan_*, dla_mean and the helpers
 * (version, build id, last error, shard range, tile size, copy batch, shutdown).  INTERNAL entry
 * points — exported for the library's own tests, benchmarks and diagnostics, not part of the
 * drop-in and free to change: dla_wsum_ex (forced launch knobs), dla_select_kernel,
 * dla_host_in_place_rounds, dla_host_reduce_deferred (dla_host_reduce_launch's body on the
 * caller's thread).
 */
#ifndef DLAGG_H
#define DLAGG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DLA_ABI_VERSION 13

/* element dtypes of the peer buffers and of the output */
#define DLA_F32 0
#define DLA_BF16 1
#define DLA_F16 2
#define DLA_F64 3

/* error codes (negative; positive values are hipError_t) */
#define DLA_OK 0
#define DLA_E_INVALID (-1)    /* bad argument (null pointer, n_peers < 1, n_elems < 0, dtype) */
#define DLA_E_ALIAS (-2)      /* out aliases a peer other than peers[0] in a multi-pass reduce */
#define DLA_E_CONFIG (-3)     /* launch configuration not supported */

/* Launch tuning knobs for dla_wsum_ex (0 = library default for each field). */
typedef struct dla_launch_cfg {
  int variant;      /* 0 = by shape: passes of bf16 / f16 peers and of more than 8 fp32
                       peers take 9 (>= 32 peers; 21 when the output is <= 8 MiB) or 12;
                       fp32 shares over 8, 16 or 32 peers beyond
                       256 MiB whose big tiles fill >= 80 % of their last round of 1024
                       resident waves take 16 (17 from one full round up), fp64 over 4..8
                       likewise; fp64 small shares over more than 8 peers 8; otherwise 4.
                       Cache policy of the 16-byte register stream:
                       1 = plain loads / plain stores   2 = nt loads / plain stores
                       4 = nt loads / sc1 stores (write-through, line not kept in L2)
                       8 = word-per-lane kernel (nt loads, sc1 stores, up to 64 peers
                           in flight per lane; chunks/block/grid are ignored)
                       9 = vector-per-lane kernel: 8 bytes per lane per load, 32 peers in
                           flight per lane (passes of more than 8 peers; fp64 and smaller
                           passes take 4); 12 = 8 bytes x 16; 21 = 9 with plain (L2
                           write-back) output stores instead of sc1.  (16-byte-per-lane forms
                           were measured slower at every shape and are not built.)
                      16 = peer-major big-tile kernel (fp32 <= 8, 16 or 32 peers, fp64 <= 8:
                           16 KiB of output per wave, one peer's 16 KiB streamed at a
                           time; chunks/block/grid are ignored; other dtypes take 4)
                      17 = 16 with the partial last round of big tiles spread over one
                           round of 64-chunk segment workgroups                       */
  int chunks;       /* 16-byte chunks per lane per peer per tile: 1, 2, 4; 0 = by shape  */
  int grid_blocks;  /* workgroups; 0 = one per work tile (no grid-stride loop)           */
  int block;        /* threads per workgroup: 64 or 256; 0 = by shape                    */
} dla_launch_cfg_t;

/* ABI version (DLA_ABI_VERSION). */
int dla_version(void);

/* Build id: a hash of the sources and compile flags this library was built from
 * (static string).  The Python loader refuses a library whose id differs from the
 * tree's, so a stale prebuilt .so fails loudly instead of running old code.  ABI v5. */
const char* dla_build_id(void);

/* Message describing the last error on this thread ("" if none). */
const char* dla_last_error(void);

/* Replaces fedavg.py:20-25 for one flat parameter buffer per peer.
 *   peers    host array of n_peers DEVICE pointers, each to n_elems elements of dtype
 *   weights  host array of n_peers doubles (already defaulted, fedavg.py:14-17)
 *   out      DEVICE pointer to n_elems elements; may alias peers[0]
 * Any n_peers >= 1 is accepted (more than DLA_MAX_PEERS_PER_PASS peers run as
 * several passes that carry the running sum in `out`, which keeps list order). */
int dla_wsum(int dtype, const void* const* peers, const double* weights, int n_peers,
             int64_t n_elems, void* out, void* stream);

/* INTERNAL: dla_wsum with explicit launch knobs (benchmarks / tuning). */
int dla_wsum_ex(int dtype, const void* const* peers, const double* weights, int n_peers,
                int64_t n_elems, void* out, void* stream, const dla_launch_cfg_t* cfg);

/* Peers stored as rows of one slab: peer k = base + k * pitch_elems elements.
 * This is the layout of the device staging slab (accdfl_amd PeerSlab). */
int dla_wsum_slab(int dtype, const void* base, int64_t pitch_elems, const double* weights,
                  int n_peers, int64_t n_elems, void* out, void* stream);

/* Peers stored in the TILE-INTERLEAVED slab layout (the many-peer PeerSlab layout):
 * the slab is [n_tiles][slab_rows][tile_elems]; element j of peer (row) k lives at
 *     base + ((j / tile_elems) * slab_rows + k) * tile_elems + j % tile_elems
 * so the rows' tiles at one offset sit side by side and a many-peer reduce streams one region
 * of HBM instead of n_peers distant ones.  Peers 0..n_peers-1 (n_peers <= slab_rows) are
 * reduced in row order into the contiguous `out` (n_elems elements).  tile_elems: a power of
 * two of >= 16 bytes; base and out 16-byte aligned; F32, BF16 or F16.  cfg (may be NULL):
 * variant 0 (by shape, as dla_wsum), 8, 9, 12, 21 or 28 picks the vector-per-lane kernel form
 * (8 / 28: 8 peers in flight per lane, sc1 / plain stores; 12: 16; 9 / 21: 32, sc1 / plain).
 * ABI v5. */
int dla_wsum_slab_tiled(int dtype, const void* base, int64_t tile_elems, int64_t slab_rows, const double* weights,
                        int n_peers, int64_t n_elems, void* out, void* stream, const dla_launch_cfg_t* cfg);

/* The tile (in elements) the library recommends for a tile-interleaved slab of slab_rows rows of
 * n_elems elements (what PeerSlab uses); 0 for invalid arguments.  ABI v5. */
int64_t dla_slab_tile_elems(int dtype, int slab_rows, int64_t n_elems);

/* Stages n_elems elements of one peer into row `row` of a tile-interleaved slab (the layout
 * dla_wsum_slab_tiled reads: [n_tiles][slab_rows][tile_elems]) at the row's flat element offset
 * dst_elem — a received model's parameters landing in HBM (accdfl/core/model_manager.py:39-47 keeps
 * them until fedavg.py:23-25 reads them; accdfl/util/eva/transfer/incoming.py:35 is where their bytes
 * arrive).  `src` is host memory (page-locked or pageable) or device memory; the copy is ONE
 * hipMemcpy2DAsync for the whole tiles (rows of one tile, destination pitch slab_rows tiles: the copy
 * engine writes each tile in place) plus up to two plain copies for the partial tiles at either end,
 * enqueued on `stream`.  No contiguous device row and no scatter pass.  The usual async-copy rules
 * hold: page-locked sources must stay untouched until the stream passes the copy; pageable sources
 * are consumed before the call returns.  n_tiles: the slab's tile count (its leading dimension); a
 * range [dst_elem, dst_elem + n_elems) beyond n_tiles * tile_elems is refused with DLA_E_INVALID
 * before any copy (ABI v13).  ABI v10. */
int dla_slab_stage(int dtype, void* base, int64_t tile_elems, int64_t slab_rows, int64_t n_tiles, int row,
                   int64_t dst_elem, const void* src, int64_t n_elems, void* stream);

/* Replaces the per-parameter inner loop of fedavg.py:24-25 for T parameter
 * tensors at once (one model = T tensors, parameters() order).
 *   peer_ptrs host array [n_tensors * n_peers]: peer_ptrs[t * n_peers + k] is
 *             peer k's DEVICE pointer for tensor t
 *   outs      host array [n_tensors] of DEVICE output pointers
 *   numels    host array [n_tensors] of element counts
 * Tensors are packed into as few launches as the kernel-argument block allows. */
int dla_wsum_multi(int dtype, int n_tensors, const void* const* peer_ptrs, void* const* outs,
                   const int64_t* numels, const double* weights, int n_peers, void* stream);

/* dla_wsum_multi for rounds of many peers (device-resident models: FedAvg.aggregate on modules in
 * HBM, accdfl/core/gradient_aggregation/fedavg.py:24 walking every parameter of every model; the
 * simulator's large-N average, simulations/gl/gl_simulation.py:96-105).  The (tensor x peer)
 * pointer table and one record per tensor travel to the device as ONE table — written into the
 * caller's page-locked `table_host` and copied into `table_dev` (both at least
 * dla_wsum_multi_table_bytes(n_tensors, n_peers) bytes, 16-byte aligned): by a copy kernel on `stream`
 * reading table_host across PCIe, or — when `stream` still has work queued and the call moves
 * >= 256 MiB — by a copy on a library side stream that overlaps that work, the call returning once the
 * copy is done (v13; before: one hipMemcpyAsync on `stream`, ~24 us of idle GPU per call) — and
 * every 16-byte aligned F32 / BF16 / F16 tensor is folded by ONE launch per pass of up to
 * DLA_MAX_PEERS_PER_PASS peers, whatever the peer and tensor counts (128 google_speech ResNet-34
 * models: 14 080 tensors, 1 launch; dla_wsum_multi: 110).  Other tensors (unaligned, F64) take the
 * per-tensor path.  Same arguments and arithmetic as dla_wsum_multi; outs[t] may alias tensor t of
 * peer 0.  The caller leaves table_host and table_dev untouched until the stream has passed this
 * work (e.g. an event recorded after the call).  ABI v8.
 * Blocking: the side-stream upload makes the CALLING THREAD wait for the table copy (~15-20 us) before
 * the reduce is enqueued.  The library takes that branch only when the call moves >= 256 MiB and its
 * own estimate (the algorithmic bytes of the table reduces it queued on `stream` at ~6 TB/s) says the
 * stream is still busy; work on `stream` from anyone else is not seen by the estimate, so on a stream
 * that also carries e.g. training kernels the call may block for the copy while those run.  Otherwise
 * the call never blocks.  The table's device (table_dev's) is made current for the call and restored. */
int64_t dla_wsum_multi_table_bytes(int n_tensors, int n_peers);
int dla_wsum_multi_table(int dtype, int n_tensors, const void* const* peer_ptrs, void* const* outs,
                         const int64_t* numels, const double* weights, int n_peers, void* table_host,
                         void* table_dev, void* stream);

/* dla_wsum_multi_table continuing a fold: with acc_in != 0, outs[t] already holds the fold of earlier
 * peers (fedavg.py:23-25 run over them in list order, in the tensor's dtype) and the n_peers given are
 * folded into it, so a round of many device-resident models can be launched group by group while the
 * caller still walks the later models' parameters — the result is the same bits as one call over all
 * of them.  outs[t] may alias no peer when acc_in != 0.  acc_in == 0 is dla_wsum_multi_table.  ABI v12. */
int dla_wsum_multi_table_acc(int dtype, int n_tensors, const void* const* peer_ptrs, void* const* outs,
                             const int64_t* numels, const double* weights, int n_peers, int acc_in, void* table_host,
                             void* table_dev, void* stream);

/* fedavg.py:20-25 for one parameter whose peers do not all share models[0]'s dtype: the reference
 * accepts such models and `c1.add_(w * p1)` (:25) then rounds the product in the PEER's dtype
 * (op-math f32, or f64 for an f64 peer) and the sum in the CENTRE's dtype after promotion (the add in
 * f64 when either side is f64, else in f32; an f64 sum reaches a 16-bit centre through float):
 *     acc = p_0 * 0                                           (in out_dtype, op-math of out_dtype)
 *     for k in list order:
 *         prod = R_{d_k}(W_{d_k}(w_k) * p_k[j])
 *         acc  = R_{out}(acc + prod)   in f64 if out or d_k is F64, else in f32
 *   peer_dtypes  host array of n_peers DLA_* codes; peer_dtypes[0] must be out_dtype (models[0]'s
 *                parameter is the result's, fedavg.py:20)
 *   peers        n_peers DEVICE pointers, peer k to n_elems elements of peer_dtypes[k]
 *   out          DEVICE pointer to n_elems elements of out_dtype; may alias peers[0] only
 * Uniform dtypes give dla_wsum's bits (it is the special case d_k = out).  Any alignment.  ABI v13. */
int dla_wsum_mixed(int out_dtype, const int* peer_dtypes, const void* const* peers, const double* weights,
                   int n_peers, int64_t n_elems, void* out, void* stream);

/* Replaces scripts/distill.py:124-129 (teacher-logit aggregation,
 * torch.mean(torch.stack(preds), dim=0)) for a whole batch of logits at once:
 *     out = (((+0 + p_0) + p_1) + ... + p_{N-1}) / N      element-wise, F32 or F64.
 * The sum is sequential in list order, op-math = storage type, and the division is
 * correctly rounded; torch's own reduction order is implementation-defined, so parity
 * with torch.mean is within |err| <= N * 2^-23 * sum_k |p_k| / N (f32).  out may alias
 * peers[0] (also when n_peers > DLA_MAX_PEERS_PER_PASS). */
int dla_mean(int dtype, const void* const* peers, int n_peers, int64_t n_elems, void* out, void* stream);

/* Largest peer count one kernel pass takes (kernel-argument pointer table). */
int dla_max_peers_per_pass(void);

/* INTERNAL (benchmarks, profilers).  Name of the kernel family dla_wsum picks (default launch, 16-byte aligned buffers) for
 * this dtype, peer count and size: "wsum_bigtile_kernel", "wsum_vec_kernel", "wsum_wide_kernel"
 * or "wsum_stream_kernel" (static string; "" for invalid arguments).  For profilers and
 * benchmarks that must name the dominant kernel.  ABI v4. */
const char* dla_select_kernel(int dtype, int n_peers, int64_t n_elems);

/* Bucket-sharded reduce over several GPUs of ONE process (replaces the
 * single-device fedavg.py:20-25 loop for models that live on several GPUs of the aggregating
 * node, e.g. the per-node models of the simulator, simulations/learning_simulation.py:335).
 *   dev_ids  n_shards HIP device ids; shard s runs on dev_ids[s] (ids may repeat)
 *   peers    n_peers DEVICE pointers, each to n_elems elements of dtype, on ANY device of the
 *            process: a shard reads the peers on other GPUs over xGMI (peer access is enabled
 *            on first use and kept until dla_shutdown)
 *   outs     n_shards DEVICE pointers, outs[s] to n_elems elements; shard s writes its bucket
 *            [start_s, end_s) (dla_shard_range) at the same offset of outs[s] (outs may all be
 *            one buffer: every shard then writes its bucket into it directly)
 *   gather   0: each outs[s] holds its own bucket only; 1: all-gather, every outs[s] receives
 *            every bucket (peer-to-peer copies over xGMI); 2: outs[0] receives every bucket
 *   streams  n_shards hipStream_t, streams[s] on dev_ids[s] (NULL = that device's null stream);
 *            nothing is synchronised: the peers must be ready when the streams reach this work,
 *            and with gather the copies into outs[d] are ordered on streams[d] behind the
 *            reduces they copy (library events)
 * Buckets are contiguous, every start a multiple of 256 bytes: B = ceil(n_elems / n_shards)
 * rounded up to 256 / sizeof(dtype) elements, shard s = [min(s*B, n), min((s+1)*B, n)).  Every
 * element keeps its list-order fold, so the result is bit-identical to dla_wsum.  ABI v5. */
int dla_wsum_sharded(int dtype, int n_shards, const int* dev_ids, const void* const* peers, const double* weights,
                     int n_peers, int64_t n_elems, void* const* outs, int gather, void* const* streams);

/* The bucket [*start, *end) of `shard` in dla_wsum_sharded's split.  ABI v5. */
int dla_shard_range(int dtype, int64_t n_elems, int n_shards, int shard, int64_t* start, int64_t* end);

/* Releases what dla_wsum_sharded keeps across calls (its synchronisation events, and the
 * peer-access pairs it enabled).  Call only when no sharded work is in flight.  ABI v5. */
int dla_shutdown(void);

/* Prepared reduce: validates and stores the peer/out pointers once, so a round
 * that reduces the same device buffers again (a PeerSlab every round, a benchmark
 * loop) pays only the launch.  Same semantics as dla_wsum. */
typedef struct dla_plan dla_plan_t;
int dla_plan_create(dla_plan_t** plan, int dtype, const void* const* peers, const double* weights,
                    int n_peers, int64_t n_elems, void* out, const dla_launch_cfg_t* cfg);
/* Replace the weights (e.g. new GL ages, fedavg.py:14-17 defaulting done by the caller). */
int dla_plan_set_weights(dla_plan_t* plan, const double* weights);
int dla_plan_launch(const dla_plan_t* plan, void* stream);
void dla_plan_destroy(dla_plan_t* plan);

/* Host-side staging for CPU-resident peers (no GPU work, HOST pointers only):
 * dsts[i] <- srcs[i] for i < n, bytes[i] bytes each, in one call.  Replaces the
 * per-parameter flatten of `m.parameters()` (the zip order of fedavg.py:24) into a
 * pinned staging row before the H2D copy, and the unflatten of the averaged row back
 * into the result's parameters (fedavg.py:20, 25: the values land in the deepcopy's
 * tensors).  One native call instead of a torch op per tensor: the GL merge of two
 * GNLeNet models (configs[1]) packs 28 tensors per round.  Regions must not overlap. */
int dla_host_copy_batch(void* const* dsts, const void* const* srcs, const int64_t* bytes, int n);
/* dla_host_copy_batch with flags.  DLA_COPY_STREAMING: streaming (non-temporal) stores, for
 * destinations only the GPU reads next — an EVA block list gathered into a page-locked ingress
 * buffer before its H2D (accdfl/util/eva/transfer/incoming.py:35's join): no read-for-ownership of
 * the destination lines and no dirty lines the DMA's reads must snoop.  ABI v9. */
#define DLA_COPY_STREAMING 1
int dla_host_copy_batch_ex(void* const* dsts, const void* const* srcs, const int64_t* bytes, int n, int flags);

/* A round of CPU-resident models in two calls — fedavg.py:20-25 for the reference's own call
 * sites, whose models live in host memory (the GL merge of N=2 models every round,
 * accdfl/gl/community.py:117; DL/DFL rounds of small models, accdfl/dl/community.py:170,
 * accdfl/dfl/community.py:673) — so the caller builds the result module (the deepcopy of
 * fedavg.py:20) while the GPU works.  ABI v6.
 *   dla_host_round_start: packs tensor t of peer k (HOST pointer tensors[k * n_tensors + t],
 *     numels[t] elements of dtype, the zip order of fedavg.py:24) into row k of `rows`
 *     (pitch_elems per row, a multiple of 16 bytes), then enqueues the reduce of rows
 *     0..n_peers-1 on `stream`.  The kernel reads the rows and writes `result`
 *     (sum(numels) elements) across PCIe, with no staging DMA: `rows` and `result` must be
 *     page-locked host memory mapped into the device at the same address (hipHostMalloc,
 *     torch pin_memory; checked), 16-byte aligned, and untouched until finish returns.
 *   dla_host_round_finish: waits for `stream`, then copies the averaged values into outs[t]
 *     (HOST pointers, numels[t] elements each).
 * Peers that already ARE page-locked rows (every tensor of peer k back to back from one 16-byte
 * aligned, page-locked, device-mapped address, as a model decoded into a page-locked ingress buffer
 * holds them) are not packed: the kernel reads them in place and `rows` is left untouched (ABI v11). */
int dla_host_round_start(int dtype, int n_peers, int n_tensors, const void* const* tensors, const int64_t* numels,
                         const double* weights, void* rows, int64_t pitch_elems, void* result, void* stream);
int dla_host_round_finish(int dtype, int n_tensors, const int64_t* numels, const void* result, void* const* outs,
                          void* stream);

/* A large round of CPU-resident models in one synchronous call — fedavg.py:20-25 at the reference's
 * call sites when the models are large (the DFL aggregator's N models, accdfl/dfl/community.py:673;
 * the simulators' averages, simulations/learning_simulation.py:335) — streamed through the GPU in
 * element chunks of the flat (parameters()-order) vector.  Only the flat elements [begin, end) are
 * reduced and written (one bucket per GPU when the round is sharded over several GPUs: one call per
 * GPU, each from its own host thread, with that GPU current).  Chunks ramp up — 1/4 and 1/2 of
 * chunk_elems, then chunk_elems — so the first DMA starts after a quarter-size pack.  For chunk c
 * (buffer c & 1):
 *   1. pack: chunk c's elements of every peer (HOST pointers tensors[k * n_tensors + t], numels[t]
 *      elements of dtype each) into row k of h_stage[buf], rows dense at the chunk's length rounded up
 *      to 256 bytes (threaded copy with streaming stores);
 *   2. one contiguous H2D DMA of the rows into d_stage[buf] on copy_stream (made to wait for the
 *      compute stream only if the reduce that last read d_stage[buf] has not finished yet);
 *   3. the list-order reduce of the rows into d_out[buf] on stream, then a D2H into h_out[buf];
 *   4. while chunk c+1 is packed and copied in: unpack chunk c into outs[t] (HOST pointers).
 * Buffers (caller-owned, untouched by anything else during the call):
 *   h_stage  page-locked host, 2 * n_peers * chunk_elems elements    d_stage device, same size
 *   h_out    page-locked host, 2 * chunk_elems elements               d_out   device, same size
 * chunk_elems * sizeof(dtype) must be a multiple of 256 bytes.  stream and copy_stream are streams of
 * the current device (they may be the same stream).  Returns after every output has been written.
 * Replaces one DMA per tensor per peer per chunk (14 080 per chunk for 128 google_speech ResNet-34
 * models of 110 tensors) by one per chunk.  ABI v7.
 * Page-locked peers (ABI v11; VERDICT r03: page-locked peers were packed like pageable ones and ran
 * slower): when every peer's tensors lie back to back in one page-locked, device-mapped row (16-byte
 * aligned at `begin`), steps 1-2 are skipped — the reduce reads chunk c of every row in place across
 * PCIe — and, when h_out is device-mapped too, writes h_out[buf] directly (no D2H DMA); h_stage and
 * d_stage are then unused.  Other peers are packed as in step 1; when h_stage and h_out are both
 * device-mapped (hipHostMalloc, torch pin_memory) the reduce reads the packed rows in h_stage[buf] and
 * writes h_out[buf] across PCIe in place of steps 2-3's DMAs (d_stage and d_out unused).  The result
 * is the same bits. */
int dla_host_reduce(int dtype, int n_peers, int n_tensors, const void* const* tensors, const int64_t* numels,
                    const double* weights, void* const* outs, int64_t begin, int64_t end, int64_t chunk_elems,
                    void* h_stage, void* d_stage, void* h_out, void* d_out, void* stream, void* copy_stream);

/* INTERNAL (diagnostics).  Host rounds (dla_host_reduce / _deferred / _launch calls and dla_host_round_start) whose peers the
 * kernel read in place from page-locked rows, since the library was loaded (diagnostics).  ABI v11. */
int64_t dla_host_in_place_rounds(void);

/* INTERNAL (tests; the product calls dla_host_reduce_launch).  dla_host_reduce with the outputs published late: outs[] is read only once *outs_ready (written by
 * the caller, read with acquire semantics) turns non-zero — > 0: outs[] is filled; < 0: the caller
 * gives up, and the call drains its copies and returns DLA_E_INVALID.  The caller starts the call on
 * one thread, allocates the result tensors on another while the first chunks are packed, copied in
 * and reduced (fedavg.py:20's deepcopy and the reduce overlap), fills outs[], then sets the flag;
 * only the first unpack waits for it.  outs_ready must not be NULL.  ABI v9. */
int dla_host_reduce_deferred(int dtype, int n_peers, int n_tensors, const void* const* tensors, const int64_t* numels,
                             const double* weights, void* const* outs, const int* outs_ready, int64_t begin,
                             int64_t end, int64_t chunk_elems, void* h_stage, void* d_stage, void* h_out, void* d_out,
                             void* stream, void* copy_stream);

/* dla_host_reduce_deferred on a thread of the library's own, with `device` current there: returns at
 * once with *job set (NULL on a validation failure).  The calling thread keeps no lock while the round
 * streams — a Python caller allocates and publishes the outputs and clones the result module under
 * its interpreter lock meanwhile, which a worker thread of its own would need for every step.
 * tensors, numels, outs, outs_ready, the staging buffers and the streams must stay valid until
 * dla_host_reduce_join; weights are copied.  Every launched job must be joined exactly once.  ABI v9. */
typedef struct dla_host_job dla_host_job_t;
int dla_host_reduce_launch(int device, int dtype, int n_peers, int n_tensors, const void* const* tensors,
                           const int64_t* numels, const double* weights, void* const* outs, const int* outs_ready,
                           int64_t begin, int64_t end, int64_t chunk_elems, void* h_stage, void* d_stage, void* h_out,
                           void* d_out, void* stream, void* copy_stream, dla_host_job_t** job);
/* Waits for a launched job and frees it; returns its status (its message: dla_last_error on this
 * thread). */
int dla_host_reduce_join(dla_host_job_t* job);

#ifdef __cplusplus
}
#endif

#endif /* DLAGG_H */
