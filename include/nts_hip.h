/*
 * nts_hip.h — C-ABI of the MI355X (gfx950) sampled-GNN hot path.
 *
 * This is the drop-in boundary: a plain-C interface (raw device pointers,
 * sizes, status codes; no torch types) that replaces the hot subset of the
 * reference's `Cuda_Stream` device layer (cuda/ntsCUDA.hpp:177-595) and its
 * NCCL wrapper (cuda/ntsCUDA.hpp:132-175).  Every entry point below names
 * the reference interface it replaces (file:line in AiX-im/Sample-based-GNN).
 *
 * Conventions
 *  - Vertex ids are uint32 (VertexId, dep/gemini/type.hpp:29; cuda/cuda_type.h:21).
 *  - Global CSC offsets are uint64 (the reference uses uint32 and overflows
 *    past 2^32 edges); per-batch sampled offsets are uint32.
 *  - Values are fp32 (ValueType, dep/gemini/type.hpp:31).
 *  - Sizes that are only known on the device (e_size, src_size of a sampled
 *    layer) are passed as device scalars plus a host-side capacity; kernels
 *    read the live size and never touch entries past it.  No entry point
 *    synchronises with the host.
 *  - All work is enqueued on the context's stream (async); buffers are owned
 *    by the caller.  Return value 0 = success; on failure the message is
 *    available from nts_hip_last_error() (thread-local).  The reference
 *    aborts instead (CHECK_CUDA_RESULT, cuda/ntsCUDAGraphOP.cu:21-28); the
 *    C++ host layer reproduces abort-on-error by throwing.
 *  - A context is re-entrant per stream and holds no global mutable state
 *    (unlike Cuda_Stream::total_*, cuda/ntsCUDAGraphOP.cu:64-66).
 */
#ifndef NTS_HIP_H
#define NTS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NTS_HIP_ABI_VERSION 11  /* 2: nts_sampcsc_dev gained dst_local_id, csr_edge_id;
                                  3: transform-first entry points, fused agg+GEMM removed,
                                     accuracy counts in the fused loss;
                                  4: PD cache entry points + omit fields, GEMM mode;
                                  5: two-piece f16 pair-table GEMMs (nts_hip_h2_*);
                                  6: nts_hip_spmm_csr_bwd_colmax + nts_hip_gemm_h2p_tn_gather_cm;
                                  7: the column maxima per part of rows (no row scales in
                                     the backward), nts_hip_csr_bwd_colmax_rows_per_part;
                                  8: nts_hip_comm_count; the CSR-backward column maxima scaled by
                                     the pair table's row scales (exact TN operand maxima);
                                  9: nts_sampcsc_dev::sizes_host;
                                  10: the activation's keep mask as bits (nts_hip_act_bits_words,
                                      nts_hip_spmm_csc_fwd_act_bits,
                                      nts_hip_spmm_csr_bwd_postmask_bits);
                                  11: MT19937 re-run of a short stream (nts_hip_mt_budget_scale,
                                      nts_hip_mt_checkpoint, nts_hip_mt_rewind) */

/* status codes */
#define NTS_OK 0
#define NTS_ERR_INVALID 1
#define NTS_ERR_HIP 2
#define NTS_ERR_OOM 3
#define NTS_ERR_UNSUPPORTED 4
#define NTS_ERR_RCCL 5

/* Random stream used by the sampler.
 *  PHILOX          : counter-based Philox4x32-10 keyed by (seed), counter
 *                    (word block, dst id, layer, batch_seq) — every dst is
 *                    independent, fully parallel (the fast default).
 *  MT19937_LEMIRE  : the reference's stream, bit-exact: one
 *                    `static thread_local std::mt19937 generator(seed)`
 *                    consumed sequentially by std::uniform_int_distribution
 *                    (core/ntsFastSampler.hpp:200-205) in libstdc++ >= 11 form
 *                    (Lemire nearly-divisionless, uniform_int_dist.h:246-263).
 *  MT19937_DIV     : same stream, libstdc++ <= 10 form (2-division rejection).
 * The MT modes consume one generator shared by all layers/batches of a
 * context, exactly like the reference's thread_local generator. */
#define NTS_RNG_PHILOX 0
#define NTS_RNG_MT19937_LEMIRE 1
#define NTS_RNG_MT19937_DIV 2

/* Edge weights, mirrors `enum class WeightType{Sum, Mean, None}`
 * (core/ntsFastSampler.hpp:27) with the CPU sampler's formulas
 * (core/ntsFastSampler.hpp:1111-1119, nts_norm_degree core/ntsBaseOp.hpp:652-657). */
#define NTS_WEIGHT_SUM 0
#define NTS_WEIGHT_MEAN 1  /* CPU sampler: norm / in_degree(dst) of the full graph (:1111-1113) */
#define NTS_WEIGHT_NONE 2
/* The reference GPU kernel get_mean_weight (cuda/ntsCUDATransferKernel.cuh:319-342):
 * norm / (sampled edge count of the dst).  Note the reference's GPU toolkits never
 * reach it: sample_gpu_fast(int, int, WeightType) drops the weight type
 * (core/ntsFastSampler.hpp:944-948), so GS_SAMPLE_ALLGPU
 * actually trains with SUM weights.  Offered for the kernel's semantics. */
#define NTS_WEIGHT_MEAN_SAMPLED 3
/* OR-ed into SUM / MEAN: UP_DEGREE — the degrees in the weights are the
 * sampled layer's own (in = sampled edges of the dst, out = sampled edges of
 * the src), SampledSubgraph::update_degrees(_GPU) (core/FullyRepGraph.hpp:189-217,
 * cfg key UP_DEGREE, core/ntsFastSampler.hpp:691-693,1107-1108). */
#define NTS_WEIGHT_UP_DEGREE 0x10

typedef struct nts_hip_ctx nts_hip_ctx;
typedef struct nts_hip_comm nts_hip_comm;

/* Replicated global graph resident in HBM (FullyRepGraph, core/FullyRepGraph.hpp:682-798
 * + Graph degrees core/graph.hpp:1157-1186,1420-1425,4525-4530). */
typedef struct {
  uint64_t n_vertices;
  uint64_t n_edges;
  const uint64_t *column_offset; /* [V+1] CSC keyed by dst                         */
  const uint32_t *row_indices;   /* [E] src ids, file order within each dst        */
  const uint32_t *in_degree;     /* [V] in_degree_for_backward  (clamped >= 1)     */
  const uint32_t *out_degree;    /* [V] out_degree_for_backward (clamped >= 1)     */
} nts_graph_dev;

/* One sampled layer (sampCSC, core/coocsc.hpp:417-460), device side.
 * Inputs: destination + v_size.  Everything else is written by
 * nts_hip_sample_layer.  CSR arrays may be NULL (no transpose built). */
typedef struct {
  uint32_t v_cap, e_cap, s_cap;    /* host capacities of the arrays below       */
  const uint32_t *destination;     /* [v_cap] global dst ids (input)           */
  const uint32_t *v_size;          /* device scalar: live dst count (input)    */
  uint32_t *column_offset;         /* [v_cap+1] local CSC offsets              */
  uint32_t *row_indices;           /* [e_cap] local src ids                    */
  uint32_t *sample_ans;            /* [e_cap] global src ids (sample_ans)      */
  uint32_t *edge_dst;              /* [e_cap] local dst of each edge (COO)     */
  uint32_t *source;                /* [s_cap] global src ids, ascending        */
  float *edge_weight_forward;      /* [e_cap] CSC order (NULL iff WEIGHT_NONE) */
  uint32_t *row_offset;            /* [s_cap+1] CSR offsets, or NULL           */
  uint32_t *column_indices;        /* [e_cap] CSR local dst ids, or NULL       */
  float *edge_weight_backward;     /* [e_cap] CSR order, or NULL               */
  uint32_t *sizes;                 /* device [4]: v_size, e_size, src_size,
                                      overflow flag (nonzero = a capacity was
                                      exceeded and the layer is truncated)     */
  uint32_t *dst_local_id;          /* [v_cap] or NULL.  Non-NULL: every dst is
                                      also put in the frontier (is_merge_src_dst,
                                      core/ntsFastSampler.hpp:1050-1052, the GAT
                                      drivers) and dst_local_id[d] = its local
                                      src id (:1095-1097; set_dst_local_index,
                                      cuda/ntsCUDAGraphOP.cu:1696).  s_cap must
                                      then allow e + v sources.               */
  uint32_t *csr_edge_id;           /* [e_cap] or NULL: CSC edge id of each CSR
                                      slot (with row_offset)                   */
  const uint32_t *omit_map;        /* [V] or NULL: a dst d with omit_map[d] ==
                                      omit_key samples no neighbours
                                      (sample_gpu_fast_omit, bottom layer of
                                      the PD-cache toolkits,
                                      core/ntsFastSampler.hpp:711-915)         */
  uint32_t omit_key;
  const uint32_t *omit_loc;        /* [V] with omit_map: the PD cache row of d */
  uint32_t *omit_row;              /* [v_cap] with omit_map: omit_loc[dst[i]]
                                      for an omitted dst i, else NTS_NOT_CACHED
                                      (the batch's own snapshot of the cache) */
  uint32_t *sizes_host;            /* NULL, or a device-visible pointer to host
                                      memory (hipHostMalloc mapped + coherent):
                                      the layer's last kernel also stores the 4
                                      sizes words there, so the host reads them
                                      after the stream's event without a D2H
                                      copy of its own                          */
} nts_sampcsc_dev;

/* ---- context ------------------------------------------------------------ */
int nts_hip_abi_version(void);
const char *nts_hip_last_error(void);
/* Replaces `new Cuda_Stream()` (cuda/ntsCUDAGraphOP.cu:201-212).  `stream` is
 * used as given; NULL is HIP's legacy default stream.  seed feeds PHILOX and
 * the MT19937 generator (reference: 2000, core/ntsFastSampler.hpp:202). */
int nts_hip_ctx_create(nts_hip_ctx **ctx, int device, void *stream, uint64_t seed);
int nts_hip_ctx_destroy(nts_hip_ctx *ctx);
/* Cuda_Stream::setNewStream (cuda/ntsCUDA.hpp:188). */
int nts_hip_ctx_set_stream(nts_hip_ctx *ctx, void *stream);
void *nts_hip_ctx_get_stream(nts_hip_ctx *ctx);
/* Pre-size the scratch arena so no allocation happens inside the hot loop
 * (keeps every call graph-capturable).  n_vertices: |V| of the graph;
 * max_items: largest e_cap / v_cap that will be passed. */
int nts_hip_ctx_reserve(nts_hip_ctx *ctx, uint64_t n_vertices, uint64_t max_items);
/* Arithmetic of the dense layer GEMMs issued through this context
 * (nts_hip_gemm_*, the bottom-layer transform): NTS_GEMM_F32 = the fp32-input
 * MFMA (one fp32 fma chain per output, the reference's fp32 GEMM semantics);
 * NTS_GEMM_SPLIT3 = fp32 operands split exactly into three bf16 pieces, the
 * six significant piece products on the bf16 MFMA with fp32 accumulation
 * (error vs fp64 of the same order as the fp32 path; csrc/gemm3.hip) for
 * the GEMMs whose reduction (NN) or output rows (TN) span >= 256 — narrower
 * ones run faster on the fp32 path and take it; NTS_GEMM_SPLIT3_ALL = the
 * split kernels for every shape they take (kernel tests).  Shapes the split
 * kernels do not take run on the fp32 path. */
#define NTS_GEMM_F32 0
#define NTS_GEMM_SPLIT3 1
#define NTS_GEMM_SPLIT3_ALL 2
int nts_hip_ctx_set_gemm_mode(nts_hip_ctx *ctx, int mode);
int nts_hip_ctx_get_gemm_mode(nts_hip_ctx *ctx);
/* Re-seed the MT19937 state (std::mt19937(seed)).  Enqueued on the stream. */
int nts_hip_rng_seed(nts_hip_ctx *ctx, uint64_t seed);
/* Copy the MT19937 state (624 words + position) to host; synchronises. */
int nts_hip_rng_state(nts_hip_ctx *ctx, uint32_t *host_state625);
/* MT19937 modes, recovery from a short stream (no reference counterpart: the
 * reference's CPU generator, core/ntsFastSampler.hpp:200-205, is unbounded;
 * the device replay generates each layer's words ahead up to a bound).
 * A layer whose draws pass its bound reports it (sizes[3] bit 2) and leaves
 * the generator where the layer began; the caller rewinds to the batch's
 * checkpoint, scales the bound up and samples the batch again — bit-exact,
 * the stream is the same.
 *   nts_hip_mt_budget_scale: multiply every later layer's word bound by
 *     `scale` (> 0; 1 = the coupon-collector mean x 1.05 + 131,072 words).
 *   nts_hip_mt_checkpoint: enqueue (on the context's stream) a copy of the
 *     generator state (625 u32: 624 words + position) into the DEVICE buffer
 *     `dev_state625` — taken before a batch's first layer.
 *   nts_hip_mt_rewind: synchronise the context's streams, make
 *     `dev_state625` the generator state and restart the word ring from it. */
int nts_hip_mt_budget_scale(nts_hip_ctx *ctx, double scale);
int nts_hip_mt_checkpoint(nts_hip_ctx *ctx, uint32_t *dev_state625);
int nts_hip_mt_rewind(nts_hip_ctx *ctx, const uint32_t *dev_state625);

/* ---- graph preprocessing ----------------------------------------------- */
/* Degrees from an edge list, clamped to >= 1:
 * Graph::load_directed (core/graph.hpp:1157-1186 out, :1420-1425 in) +
 * generate_backward_structure clamp (core/graph.hpp:4525-4530). */
int nts_hip_degrees(nts_hip_ctx *ctx, const uint32_t *src, const uint32_t *dst,
                    uint64_t n_edges, uint64_t n_vertices, uint32_t *out_degree,
                    uint32_t *in_degree);
/* Global CSC keyed by dst, src ids in edge-list (file) order within each dst:
 * FullyRepGraph::ReadRepGraphFromRawFile (core/FullyRepGraph.hpp:724-798). */
int nts_hip_build_csc(nts_hip_ctx *ctx, const uint32_t *src, const uint32_t *dst,
                      uint64_t n_edges, uint64_t n_vertices, uint64_t *column_offset,
                      uint32_t *row_indices);

/* ---- sampler ------------------------------------------------------------ */
/* One hop of FastSampler::sample_fast / sample_gpu_fast
 * (core/ntsFastSampler.hpp:962-1140, :648-709):
 *   num_d = min(deg(d), fanout) (fanout < 0: all), draw num_d distinct
 *   neighbour positions by rejection (deg > fanout) or take all in CSC order,
 *   frontier = distinct sampled ids in ascending global order (source),
 *   row_indices relabelled to local ids, CSR transpose (csc_to_csr,
 *   core/coocsc.hpp:82-111, stable = ascending dst) and edge weights
 *   (WeightCompute, core/coocsc.hpp:301-324).  Replaces
 *   sample_processing_get_co_gpu + sample_processing_traverse_gpu +
 *   sample_processing_update_ri_gpu + GetWeight (cuda/ntsCUDAGraphOP.cu:1246-1700).
 * batch_seq/layer key the PHILOX stream; MT modes ignore them. */
int nts_hip_sample_layer(nts_hip_ctx *ctx, const nts_graph_dev *graph, int fanout,
                         int layer, uint64_t batch_seq, int rng_mode, int weight_type,
                         nts_sampcsc_dev *out);

/* ---- feature / label movement ------------------------------------------- */
/* out[i,:] = table[index[i],:] for i < *n (n == NULL: n_cap rows).
 * Replaces zero_copy_feature_move_gpu (cuda/ntsCUDAGraphOP.cu:1711-1729) and
 * nts::op::get_feature (core/ntsMiniBatchGraphOp.hpp:45-60); the table is
 * HBM-resident instead of pinned host memory; 64-bit row offsets. */
int nts_hip_gather_rows(nts_hip_ctx *ctx, const float *table, uint64_t ld_table,
                        const uint32_t *index, const uint32_t *n, uint32_t n_cap,
                        uint32_t feature_size, float *out, uint64_t ld_out);
/* out[i] = labels[index[i]]: global_copy_label_move_gpu (cuda/ntsCUDAGraphOP.cu,
 * kernel cuda/ntsCUDATransferKernel.cuh:203-212) / get_label (core/ntsMiniBatchGraphOp.hpp:36-43). */
int nts_hip_gather_labels(nts_hip_ctx *ctx, const int64_t *labels, const uint32_t *index,
                          const uint32_t *n, uint32_t n_cap, int64_t *out);

/* ---- HBM feature cache + host-pinned spill -------------------------------- */
/* The reference keeps the feature table in pinned host memory and caches the
 * rows of the highest-degree vertices on the GPU (GS_SAMPLE_PD_CACHE:
 * determine_cache_node_idx / cache_high_degree / mark_cache_node,
 * toolkits/GS_SAMPLE_PD_CACHE.hpp:1019-1112).  On MI355X every BASELINE
 * config fits HBM, so this two-tier table is the path for tables that do not.
 *
 * Selection: cache_map[v] = slot of v if v is among the n_cache vertices of
 * largest out_degree (ties: ascending id), else NTS_NOT_CACHED;
 * cache_ids[slot] = v (may be NULL when n_cache == 0).  Slots follow the
 * (degree descending, id ascending) order.  n_vertices < 2^31.  Fill the
 * cache with nts_hip_gather_rows(table, cache_ids -> cache). */
#define NTS_NOT_CACHED 0xFFFFFFFFu
int nts_hip_cache_select(nts_hip_ctx *ctx, const uint32_t *out_degree, uint64_t n_vertices,
                         uint64_t n_cache, uint32_t *cache_map, uint32_t *cache_ids);
/* Pinned host memory mapped into the device address space (coarse-grained),
 * for the spilled feature table (cudaMallocPinned, core/ntsDataloador.hpp:483). */
int nts_hip_host_alloc(uint64_t bytes, void **host_ptr);
int nts_hip_host_free(void *host_ptr);
int nts_hip_host_device_pointer(void *host_ptr, void **dev_ptr);
/* load_feature_gpu_cache (core/ntsFastSampler.hpp:263-317; kernels
 * cuda/ntsCUDATransferKernel.cuh:154-183) in one pass:
 *   out[i,:] = cache_map[index[i]] != NTS_NOT_CACHED ? cache[cache_map[index[i]],:]
 *                                                   : host_table[index[i],:]
 * host_table: device-visible pointer of the pinned host table (zero-copy). */
int nts_hip_gather_rows_cached(nts_hip_ctx *ctx, const float *cache, uint64_t ld_cache,
                               const uint32_t *cache_map, const float *host_table,
                               uint64_t ld_host, const uint32_t *index, const uint32_t *n,
                               uint32_t n_cap, uint32_t feature_size, float *out,
                               uint64_t ld_out);

/* ---- sampled aggregation ------------------------------------------------ */
/* Y[d,:] = sum_{e in [co[d],co[d+1])} w[e] * X[row(e),:], summed in CSC edge
 * order as (x*w)+acc with no FMA contraction — the exact arithmetic of
 * MiniBatchFuseOp::forward / nts_comp (core/ntsMiniBatchGraphOp.hpp:153-182,
 * core/ntsBaseOp.hpp:546-562).  row(e) = row_indices[e], or
 * x_row_map[row_indices[e]] when x_row_map != NULL (fused feature gather:
 * X is then the global feature table and x_row_map the layer's `source`).
 * Every row d < *v is written (no pre-zeroing needed).  Replaces
 * Gather_By_Dst_From_Src(_Spmm) (cuda/ntsCUDAGraphOP.cu:340-373,425-587). */
int nts_hip_spmm_csc_fwd(nts_hip_ctx *ctx, const uint32_t *column_offset,
                         const uint32_t *row_indices, const float *weight,
                         const uint32_t *v, uint32_t v_cap, const float *x, uint64_t ldx,
                         const uint32_t *x_row_map, uint32_t feature_size, float *y,
                         uint64_t ldy);
/* Stage the NON-cached rows of a layer's sources once into HBM:
 *   stage[i,:] = host_table[index[i],:]  for every i with cache_map[index[i]] ==
 *   NTS_NOT_CACHED (other rows of stage are left untouched).
 * The host link then carries each distinct spilled row once per batch
 * instead of once per sampled edge. */
int nts_hip_stage_uncached_rows(nts_hip_ctx *ctx, const uint32_t *cache_map,
                                const float *host_table, uint64_t ld_host, const uint32_t *index,
                                const uint32_t *n, uint32_t n_cap, uint32_t feature_size,
                                float *stage, uint64_t ld_stage);
/* nts_hip_spmm_csc_fwd with the fused feature gather reading the two-tier
 * table: for local src r = row_indices[e] and g = x_row_map[r], the row comes
 * from cache[cache_map[g],:] when cached, else from spill[host_local ? r : g,:]
 * — the pinned host table (host_local = 0) or the rows staged by
 * nts_hip_stage_uncached_rows (host_local = 1).  load_feature_gpu_cache + the
 * bottom graph op; bit-identical to nts_hip_spmm_csc_fwd on the full table
 * for every cache content. */
int nts_hip_spmm_csc_fwd_cached(nts_hip_ctx *ctx, const uint32_t *column_offset,
                                const uint32_t *row_indices, const float *weight,
                                const uint32_t *v, uint32_t v_cap, const float *cache,
                                uint64_t ld_cache, const uint32_t *cache_map,
                                const float *spill, uint64_t ld_spill, int host_local,
                                const uint32_t *x_row_map, uint32_t feature_size, float *y,
                                uint64_t ldy);
/* G_in[s,:] = sum_{j in [ro[s],ro[s+1])} w_b[j] * G_out[ci[j],:] (ascending dst
 * order, deterministic, atomic-free).  Replaces Gather_By_Src_From_Dst_Spmm
 * (cuda/ntsCUDAGraphOP.cu:901-1042) and MiniBatchFuseOp::backward
 * (core/ntsMiniBatchGraphOp.hpp:214-268). */
int nts_hip_spmm_csr_bwd(nts_hip_ctx *ctx, const uint32_t *row_offset,
                         const uint32_t *column_indices, const float *weight_backward,
                         const uint32_t *s, uint32_t s_cap, const float *g_out,
                         uint64_t ld_gout, uint32_t feature_size, float *g_in,
                         uint64_t ld_gin);
/* nts_hip_spmm_csr_bwd that also leaves its output's column maxima per part
 * of R = nts_hip_csr_bwd_colmax_rows_per_part(feature_size) rows:
 * part_max[p * feature_size + c] = the float bits of max |rs(s) G_in[s, c]|
 * over s in [p R, (p+1) R) (0 past the live rows; exact — an unordered max),
 * ceil(s_cap / R) parts, with the row scale rs(s) = row_scale[row_map[s]]
 * (row_map NULL: row_scale[s]; row_scale NULL: 1).  With the pair table's row
 * scales and the GEMM's row map these are exactly the operand maxima
 * nts_hip_gemm_h2p_tn_gather_cm takes when G_in is its B, so that GEMM reads
 * G_in once.  feature_size <= 512, G rows 16-byte aligned with ld % 4 == 0. */
uint32_t nts_hip_csr_bwd_colmax_rows_per_part(uint32_t feature_size);
int nts_hip_spmm_csr_bwd_colmax(nts_hip_ctx *ctx, const uint32_t *row_offset,
                                const uint32_t *column_indices, const float *weight_backward,
                                const uint32_t *s, uint32_t s_cap, const float *g_out,
                                uint64_t ld_gout, uint32_t feature_size, float *g_in,
                                uint64_t ld_gin, uint32_t *part_max, const float *row_scale,
                                const uint32_t *row_map);
/* Transform-first bottom layer: when the layer narrows the rows
 * (F_in > F_out), A (X W) replaces (A X) W — the reference aggregates first
 * (SingleGPUAllSampleGraphOp::forward then Parameter::forward,
 * toolkits/GCN_SAMPLE_GPU.hpp:252-266); both are linear, so they agree up to
 * fp32 summation order.  The aggregation then runs over F_out-wide rows and
 * vertexForward's activation moves into its epilogue:
 *   y = dropout(relu(A x), p) with the Philox keep bits of
 *   nts_hip_gemm_relu_dropout_f32 (same seed/offset/(row, col) keys, so both
 *   orders drop the same elements); p == 0: relu only.  A, weights, v as in
 *   nts_hip_spmm_csc_fwd (no row map). */
int nts_hip_spmm_csc_fwd_act(nts_hip_ctx *ctx, const uint32_t *column_offset,
                             const uint32_t *row_indices, const float *weight, const uint32_t *v,
                             uint32_t v_cap, const float *x, uint64_t ldx, uint32_t feature_size,
                             float *y, uint64_t ldy, float p, uint64_t seed, uint64_t offset);
/* Its backward through the CSR, the activation's backward fused into the loads:
 *   G_in[s,:] = sum_j w_b[j] * (G_out[ci[j],:] ⊙ [X_act[ci[j],:] > 0] * scale)
 * (X_act = the forward output of nts_hip_spmm_csc_fwd_act, scale = 1/(1-p));
 * ascending dst order, deterministic. */
int nts_hip_spmm_csr_bwd_masked(nts_hip_ctx *ctx, const uint32_t *row_offset,
                                const uint32_t *column_indices, const float *weight_backward,
                                const uint32_t *s, uint32_t s_cap, const float *g_out,
                                uint64_t ld_gout, const float *x_act, uint64_t ld_act, float scale,
                                uint32_t feature_size, float *g_in, uint64_t ld_gin);
/* A graph-op backward whose result feeds that activation's backward:
 *   G_in[s,:] = (sum_j w_b[j] * G_out[ci[j],:]) ⊙ [X_act[s,:] > 0] * scale
 * — nts_hip_spmm_csr_bwd followed by nts_hip_act_backward on its output, in
 * one pass, the same arithmetic (the mask is read once per output row). */
int nts_hip_spmm_csr_bwd_postmask(nts_hip_ctx *ctx, const uint32_t *row_offset,
                                  const uint32_t *column_indices, const float *weight_backward,
                                  const uint32_t *s, uint32_t s_cap, const float *g_out,
                                  uint64_t ld_gout, const float *x_act, uint64_t ld_act, float scale,
                                  uint32_t feature_size, float *g_in, uint64_t ld_gin);
/* The same pair with the activation's keep mask [X_act > 0] carried as bits
 * instead of re-read from X_act's rows (16 bytes a 128-float row instead of
 * 512): nts_hip_act_bits_words(F) words per row (0: F unsupported — F must be
 * a multiple of 4 from 68 to 2048; the caller then uses the float forms),
 * 16-byte aligned.
 * nts_hip_spmm_csc_fwd_act_bits = nts_hip_spmm_csc_fwd_act that also writes
 * mask_bits[v_cap rows]; nts_hip_spmm_csr_bwd_postmask_bits =
 * nts_hip_spmm_csr_bwd_postmask reading those bits (X_act's rows = g_in's
 * rows).  Results identical to the float forms. */
uint32_t nts_hip_act_bits_words(uint32_t feature_size);
int nts_hip_spmm_csc_fwd_act_bits(nts_hip_ctx *ctx, const uint32_t *column_offset,
                                  const uint32_t *row_indices, const float *weight,
                                  const uint32_t *v, uint32_t v_cap, const float *x, uint64_t ldx,
                                  uint32_t feature_size, float *y, uint64_t ldy, float p,
                                  uint64_t seed, uint64_t offset, uint32_t *mask_bits);
int nts_hip_spmm_csr_bwd_postmask_bits(nts_hip_ctx *ctx, const uint32_t *row_offset,
                                       const uint32_t *column_indices,
                                       const float *weight_backward, const uint32_t *s,
                                       uint32_t s_cap, const float *g_out, uint64_t ld_gout,
                                       const uint32_t *mask_bits, float scale,
                                       uint32_t feature_size, float *g_in, uint64_t ld_gin);
/* The activation's backward alone: out = g ⊙ [x_act > 0] * scale ([rows x
 * feature_size], each with its leading dimension) — what libtorch's relu and
 * dropout backward compute for vertexForward (toolkits/GCN_SAMPLE_GPU.hpp:252-266),
 * in one pass; followed by nts_hip_spmm_csr_bwd it equals
 * nts_hip_spmm_csr_bwd_masked (same arithmetic per element). */
int nts_hip_act_backward(nts_hip_ctx *ctx, uint32_t rows, uint32_t feature_size, const float *g,
                         uint64_t ldg, const float *x_act, uint64_t ldx, float scale, float *out,
                         uint64_t ldo);
/* G_in[row_indices[e],:] += w[e] * G_out[d,:] with float atomics over the CSC
 * (g_in must be zeroed by the caller; summation order is not deterministic).
 * Replaces Push_From_Dst_To_Src_Spmm (cuda/ntsCUDAGraphOP.cu:621-770). */
int nts_hip_spmm_csc_bwd_atomic(nts_hip_ctx *ctx, const uint32_t *column_offset,
                                const uint32_t *row_indices, const float *weight,
                                const uint32_t *v, uint32_t v_cap, const float *g_out,
                                uint64_t ld_gout, uint32_t feature_size, float *g_in,
                                uint64_t ld_gin);

/* ---- NeutronOrch PD cache (toolkits/GCN_SAMPLE_PD_CACHE.hpp) -------------- */
/* preSample's hot-vertex count (get_most_neighbor, core/ntsBaseOp.hpp:330-404):
 * old[seeds[i]] = 1; then (layers - 1) times new[u] += old[v] for every
 * in-neighbour u of v in the CSC (column_offset[v] .. [v+1]); counts = the
 * last `new` (all zeros when layers == 1, as the reference's).  tmp: [V]. */
int nts_hip_presample_counts(nts_hip_ctx *ctx, const nts_graph_dev *graph, const uint32_t *seeds,
                             uint32_t n_seeds, int layers, uint32_t *counts, uint32_t *tmp);
/* ... and its selection: total = (number of non-zero counts) + 1 (V when none
 * is zero), n = (uint32)((float)total * cache_rate) (clamped to V), pivot =
 * the n-th largest count (0-based, descending), out_ids = the first n vertex
 * ids in ascending order whose count >= pivot (the reference's single-thread
 * order), *out_n = n (device scalar).  out_ids: [V]. */
int nts_hip_presample_select(nts_hip_ctx *ctx, const uint32_t *counts, uint64_t n_vertices,
                             float cache_rate, uint32_t *out_ids, uint32_t *out_n);
/* set_cache_index for one super-batch: cache_map[ids[i]] = key,
 * cache_location[ids[i]] = i for i < n (gnndatum->set_cache_index). */
int nts_hip_pd_set_cache(nts_hip_ctx *ctx, const uint32_t *ids, uint32_t n, uint32_t key,
                         uint32_t *cache_map, uint32_t *cache_location);
/* load_share_embedding (dev_load_share_embedding_kernel,
 * cuda/ntsCUDATransferKernel.cuh:454-500): for the bottom layer's dsts
 * i < *v, emb[i,:] = share[omit_row[i],:] when omit_row[i] != NTS_NOT_CACHED
 * (omit_row: written by nts_hip_sample_layer with omit_map; rows of other dsts
 * untouched).  The reference tests cache_map[dst[i]] == super_batch_id at
 * this point; the sampled layer's own record is the same decision, taken when
 * it was sampled, so a later super-batch may already reuse cache_map. */
int nts_hip_pd_load_share(nts_hip_ctx *ctx, const uint32_t *omit_row, const uint32_t *v,
                          uint32_t v_cap, const float *share, uint64_t ld_share,
                          uint32_t feature_size, float *emb, uint64_t ld_emb);
/* vertexForward's activation alone, y = dropout(relu(x), p) with the keep
 * bits of nts_hip_gemm_relu_dropout_f32 (same seed/offset/(row, col) keys):
 * after a GEMM whose rows are replaced by the PD cache. */
int nts_hip_relu_dropout_f32(nts_hip_ctx *ctx, uint32_t rows, uint32_t feature_size,
                             const float *x, uint64_t ldx, float p, uint64_t seed,
                             uint64_t offset, float *y, uint64_t ldy);

/* ---- GAT layer on a merged src/dst sampled block ------------------------- */
/* The GAT_SAMPLE_ALL_GPU layer (toolkits/GAT_SAMPLE_ALL_GPU.hpp:308-391:
 * BatchGPUSrcDstScatterOp -> leaky_relu(msg . W_att, 0.2) -> BatchGPUEdgeSoftMax
 * -> e_msg * a -> BatchGPUAggregateDst -> relu; core/ntsPushdownGraphOp.hpp:490-748)
 * without materialising the [e, 2F] messages.  H = X W [src_size x F] is the
 * layer's transformed input (caller's GEMM); att = W_att [2F] (a1 = att[0:F]
 * for the source half, a2 = att[F:2F] for the destination half).  Forward:
 *   m[e] = leaky_relu(H[src_e].a1 + H[dst_local(d)].a2, 0.2),
 *   a[e] = softmax over the edges of d of m,  Y[d] = relu(sum_e a[e] H[src_e]).
 * One wave per destination, online softmax (running max/sum), edge order. */
int nts_hip_gat_forward(nts_hip_ctx *ctx, const uint32_t *column_offset,
                        const uint32_t *row_indices, const uint32_t *dst_local_id,
                        uint32_t v_size, const float *H, uint64_t ldh, uint32_t F,
                        const float *att, float *m_out, float *a_out, float *Y, uint64_t ldy);
/* Its backward for dL/dY = GY (deterministic: a per-destination pass and a
 * per-source pass over the CSR with csr_edge_id; no atomics):
 *   du[e] = dL/d(pre-leaky score of e), ds2[v] = dL/d(H[v].a2) (zero for
 *   non-destinations), GM [v_size x F] = GY masked by Y > 0 (scratch, ld ldm),
 *   dH [src_size x F] = dL/dH, dS [src_size x 2] =
 *   (dL/d(H[v].a1), dL/d(H[v].a2)) so that dW_att = H^T dS (caller's GEMM). */
int nts_hip_gat_backward(nts_hip_ctx *ctx, const uint32_t *column_offset,
                         const uint32_t *row_indices, const uint32_t *dst_local_id,
                         uint32_t v_size, const uint32_t *row_offset,
                         const uint32_t *column_indices, const uint32_t *csr_edge_id,
                         uint32_t src_size, const float *H, uint64_t ldh, uint32_t F,
                         const float *att, const float *a, const float *m, const float *Y,
                         uint64_t ldy, const float *GY, uint64_t ldg, float *du, float *ds2,
                         float *GM, uint64_t ldm, float *dH, uint64_t lddh, float *dS);

/* ---- dense layer update (MFMA fp32) -------------------------------------- */
/* Row-major fp32 GEMM on the matrix cores (v_mfma_f32_16x16x4_f32 /
 * v_mfma_f32_32x32x2_f32, exact fp32 products, fp32 accumulate):
 *  trans_a == 0: C[M,N] = A[M,K] B[K,N]   — Parameter::forward x.matmul(W)
 *                (core/NtsScheduler.hpp:859-862)
 *  trans_a != 0: C[M,N] = A[K,M]^T B[K,N] — the weight gradient Y^T dZ that
 *                libtorch's matmul backward computes for it.
 * Long reductions are split over blocks and summed in a fixed order
 * (deterministic).  May grow the context's scratch arena. */
int nts_hip_gemm_f32(nts_hip_ctx *ctx, int trans_a, int M, int N, int K, const float *A,
                     uint64_t lda, const float *B, uint64_t ldb, float *C, uint64_t ldc);

/* Row-gathered forms for the transform-first bottom layer (A = the feature
 * table, a_rows = the layer's `source`, so the gathered rows never land in HBM
 * — the fused load_feature_gpu of core/ntsFastSampler.hpp:244-261):
 *   nts_hip_gemm_gather_f32:    C[i,:] = A[a_rows[i],:] B        (i < M; A rows of K floats)
 *   nts_hip_gemm_tn_gather_f32: C[M,N] = A[a_rows[0..K),:]^T B[K,N] (A rows of M floats)
 * Same kernels and summation order as nts_hip_gemm_f32 on the gathered matrix
 * (bit-identical to it). */
int nts_hip_gemm_gather_f32(nts_hip_ctx *ctx, int M, int N, int K, const float *A, uint64_t lda,
                            const uint32_t *a_rows, const float *B, uint64_t ldb, float *C,
                            uint64_t ldc);
int nts_hip_gemm_tn_gather_f32(nts_hip_ctx *ctx, int M, int N, int K, const float *A,
                               uint64_t lda, const uint32_t *a_rows, const float *B, uint64_t ldb,
                               float *C, uint64_t ldc);

/* Two-piece f16 forms of the two GEMMs above (csrc/gemmh2.hip), for a STATIC
 * A table pre-split once ("pair table"): row r is scaled by a power of two
 * rs[r] so that its largest |x| / rs[r] lies in [2^14, 2^15), and each
 * x / rs[r] is stored as one 32-bit word = f16 y0 (low half) + f16 y1 (high
 * half), y0 = f16(y), y1 = f16(y - y0): 22 significant bits.  Products run as
 * y0 b0 + y0 b1 + y1 b0 on the f16 MFMA with fp32 accumulation (three MFMAs
 * per k-slice where NTS_GEMM_SPLIT3 needs six), the scales applied exactly
 * to the fp32 result: error vs fp64 within a small factor of the fp32 GEMM's
 * (tests/test_gemm_h2.py).  Same operations as nts_hip_gemm_gather_f32 /
 * nts_hip_gemm_tn_gather_f32 on the transform-first bottom layer
 * (toolkits/GCN_SAMPLE_ALLGPU.hpp:247-266 x.matmul(W) and its weight gradient).
 *   nts_hip_h2_split_rows:  X [R x K] (ld ldx) -> P [R x Kp] words (ld ldp,
 *                           Kp % 32 == 0, zero past K) + rs [R]
 *   nts_hip_gemm_h2_gather: C[i,:] = act(X[a_rows[i],:] W) with X given as
 *                           (P, rs); W [K x N] fp32 (N % 16 == 0, N <= 1024);
 *                           relu_dropout != 0: the fused relu + inverted
 *                           dropout of nts_hip_gemm_relu_dropout_f32 (same
 *                           mask bits); a_rows NULL = rows 0..M-1
 *   nts_hip_gemm_h2_tn_gather: C[M,N] = X[a_rows[0..K),:M]^T op(B[K,N]),
 *                           op(B) = B, or B * bscale where Xm > 0 when Xm != NULL
 * May grow the context's scratch arena. */
int nts_hip_h2_split_rows(nts_hip_ctx *ctx, uint64_t R, uint32_t K, const float *X, uint64_t ldx,
                          uint32_t Kp, uint32_t *P, uint64_t ldp, float *rs);
int nts_hip_gemm_h2_gather(nts_hip_ctx *ctx, int relu_dropout, int M, int N, int Kp,
                           const uint32_t *P, uint64_t ldp, const float *rs, const uint32_t *a_rows,
                           const float *W, uint64_t ldw, int K, float *C, uint64_t ldc, float p,
                           uint64_t seed, uint64_t offset);
int nts_hip_gemm_h2_tn_gather(nts_hip_ctx *ctx, int M, int N, int K, const uint32_t *P, uint64_t ldp,
                              const float *rs, const uint32_t *a_rows, const float *B, uint64_t ldb,
                              const float *Xm, uint64_t ldx, float bscale, float *C, uint64_t ldc);
/* The same weight gradient on a "planar" pair table (per row the y0 plane of
 * Kp f16, then the y1 plane; row scales as above), whole rows streamed once by
 * LDS DMA, every output row in one block (csrc/gemmh2.hip k_h2_tn3):
 * N % 128 == 0, M <= 640, M <= Kp <= 640. */
int nts_hip_h2_split_rows_planar(nts_hip_ctx *ctx, uint64_t R, uint32_t K, const float *X,
                                 uint64_t ldx, uint32_t Kp, uint16_t *Q, uint64_t ldq, float *rs);
int nts_hip_gemm_h2p_tn_gather(nts_hip_ctx *ctx, int M, int N, int K, const uint16_t *Q, uint64_t ldq,
                               int Kp, const float *rs, const uint32_t *a_rows, const float *B,
                               uint64_t ldb, float *C, uint64_t ldc);
/* The same with per-part column maxima of |rs[a_rows[k]] B[k, c]| given
 * (part p = B rows [p R, (p+1) R), N words per part —
 * nts_hip_spmm_csr_bwd_colmax's output with row_scale = rs and row_map =
 * a_rows, R = rows_per_part): each k-chunk's column scales come from the
 * parts that cover its rows, with no pre-pass over B in the kernel. */
int nts_hip_gemm_h2p_tn_gather_cm(nts_hip_ctx *ctx, int M, int N, int K, const uint16_t *Q,
                                  uint64_t ldq, int Kp, const float *rs, const uint32_t *a_rows,
                                  const float *B, uint64_t ldb, float *C, uint64_t ldc,
                                  const uint32_t *part_max, uint32_t rows_per_part);
/* The forward GEMM on the planar table (k_h2_nn3: W's 16-column slices held
 * in registers, 16-row tiles of whole rows by LDS DMA): N % 128 == 0,
 * K <= Kp <= 640; arguments as nts_hip_gemm_h2_gather. */
int nts_hip_gemm_h2p_gather(nts_hip_ctx *ctx, int relu_dropout, int M, int N, int Kp, const uint16_t *Q,
                            uint64_t ldq, const float *rs, const uint32_t *a_rows, const float *W,
                            uint64_t ldw, int K, float *C, uint64_t ldc, float p, uint64_t seed,
                            uint64_t offset);

/* Layer forward on a dynamic fp32 input with at most 128 columns (the
 * aggregate-first layer of the products / papers-shaped configs, 100 or 128
 * -> 256): C = act(A W), A split into f16 pairs with power-of-two row scales
 * inside the kernel, W into pairs with column scales, 3 f16 MFMA products,
 * fp32 accumulate (the pair-table arithmetic of nts_hip_gemm_h2p_gather).
 * relu_dropout: the activation of nts_hip_gemm_relu_dropout_f32 (same Philox
 * keys, so the same elements are dropped).  K <= 128 with K % 4 == 0, A rows
 * 16-byte aligned, N 128 or 256.  Q != NULL: A's planar pair table
 * (rows of 2 Kp f16, Kp = K rounded up to 32) and row scales rs[M] are also
 * written (the weight gradient's operand). */
int nts_hip_gemm_h2d_act(nts_hip_ctx *ctx, int relu_dropout, int M, int N, int K, const float *A,
                         uint64_t lda, const float *W, uint64_t ldw, float *C, uint64_t ldc, float p,
                         uint64_t seed, uint64_t offset, uint16_t *Q, uint64_t ldq, float *rs);

/* Hidden-layer forward with its activation fused into the GEMM epilogue:
 *   C = dropout(relu(A B), p)   — vertexForward's
 *   torch::dropout(torch::relu(x.matmul(W)), drop_rate, training)
 *   (toolkits/GCN_SAMPLE_GPU.hpp:252-266).  Inverted dropout: kept elements
 *   are scaled by 1/(1-p); keep(row, col) comes from Philox4x32-10 keyed by
 *   `seed`, counter {row/4, col/2, offset}: 16 bits per element (word row%4,
 *   low half for even col, high half for odd col) >= floor(p*2^16), so the
 *   mask is reproducible and never stored.  p == 0: plain relu (eval). */
int nts_hip_gemm_relu_dropout_f32(nts_hip_ctx *ctx, int M, int N, int K, const float *A,
                                  uint64_t lda, const float *B, uint64_t ldb, float *C,
                                  uint64_t ldc, float p, uint64_t seed, uint64_t offset);

/* Its weight gradient: C[M,N] = A[K,M]^T (B ⊙ [X > 0] · scale), with B = dX
 * (the gradient of the layer output) and X the forward output, scale =
 * 1/(1-p): the relu and dropout backward fused into the operand load. */
int nts_hip_gemm_tn_masked_f32(nts_hip_ctx *ctx, int M, int N, int K, const float *A,
                               uint64_t lda, const float *B, uint64_t ldb, const float *X,
                               uint64_t ldx, float scale, float *C, uint64_t ldc);

/* ---- output layer + loss (fused) ------------------------------------------ */
/* Training forward of the last layer and the loss, in the reference's
 * arithmetic: logits = Y W, log_softmax (vertexForward,
 * toolkits/GCN_SAMPLE_ALLGPU.hpp:247-252), log_softmax again + mean
 * nll_loss (Loss, :214-222).  Y [n x K] (ld ldy), W [K x C] row-major,
 * labels int64 [n] in [0, C), C <= 64.  Writes the scalar loss (device).
 * correct != NULL: *correct += the rows whose argmax (first index of the
 * largest log_softmax value) is the label — getCorrect
 * (toolkits/GCN_SAMPLE_ALLGPU.hpp:166-172) accumulated on the device.
 * Replaces the libtorch matmul/log_softmax/nll_loss kernels of those lines. */
int nts_hip_linear_xent_fwd(nts_hip_ctx *ctx, const float *Y, uint64_t ldy, int n, int K,
                            const float *W, int C, const int64_t *labels, float *loss,
                            uint32_t *correct);
/* Its backward for an upstream gradient *grad_loss (device scalar):
 * dY [n x K] (ld K) and dW [K x C] (row-major), i.e. what libtorch's
 * autograd produces through nll_loss, both log_softmaxes and the matmul.
 * Deterministic (fixed-order reductions). */
int nts_hip_linear_xent_bwd(nts_hip_ctx *ctx, const float *Y, uint64_t ldy, int n, int K,
                            const float *W, int C, const int64_t *labels,
                            const float *grad_loss, float *dY, float *dW);

/* Training call of the same layer: the loss AND its gradients dY, dW for an
 * upstream gradient of exactly 1 (Loss followed by loss.backward(),
 * toolkits/GCN_SAMPLE_ALLGPU.hpp:214-222 + core/ntsContext.hpp:436-440), in
 * one pass over Y.  Bit-identical to nts_hip_linear_xent_fwd followed by
 * nts_hip_linear_xent_bwd with *grad_loss == 1. */
int nts_hip_linear_xent_train(nts_hip_ctx *ctx, const float *Y, uint64_t ldy, int n, int K,
                              const float *W, int C, const int64_t *labels, float *loss,
                              float *dY, float *dW, uint32_t *correct);

/* ---- optimiser ---------------------------------------------------------- */
/* Fused Adam step on one parameter (n elements), element-wise identical to
 *  bias_correction != 0: Parameter::learnC2C_with_decay_Adam (core/NtsScheduler.hpp:863-880)
 *  bias_correction == 0: Parameter::learn_local_with_decay_Adam (core/NtsScheduler.hpp:937-945)
 * beta1_t/beta2_t are the running powers kept by Parameter::next(). */
int nts_hip_adam(nts_hip_ctx *ctx, float *w, const float *grad, float *m, float *v,
                 uint64_t n, float alpha, float beta1, float beta2, float epsilon,
                 float weight_decay, float beta1_t, float beta2_t, int bias_correction);

/* ---- RCCL over xGMI (replaces NCCL_Communicator, cuda/ntsCUDA.hpp:132-175,
 *      cuda/ntsCUDAGraphOP.cu:173-200) --------------------------------------- */
int nts_hip_comm_unique_id(uint8_t out_id[128]);
/* One communicator per process/GPU (ncclCommInitRank) instead of the
 * reference's single-process ncclCommInitAll clique. */
int nts_hip_comm_init(nts_hip_comm **comm, int nranks, int rank, const uint8_t id[128],
                      int device);
int nts_hip_comm_destroy(nts_hip_comm *comm);
/* Ranks in the communicator as RCCL itself reports them (ncclCommCount) and
 * this process's rank (ncclCommUserRank): the check that an N-process launch
 * really built one N-rank clique (the reference's ncclCommInitAll over
 * `device_num` GPUs, toolkits/GCN_SAMPLE_ALL_MULTI.hpp:89-113). */
int nts_hip_comm_count(nts_hip_comm *comm, int *nranks, int *rank);
/* In-place float SUM all-reduce (NCCL_Communicator::AllReduce, cuda/ntsCUDAGraphOP.cu:180-186). */
int nts_hip_allreduce_sum_f32(nts_hip_comm *comm, float *buf, uint64_t count, void *stream);
/* In-place broadcast from root (NCCL_Communicator::Bcast, cuda/ntsCUDAGraphOP.cu:188-193). */
int nts_hip_broadcast_f32(nts_hip_comm *comm, float *buf, uint64_t count, int root,
                          void *stream);

#ifdef __cplusplus
}
#endif
#endif /* NTS_HIP_H */
