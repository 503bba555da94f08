// NeutronOrch PD cache on the device (toolkits/GCN_SAMPLE_PD_CACHE.hpp).
//
// The reference splits each super-batch (PIPELINE_NUM mini-batches) between
// the CPU and the GPU: preSample picks the super-batch's hot vertices (the
// most reached L-1 hops out from its seeds, get_most_neighbor,
// core/ntsBaseOp.hpp:330-404), a CPU thread computes their bottom-layer
// embedding (PushDownBatchOp + X W, :740-840), the GPU skips sampling their
// bottom-layer neighbourhoods (sample_gpu_fast_omit) and overwrites their rows
// of the first layer's X W with the CPU's (load_share_embedding).  Here every
// part runs on the GPU; these are the kernels only it needs:
//   k_presample_push / select  — get_most_neighbor's counts and selection
//   k_pd_set_cache             — set_cache_index (cache_map, cache_location)
//   k_pd_load_share            — dev_load_share_embedding_kernel
//   k_relu_dropout             — vertexForward's activation after the overwrite
// The omitted sampling itself is count_scan's omit_map (primitives.hip, sampler.hip).
#include "common.hpp"

namespace nts_hip {

__global__ void k_presample_seed(const uint32_t* __restrict__ seeds, uint32_t n,
                                 uint32_t* __restrict__ cnt) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    cnt[seeds[i]] = 1;
}

// new[u] += old[v] for every in-neighbour u of v with old[v] > 0: one wave per
// v (lanes stride its CSC segment; hubs have tens of thousands of entries);
// integer atomics, so the result does not depend on the order
__global__ void k_presample_push(const uint64_t* __restrict__ off, const uint32_t* __restrict__ rows,
                                 uint64_t V, const uint32_t* __restrict__ oldc,
                                 uint32_t* __restrict__ newc) {
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / kWave);
  const int lane = threadIdx.x & 63;
  for (uint64_t v = (uint64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave; v < V;
       v += nw) {
    const uint32_t c = oldc[v];
    if (c == 0) continue;
    const uint64_t b = off[v], e = off[v + 1];
    for (uint64_t k = b + lane; k < e; k += kWave) atomicAdd(newc + rows[k], c);
  }
}

// The selection needs only the count at descending rank n (the pivot): a
// three-level radix select (11 + 11 + 10 bits) over the non-zero counts
// instead of a sort of all V keys (papers100M-shaped: 111 M vertices per
// super-batch).  nnz = number of non-zero counts.
__global__ void k_presample_nnz(const uint32_t* __restrict__ cnt, uint64_t V, uint32_t* nnz) {
  uint32_t local = 0;
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < V;
       v += (uint64_t)gridDim.x * blockDim.x)
    local += cnt[v] != 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) local += __shfl_down(local, o, kWave);
  if ((threadIdx.x & 63) == 0 && local) atomicAdd(nnz, local);
}

// n = (uint32)((float)total * rate) with total = nnz + 1 (V when none is zero);
// the select state: st[0] = rank still wanted, st[1] = pivot bits so far,
// st[2] = 1 when the pivot lies among the non-zero counts
__global__ void k_presample_n(const uint32_t* nnz, uint64_t V, float rate, uint32_t* n_out,
                              uint32_t* st) {
  const uint64_t total = *nnz < V ? (uint64_t)*nnz + 1 : V;
  uint64_t n = (uint64_t)((float)total * rate);
  if (n > V) n = V;
  *n_out = (uint32_t)n;
  st[0] = (uint32_t)n;
  st[1] = 0;
  st[2] = n < *nnz ? 1u : 0u;
}

constexpr int kSelBins = 2048;
// histogram of bits [shift, shift + width) of the non-zero counts whose bits
// above shift + width equal the pivot prefix so far
__global__ __launch_bounds__(256) void k_presample_hist(const uint32_t* __restrict__ cnt, uint64_t V,
                                                        const uint32_t* st, int shift, int width,
                                                        uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kSelBins];
  if (!st[2]) return;  // pivot is 0: nothing to select
  for (int i = threadIdx.x; i < kSelBins; i += 256) h[i] = 0;
  __syncthreads();
  const uint32_t prefix = st[1];
  const int hi = shift + width;
  const uint32_t mask = (1u << width) - 1u;
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < V;
       v += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = cnt[v];
    if (c != 0 && (hi >= 32 || (c >> hi) == prefix)) atomicAdd(&h[(c >> shift) & mask], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kSelBins; i += 256)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// one block: the bin holding the wanted rank (from the top), appended to the
// prefix; the histogram is cleared for the next level
__global__ __launch_bounds__(256) void k_presample_pick(uint32_t* __restrict__ hist, int width,
                                                        uint32_t* st) {
  __shared__ uint32_t h[kSelBins];
  const int bins = 1 << width;
  for (int i = threadIdx.x; i < kSelBins; i += 256) {
    h[i] = i < bins ? hist[i] : 0u;
    hist[i] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0 && st[2]) {
    uint32_t want = st[0], acc = 0;
    int b = bins - 1;
    for (; b > 0; --b) {
      if (acc + h[b] > want) break;
      acc += h[b];
    }
    st[0] = want - acc;
    st[1] = (st[1] << width) | (uint32_t)b;
  }
}

// the pivot: the selected count, or 0 when the rank falls among the zeros
__global__ void k_presample_pivot(const uint32_t* st, uint32_t* pivot) {
  *pivot = st[2] ? st[1] : 0u;
}

__global__ void k_presample_flag(const uint32_t* __restrict__ cnt, uint64_t V,
                                 const uint32_t* pivot, uint32_t* __restrict__ flag) {
  const uint32_t pv = *pivot;
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < V;
       v += (uint64_t)gridDim.x * blockDim.x)
    flag[v] = cnt[v] >= pv ? 1u : 0u;
}

__global__ void k_presample_write(const uint32_t* __restrict__ flag, const uint32_t* __restrict__ pos,
                                  uint64_t V, const uint32_t* n_out, uint32_t* __restrict__ ids) {
  const uint32_t n = *n_out;
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < V;
       v += (uint64_t)gridDim.x * blockDim.x)
    if (flag[v] && pos[v] < n) ids[pos[v]] = (uint32_t)v;
}

__global__ void k_pd_set_cache(const uint32_t* __restrict__ ids, uint32_t n, uint32_t key,
                               uint32_t* __restrict__ cmap, uint32_t* __restrict__ cloc) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    cmap[ids[i]] = key;
    cloc[ids[i]] = i;
  }
}

// one 64-lane group per dst row, float columns strided
__global__ void k_pd_load_share(const uint32_t* __restrict__ omit_row, const uint32_t* v_dev,
                                uint32_t v_cap, const float* __restrict__ share, uint64_t lds,
                                uint32_t F, float* __restrict__ emb, uint64_t lde) {
  const uint32_t v = v_dev ? min(*v_dev, v_cap) : v_cap;
  const int lane = threadIdx.x & 63;
  for (uint32_t i = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave; i < v;
       i += gridDim.x * (blockDim.x / kWave)) {
    const uint32_t row = omit_row[i];
    if (row == 0xFFFFFFFFu) continue;
    const float* s = share + (uint64_t)row * lds;
    float* o = emb + (uint64_t)i * lde;
    for (uint32_t c = lane; c < F; c += kWave) o[c] = s[c];
  }
}

__global__ void k_relu_dropout(const float* __restrict__ x, uint64_t ldx, uint32_t rows,
                               uint32_t F, uint32_t keep_threshold, float scale, uint64_t seed,
                               uint64_t offset, float* __restrict__ y, uint64_t ldy) {
  // thread = a 4-row x 2-column block (one Philox call, the GEMM epilogue's keys)
  const uint32_t cpairs = (F + 1) / 2;
  const uint64_t blocks = (uint64_t)((rows + 3) / 4) * cpairs;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < blocks;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t r4 = (uint32_t)(t / cpairs) * 4, c2 = (uint32_t)(t % cpairs) * 2;
    uint4 rnd = make_uint4(0u, 0u, 0u, 0u);
    if (keep_threshold) rnd = dropout_words(r4, c2, seed, offset);
    const uint32_t wd[4] = {rnd.x, rnd.y, rnd.z, rnd.w};
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const uint32_t r = r4 + v;
      if (r >= rows) break;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t c = c2 + h;
        if (c >= F) break;
        const float a = x[(uint64_t)r * ldx + c];
        y[(uint64_t)r * ldy + c] =
            (dropout_bits(wd[v], c) >= keep_threshold && a > 0.f) ? a * scale : 0.f;
      }
    }
  }
}

}  // namespace nts_hip

using namespace nts_hip;

extern "C" {

int nts_hip_presample_counts(nts_hip_ctx* ctx, const nts_graph_dev* g, const uint32_t* seeds,
                             uint32_t n_seeds, int layers, uint32_t* counts, uint32_t* tmp) {
  NTS_CHECK_ARG(ctx && g && g->column_offset && g->row_indices && counts && tmp, "NULL argument");
  NTS_CHECK_ARG(seeds || n_seeds == 0, "NULL seeds");
  NTS_CHECK_ARG(layers >= 1, "layers >= 1");
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const uint64_t V = g->n_vertices;
  // ping-pong so that the last `new` lands in `counts`
  uint32_t* bufs[2] = {tmp, counts};
  const int passes = layers - 1;
  uint32_t* oldc = (passes % 2 == 0) ? counts : tmp;
  NTS_HIP_TRY(hipMemsetAsync(oldc, 0, V * sizeof(uint32_t), st));
  if (n_seeds) {
    const uint32_t gs = std::max(1u, std::min(ceil_div(n_seeds, 256), kMaxGrid));
    hipLaunchKernelGGL(k_presample_seed, dim3(gs), dim3(256), 0, st, seeds, n_seeds, oldc);
    NTS_LAUNCH_CHECK();
  }
  if (passes == 0) {  // the reference's loop does not run: counts stay 0
    NTS_HIP_TRY(hipMemsetAsync(counts, 0, V * sizeof(uint32_t), st));
    return NTS_OK;
  }
  (void)bufs;
  for (int p = 0; p < passes; ++p) {
    uint32_t* newc = (oldc == tmp) ? counts : tmp;
    NTS_HIP_TRY(hipMemsetAsync(newc, 0, V * sizeof(uint32_t), st));
    const uint32_t gw = std::max(1u, std::min(ceil_div(V, 4), 8192u));
    hipLaunchKernelGGL(k_presample_push, dim3(gw), dim3(256), 0, st, g->column_offset,
                       g->row_indices, V, oldc, newc);
    NTS_LAUNCH_CHECK();
    oldc = newc;
  }
  return NTS_OK;
}

int nts_hip_presample_select(nts_hip_ctx* ctx, const uint32_t* counts, uint64_t V,
                             float cache_rate, uint32_t* out_ids, uint32_t* out_n) {
  NTS_CHECK_ARG(ctx && counts && out_ids && out_n, "NULL argument");
  NTS_CHECK_ARG(V > 0 && V <= 0xFFFFFFFFull, "vertex count");
  NTS_CHECK_ARG(cache_rate >= 0.f, "cache_rate >= 0");
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  auto al = [](uint64_t x) { return (x + 63) / 64 * 64; };
  const uint64_t w = al(V + 1);
  const size_t scan_tmp = scan_tmp_elems<uint32_t>(V) + 64;
  NTS_RET(ensure_scratch(ctx, (2 * w + kSelBins + scan_tmp + 64) * sizeof(uint32_t) + 256));
  uint32_t* flag = (uint32_t*)ctx->scratch;
  uint32_t* pos = flag + w;
  uint32_t* hist = pos + w;  // [kSelBins]
  uint32_t* misc = hist + kSelBins;  // [0] nnz, [1] pivot, [4..6] select state
  uint32_t* stmp = misc + 64;
  NTS_HIP_TRY(hipMemsetAsync(hist, 0, (kSelBins + 64) * sizeof(uint32_t), st));
  const uint32_t gs = std::max(1u, std::min(ceil_div(V, 256), kMaxGrid));
  hipLaunchKernelGGL(k_presample_nnz, dim3(gs), dim3(256), 0, st, counts, V, misc);
  NTS_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_presample_n, dim3(1), dim3(1), 0, st, misc, V, cache_rate, out_n, misc + 4);
  NTS_LAUNCH_CHECK();
  const int levels[3][2] = {{21, 11}, {10, 11}, {0, 10}};  // (shift, width), high bits first
  for (const auto& lv : levels) {
    hipLaunchKernelGGL(k_presample_hist, dim3(gs), dim3(256), 0, st, counts, V, misc + 4, lv[0],
                       lv[1], hist);
    NTS_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_presample_pick, dim3(1), dim3(256), 0, st, hist, lv[1], misc + 4);
    NTS_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_presample_pivot, dim3(1), dim3(1), 0, st, misc + 4, misc + 1);
  NTS_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_presample_flag, dim3(gs), dim3(256), 0, st, counts, V, misc + 1, flag);
  NTS_LAUNCH_CHECK();
  NTS_RET(scan_exclusive<uint32_t>(flag, pos, nullptr, V, stmp, st));
  hipLaunchKernelGGL(k_presample_write, dim3(gs), dim3(256), 0, st, flag, pos, V, out_n, out_ids);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

int nts_hip_pd_set_cache(nts_hip_ctx* ctx, const uint32_t* ids, uint32_t n, uint32_t key,
                         uint32_t* cache_map, uint32_t* cache_location) {
  NTS_CHECK_ARG(ctx && cache_map && cache_location && (ids || n == 0), "NULL argument");
  if (n == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  const uint32_t gs = std::max(1u, std::min(ceil_div(n, 256), kMaxGrid));
  hipLaunchKernelGGL(k_pd_set_cache, dim3(gs), dim3(256), 0, ctx->stream, ids, n, key, cache_map,
                     cache_location);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

int nts_hip_pd_load_share(nts_hip_ctx* ctx, const uint32_t* omit_row, const uint32_t* v,
                          uint32_t v_cap, const float* share, uint64_t ld_share,
                          uint32_t feature_size, float* emb, uint64_t ld_emb) {
  NTS_CHECK_ARG(ctx && omit_row && share && emb, "NULL argument");
  NTS_CHECK_ARG(ld_share >= feature_size && ld_emb >= feature_size, "leading dimension");
  if (v_cap == 0 || feature_size == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  const uint32_t gs = std::max(1u, std::min(ceil_div(v_cap, 4), kMaxGrid));
  hipLaunchKernelGGL(k_pd_load_share, dim3(gs), dim3(256), 0, ctx->stream, omit_row, v, v_cap,
                     share, ld_share, feature_size, emb, ld_emb);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

int nts_hip_relu_dropout_f32(nts_hip_ctx* ctx, uint32_t rows, uint32_t feature_size,
                             const float* x, uint64_t ldx, float p, uint64_t seed,
                             uint64_t offset, float* y, uint64_t ldy) {
  NTS_CHECK_ARG(ctx && x && y, "NULL argument");
  NTS_CHECK_ARG(ldx >= feature_size && ldy >= feature_size, "leading dimension");
  NTS_CHECK_ARG(p >= 0.f && p <= 1.f, "dropout probability must be in [0, 1]");
  if (rows == 0 || feature_size == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  const uint64_t blocks = (uint64_t)((rows + 3) / 4) * ((feature_size + 1) / 2);
  const uint32_t gs = std::max(1u, std::min(ceil_div(blocks, 256), kMaxGrid));
  hipLaunchKernelGGL(k_relu_dropout, dim3(gs), dim3(256), 0, ctx->stream, x, ldx, rows,
                     feature_size, dropout_threshold(p), p >= 1.f ? 0.f : 1.0f / (1.0f - p), seed,
                     offset, y, ldy);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

}  // extern "C"
