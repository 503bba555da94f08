// Graph preprocessing on the device: degrees and the replicated global CSC.
// Reference: Graph::load_directed degree counting (core/graph.hpp:1157-1186,
// 1420-1425), the >=1 clamp (core/graph.hpp:4525-4530) and
// FullyRepGraph::ReadRepGraphFromRawFile (core/FullyRepGraph.hpp:724-798),
// a two-pass counting sort keyed by dst that keeps file order inside a dst.
// Here the stable order comes from a stable LSD radix sort on dst.
#include "common.hpp"

namespace nts_hip {

__global__ void k_count_degrees(const uint32_t* __restrict__ src,
                                const uint32_t* __restrict__ dst, uint64_t n_edges,
                                uint32_t* out_degree, uint32_t* in_degree) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n_edges;
       e += (uint64_t)gridDim.x * blockDim.x) {
    atomicAdd(&out_degree[src[e]], 1u);
    atomicAdd(&in_degree[dst[e]], 1u);
  }
}

__global__ void k_clamp_degrees(uint64_t n, uint32_t* a, uint32_t* b) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    if (a[i] < 1) a[i] = 1;
    if (b[i] < 1) b[i] = 1;
  }
}

__global__ void k_count_dst_u64(const uint32_t* __restrict__ dst, uint64_t n_edges,
                                unsigned long long* cnt) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n_edges;
       e += (uint64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[dst[e]], 1ull);
}

}  // namespace nts_hip

using namespace nts_hip;

extern "C" {

int nts_hip_degrees(nts_hip_ctx* ctx, const uint32_t* src, const uint32_t* dst,
                    uint64_t n_edges, uint64_t n_vertices, uint32_t* out_degree,
                    uint32_t* in_degree) {
  NTS_CHECK_ARG(ctx && out_degree && in_degree, "NULL argument");
  NTS_CHECK_ARG(n_edges == 0 || (src && dst), "NULL edge list");
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  NTS_HIP_TRY(hipMemsetAsync(out_degree, 0, n_vertices * 4, ctx->stream));
  NTS_HIP_TRY(hipMemsetAsync(in_degree, 0, n_vertices * 4, ctx->stream));
  if (n_edges) {
    uint32_t g = (uint32_t)std::min<uint64_t>(ceil_div(n_edges, 256), 8192);
    hipLaunchKernelGGL(k_count_degrees, dim3(g), dim3(256), 0, ctx->stream, src, dst, n_edges,
                       out_degree, in_degree);
    NTS_LAUNCH_CHECK();
  }
  if (n_vertices) {
    uint32_t g = (uint32_t)std::min<uint64_t>(ceil_div(n_vertices, 256), kMaxGrid);
    hipLaunchKernelGGL(k_clamp_degrees, dim3(g), dim3(256), 0, ctx->stream, n_vertices,
                       out_degree, in_degree);
    NTS_LAUNCH_CHECK();
  }
  return NTS_OK;
}

int nts_hip_build_csc(nts_hip_ctx* ctx, const uint32_t* src, const uint32_t* dst,
                      uint64_t n_edges, uint64_t n_vertices, uint64_t* column_offset,
                      uint32_t* row_indices) {
  NTS_CHECK_ARG(ctx && column_offset, "NULL argument");
  NTS_CHECK_ARG(n_edges == 0 || (src && dst && row_indices), "NULL edge list");
  NTS_CHECK_ARG(n_vertices > 0 && n_vertices <= 0xFFFFFFFFull, "vertex count out of range");
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  // 1) per-dst counts -> exclusive scan -> column_offset[V+1] (64-bit)
  NTS_HIP_TRY(hipMemsetAsync(column_offset, 0, (n_vertices + 1) * 8, ctx->stream));
  if (n_edges) {
    uint32_t g = (uint32_t)std::min<uint64_t>(ceil_div(n_edges, 256), 8192);
    hipLaunchKernelGGL(k_count_dst_u64, dim3(g), dim3(256), 0, ctx->stream, dst, n_edges,
                       (unsigned long long*)column_offset);
    NTS_LAUNCH_CHECK();
  }
  size_t scan_bytes = scan_tmp_elems<uint64_t>(n_vertices) * 8 + 256;
  size_t sort_bytes = n_edges ? ((n_edges + 63) / 64 * 64) * 4 + radix_tmp_bytes(n_edges) : 0;
  NTS_RET(ensure_scratch(ctx, std::max(scan_bytes, sort_bytes)));
  NTS_RET(scan_exclusive<uint64_t>(column_offset, column_offset, nullptr, n_vertices,
                                   (uint64_t*)ctx->scratch, ctx->stream));
  if (!n_edges) return NTS_OK;
  // 2) stable sort of (dst, src) pairs on dst: row_indices = src in file order per dst
  uint32_t* keys_sorted = (uint32_t*)ctx->scratch;
  void* tmp = keys_sorted + (n_edges + 63) / 64 * 64;
  NTS_RET(radix_sort_pairs(dst, src, keys_sorted, row_indices, nullptr, n_edges,
                           ceil_log2(n_vertices), tmp, ctx->stream));
  return NTS_OK;
}

}  // extern "C"
