// HBM feature cache + host-pinned spill: selection of the cached vertices and
// the host allocation the spill lives in.
//
// The reference keeps the full feature table in pinned host memory and the
// rows of the highest-out-degree vertices in a GPU cache
// (toolkits/GS_SAMPLE_PD_CACHE.hpp:1019-1112: cache_high_degree sorts the ids
// by out_degree_for_backward descending, mark_cache_node gives the first
// cache_node_num of them slots 0, 1, ... in that order, and
// gater_cpu_cache_feature_and_trans_to_gpu copies their rows to the device).
// Here the selection is a stable device radix sort of (~degree, id): slot s
// holds the vertex of rank s in (degree descending, id ascending) order.  The
// reference's std::sort leaves the order of equal degrees unspecified; the
// stable order is this build's tie rule.  Which rows are cached never changes
// a gathered value — only where it is read from.
#include "common.hpp"

namespace nts_hip {

__global__ void k_cache_keys(const uint32_t* __restrict__ deg, uint64_t n, uint32_t* __restrict__ key) {
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
       v += (uint64_t)gridDim.x * blockDim.x)
    key[v] = ~deg[v];  // ascending ~deg = descending degree
}

// rank s of the sorted order: slot s if s < n_cache, else not cached
__global__ void k_cache_mark(const uint32_t* __restrict__ order, uint64_t n, uint64_t n_cache,
                             uint32_t* __restrict__ cache_map, uint32_t* __restrict__ cache_ids) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = order[s];
    const bool hot = s < n_cache;
    cache_map[v] = hot ? (uint32_t)s : 0xFFFFFFFFu;
    if (hot && cache_ids) cache_ids[s] = v;
  }
}

}  // namespace nts_hip

using namespace nts_hip;

extern "C" {

int nts_hip_cache_select(nts_hip_ctx* ctx, const uint32_t* out_degree, uint64_t n_vertices,
                         uint64_t n_cache, uint32_t* cache_map, uint32_t* cache_ids) {
  NTS_CHECK_ARG(ctx && out_degree && cache_map, "NULL argument");
  NTS_CHECK_ARG(n_vertices < 0x80000000ull, "vertex ids must be < 2^31 (the gather tags the tier in bit 31)");
  NTS_CHECK_ARG(n_cache <= n_vertices, "n_cache > n_vertices");
  NTS_CHECK_ARG(n_cache == 0 || cache_ids, "cache_ids is NULL");
  if (n_vertices == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  const uint64_t n_al = (n_vertices + 63) / 64 * 64;
  // keys | sorted keys | sorted ids | radix temporaries (one-off setup call)
  NTS_RET(ensure_scratch(ctx, 3 * n_al * sizeof(uint32_t) + radix_tmp_bytes(n_vertices)));
  uint32_t* key = (uint32_t*)ctx->scratch;
  uint32_t* skey = key + n_al;
  uint32_t* order = skey + n_al;
  void* tmp = order + n_al;
  const uint32_t grid = std::max(1u, std::min(ceil_div(n_vertices, 256), 8192u));
  hipLaunchKernelGGL(k_cache_keys, dim3(grid), dim3(256), 0, ctx->stream, out_degree, n_vertices,
                     key);
  NTS_LAUNCH_CHECK();
  NTS_RET(radix_sort_pairs(key, nullptr, skey, order, nullptr, n_vertices, 32, tmp, ctx->stream));
  hipLaunchKernelGGL(k_cache_mark, dim3(grid), dim3(256), 0, ctx->stream, order, n_vertices,
                     n_cache, cache_map, cache_ids);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

int nts_hip_host_alloc(uint64_t bytes, void** host_ptr) {
  NTS_CHECK_ARG(host_ptr, "NULL argument");
  *host_ptr = nullptr;
  if (bytes == 0) return NTS_OK;
  // mapped into every device's address space; non-coherent (coarse-grained):
  // the table is written by the host before any kernel reads it, and the GPU
  // may then keep the rows it reads in its caches
  NTS_HIP_TRY(hipHostMalloc(host_ptr, (size_t)bytes,
                            hipHostMallocMapped | hipHostMallocPortable | hipHostMallocNonCoherent));
  return NTS_OK;
}

int nts_hip_host_free(void* host_ptr) {
  if (host_ptr) NTS_HIP_TRY(hipHostFree(host_ptr));
  return NTS_OK;
}

int nts_hip_host_device_pointer(void* host_ptr, void** dev_ptr) {
  NTS_CHECK_ARG(host_ptr && dev_ptr, "NULL argument");
  NTS_HIP_TRY(hipHostGetDevicePointer(dev_ptr, host_ptr, 0));
  return NTS_OK;
}

}  // extern "C"
