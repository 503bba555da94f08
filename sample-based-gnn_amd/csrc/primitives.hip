// Device-wide primitives used by the sampler and the graph builder:
//  * exclusive scan (u32 / u64) whose length lives in device memory,
//  * stable LSD radix sort of (u32 key, u32 value) pairs, length in device memory.
// Both are written for wave64 (ballot-based digit matching, 64-lane shuffles)
// and never synchronise with the host, so a whole sampling hop can be
// enqueued (or graph-captured) without knowing e_size / src_size on the host.
#include "common.hpp"

namespace nts_hip {

// ============================================================================
// exclusive scan
// ============================================================================
constexpr int kScanThreads = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kScanThreads * kScanItems;  // 4096

__device__ __forceinline__ uint32_t pad_idx(uint32_t j) { return j + (j >> 4); }

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T x, int lane) {
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    T y = __shfl_up(x, o, kWave);
    if (lane >= o) x += y;
  }
  return x;
}

// Block-wide exclusive scan of one value per thread; returns exclusive prefix,
// writes block total to *total.
template <typename T>
__device__ __forceinline__ T block_excl_scan(T x, T* wsum /*[4]*/, T* total) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  T inc = wave_incl_scan(x, lane);
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  T off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kScanThreads / kWave; ++i) {
    T s = wsum[i];
    if (i < w) off += s;
    tot += s;
  }
  *total = tot;
  return off + inc - x;
}

template <typename T>
__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const T* __restrict__ in,
                                                             const uint32_t* n_dev,
                                                             uint64_t n_cap, T* partials) {
  const uint64_t n = n_dev ? (uint64_t)*n_dev : n_cap;
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  T s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    uint64_t i = base + (uint64_t)k * kScanThreads + threadIdx.x;
    if (i < n) s += in[i];
  }
  __shared__ T wsum[kScanThreads / kWave];
  T tot;
  (void)block_excl_scan(s, wsum, &tot);
  if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

// Sum of partials[0 .. count) by the whole block (fixed order per thread,
// fixed tree across threads: the same value in every block that asks).
template <typename T>
__device__ __forceinline__ T block_prefix_of(const T* partials, uint32_t count, T* wsum) {
  T s = 0;
  for (uint32_t i = threadIdx.x; i < count; i += kScanThreads) s += partials[i];
  T tot;
  (void)block_excl_scan(s, wsum, &tot);
  __syncthreads();
  return tot;
}

// Scan one tile with a starting offset; writes out[i] for i <= n inside the tile.
// DIRECT: the offset is the sum of partials[0 .. blockIdx.x) (tile totals),
// computed here — no separate scan of the partials (and no single-workgroup
// kernel, which stalls for tens of microseconds behind a concurrent stream's
// large kernels).  Otherwise partials[blockIdx.x] is already the offset.
template <typename T, bool DIRECT>
__global__ __launch_bounds__(kScanThreads) void k_scan_down(const T* in, T* out,
                                                           const uint32_t* n_dev,
                                                           uint64_t n_cap,
                                                           const T* partials) {
  const uint64_t n = n_dev ? (uint64_t)*n_dev : n_cap;
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  if (base > n) return;
  __shared__ T tile[kScanTile + kScanTile / 16];
  __shared__ T wsum[kScanThreads / kWave];
  const int t = threadIdx.x;
  T start = 0;
  if (DIRECT) start = block_prefix_of(partials, blockIdx.x, wsum);
  else if (partials) start = partials[blockIdx.x];
  // striped, coalesced load -> padded LDS
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    uint32_t j = k * kScanThreads + t;
    uint64_t i = base + j;
    tile[pad_idx(j)] = (i < n) ? in[i] : T(0);
  }
  __syncthreads();
  T v[kScanItems];
  T s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = tile[pad_idx(t * kScanItems + k)];
    s += v[k];
  }
  T tot;
  T run = block_excl_scan(s, wsum, &tot) + start;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    tile[pad_idx(t * kScanItems + k)] = run;
    run += v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    uint32_t j = k * kScanThreads + t;
    uint64_t i = base + j;
    if (i <= n) out[i] = tile[pad_idx(j)];
  }
}

template <typename T>
size_t scan_tmp_elems(uint64_t n_cap) {
  uint64_t nb = n_cap / kScanTile + 1;
  if (nb == 1) return 0;
  return (nb + 1 + 63) / 64 * 64 + scan_tmp_elems<T>(nb);
}

// Tile counts up to which every block sums the preceding tile totals itself
// (reduce + down: two kernels); beyond, the totals are scanned recursively.
constexpr uint64_t kScanDirectTiles = 1024;

template <typename T>
int scan_exclusive(const T* in, T* out, const uint32_t* n_dev, uint64_t n_cap, T* tmp,
                   hipStream_t stream) {
  uint64_t nb = n_cap / kScanTile + 1;
  if (nb == 1) {
    hipLaunchKernelGGL((k_scan_down<T, false>), dim3(1), dim3(kScanThreads), 0, stream, in, out,
                       n_dev, n_cap, (const T*)nullptr);
    NTS_LAUNCH_CHECK();
    return NTS_OK;
  }
  T* partials = tmp;
  T* rest = tmp + (nb + 1 + 63) / 64 * 64;
  hipLaunchKernelGGL(k_scan_reduce<T>, dim3((uint32_t)nb), dim3(kScanThreads), 0, stream, in,
                     n_dev, n_cap, partials);
  NTS_LAUNCH_CHECK();
  if (nb <= kScanDirectTiles) {
    hipLaunchKernelGGL((k_scan_down<T, true>), dim3((uint32_t)nb), dim3(kScanThreads), 0, stream,
                       in, out, n_dev, n_cap, (const T*)partials);
    NTS_LAUNCH_CHECK();
    return NTS_OK;
  }
  NTS_RET(scan_exclusive<T>(partials, partials, nullptr, nb, rest, stream));
  hipLaunchKernelGGL((k_scan_down<T, false>), dim3((uint32_t)nb), dim3(kScanThreads), 0, stream,
                     in, out, n_dev, n_cap, (const T*)partials);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

template int scan_exclusive<uint32_t>(const uint32_t*, uint32_t*, const uint32_t*, uint64_t,
                                      uint32_t*, hipStream_t);
template int scan_exclusive<uint64_t>(const uint64_t*, uint64_t*, const uint32_t*, uint64_t,
                                      uint64_t*, hipStream_t);
template size_t scan_tmp_elems<uint32_t>(uint64_t);
template size_t scan_tmp_elems<uint64_t>(uint64_t);

// ============================================================================
// stable LSD radix sort (8-bit digits)
// ============================================================================
constexpr int kRadixThreads = 256;
constexpr int kRadixItems = 8;
constexpr int kRadixTile = kRadixThreads * kRadixItems;  // 2048
constexpr int kRadixBins = 256;

__global__ __launch_bounds__(kRadixThreads) void k_radix_hist(const uint32_t* __restrict__ keys,
                                                              const uint32_t* n_dev,
                                                              uint64_t n_cap, uint32_t shift,
                                                              uint32_t* hist, uint32_t nb) {
  __shared__ uint32_t h[kRadixBins];
  const int t = threadIdx.x;
  h[t] = 0;
  __syncthreads();
  const uint64_t n = n_dev ? (uint64_t)*n_dev : n_cap;
  const uint64_t base = (uint64_t)blockIdx.x * kRadixTile;
#pragma unroll
  for (int k = 0; k < kRadixItems; ++k) {
    uint64_t i = base + (uint64_t)k * kRadixThreads + t;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[(uint64_t)t * nb + blockIdx.x] = h[t];  // digit-major
}

__global__ __launch_bounds__(kRadixThreads) void k_radix_scatter(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out, const uint32_t* n_dev,
    uint64_t n_cap, uint32_t shift, const uint32_t* __restrict__ hist, uint32_t nb) {
  __shared__ uint32_t goff[kRadixBins];                    // global offset of this block's digit run
  __shared__ uint32_t wcnt[kRadixThreads / kWave][kRadixBins];  // per-wave digit counts -> prefixes
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint64_t n = n_dev ? (uint64_t)*n_dev : n_cap;
  const uint64_t base = (uint64_t)blockIdx.x * kRadixTile;
  goff[t] = hist[(uint64_t)t * nb + blockIdx.x];
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int k = 0; k < kRadixItems; ++k) {
    const uint64_t i = base + (uint64_t)k * kRadixThreads + t;
    const bool valid = i < n;
    uint32_t key = valid ? keys_in[i] : 0u;
    uint32_t val = valid ? (vals_in ? vals_in[i] : (uint32_t)i) : 0u;
    uint32_t d = (key >> shift) & 255u;
#pragma unroll
    for (int ww = 0; ww < kRadixThreads / kWave; ++ww) wcnt[ww][t] = 0;
    __syncthreads();
    // lanes of this wave holding the same digit (match-any via 8 ballots)
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      bool bit = (d >> b) & 1u;
      uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    uint32_t rank = __popcll(peers & lt_mask);
    if (valid && rank == 0) wcnt[w][d] = __popcll(peers);
    __syncthreads();
    {  // thread t owns digit t: exclusive prefix over waves, advance running base
      uint32_t run = goff[t];
#pragma unroll
      for (int ww = 0; ww < kRadixThreads / kWave; ++ww) {
        uint32_t c = wcnt[ww][t];
        wcnt[ww][t] = run;
        run += c;
      }
      goff[t] = run;
    }
    __syncthreads();
    if (valid) {
      uint32_t pos = wcnt[w][d] + rank;
      keys_out[pos] = key;
      vals_out[pos] = val;
    }
    __syncthreads();
  }
}

size_t radix_tmp_bytes(uint64_t n_cap) {
  uint64_t nb = (n_cap + kRadixTile - 1) / kRadixTile;
  if (nb == 0) nb = 1;
  size_t hist = (size_t)kRadixBins * nb + 1;
  size_t elems = 2 * ((n_cap + 63) / 64 * 64) + (hist + 63) / 64 * 64 +
                 scan_tmp_elems<uint32_t>(kRadixBins * nb) + 64;
  return elems * sizeof(uint32_t);
}

int radix_sort_pairs(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* keys_out,
                     uint32_t* vals_out, const uint32_t* n_dev, uint64_t n_cap, uint32_t bits,
                     void* tmp, hipStream_t stream) {
  if (n_cap == 0) return NTS_OK;
  uint32_t nb = ceil_div(n_cap, kRadixTile);
  uint64_t n_al = (n_cap + 63) / 64 * 64;
  uint32_t* ktmp = (uint32_t*)tmp;
  uint32_t* vtmp = ktmp + n_al;
  uint32_t* hist = vtmp + n_al;
  uint64_t hist_n = (uint64_t)kRadixBins * nb;
  uint32_t* stmp = hist + (hist_n + 1 + 63) / 64 * 64;
  int npass = (int)((bits + 7) / 8);
  if (npass < 1) npass = 1;
  const uint32_t* ksrc = keys_in;
  const uint32_t* vsrc = vals_in;
  for (int p = 0; p < npass; ++p) {
    bool to_out = ((npass - 1 - p) % 2) == 0;
    uint32_t* kdst = to_out ? keys_out : ktmp;
    uint32_t* vdst = to_out ? vals_out : vtmp;
    uint32_t shift = 8u * p;
    hipLaunchKernelGGL(k_radix_hist, dim3(nb), dim3(kRadixThreads), 0, stream, ksrc, n_dev,
                       n_cap, shift, hist, nb);
    NTS_LAUNCH_CHECK();
    NTS_RET(scan_exclusive<uint32_t>(hist, hist, nullptr, hist_n, stmp, stream));
    hipLaunchKernelGGL(k_radix_scatter, dim3(nb), dim3(kRadixThreads), 0, stream, ksrc, vsrc,
                       kdst, vdst, n_dev, n_cap, shift, (const uint32_t*)hist, nb);
    NTS_LAUNCH_CHECK();
    ksrc = kdst;
    vsrc = vdst;
  }
  return NTS_OK;
}

}  // namespace nts_hip
