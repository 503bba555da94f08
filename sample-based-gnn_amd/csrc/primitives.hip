// Device-wide primitives used by the sampler and the graph builder:
//  * exclusive scan (u32 / u64) whose length lives in device memory,
//  * stable LSD radix sort of (u32 key, u32 value) pairs, length in device memory.
// Both are written for wave64 (ballot-based digit matching, 64-lane shuffles)
// and never synchronise with the host, so a whole sampling hop can be
// enqueued (or graph-captured) without knowing e_size / src_size on the host.
#include "common.hpp"
#include "radix_tile.hpp"

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
// CNT: the input is the sampler's counts (k_count_reduce) and out[n] is also
// e_size: sizes[1] = out[n], or past e_cap the offset of the first dst whose
// edges do not fit (overflow flagged in sizes[3]).
template <typename T, bool DIRECT, bool CNT = false>
__global__ __launch_bounds__(kScanThreads) void k_scan_down(const T* in, T* out,
                                                           const uint32_t* n_dev,
                                                           uint64_t n_cap,
                                                           const T* partials,
                                                           uint32_t* sizes, uint32_t e_cap) {
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
    // CNT: the item whose edges cross the capacity truncates the layer at
    // its first edge (never inside a destination: the selection skips a dst
    // that does not fit whole, so no edge array holds unwritten slots)
    if (CNT && run <= (T)e_cap && run + v[k] > (T)e_cap) sizes[1] = (uint32_t)run;
    run += v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    uint32_t j = k * kScanThreads + t;
    uint64_t i = base + j;
    if (i <= n) out[i] = tile[pad_idx(j)];
    if (CNT && i == n) {
      const T e = tile[pad_idx(j)];
      if (e <= (T)e_cap) sizes[1] = (uint32_t)e;
      if (e > (T)e_cap) atomicOr(&sizes[3], 1u);
    }
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
                       n_dev, n_cap, (const T*)nullptr, nullptr, 0u);
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
                       in, out, n_dev, n_cap, (const T*)partials, nullptr, 0u);
    NTS_LAUNCH_CHECK();
    return NTS_OK;
  }
  NTS_RET(scan_exclusive<T>(partials, partials, nullptr, nb, rest, stream));
  hipLaunchKernelGGL((k_scan_down<T, false>), dim3((uint32_t)nb), dim3(kScanThreads), 0, stream,
                     in, out, n_dev, n_cap, (const T*)partials, nullptr, 0u);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

// ---------------------------------------------------------------------------
// Single-pass exclusive scan (u32) with decoupled look-back: one kernel where
// scan_exclusive needs two.  Tile t publishes its aggregate, then its
// inclusive prefix once the look-back over tiles t-1, t-2, ... has found an
// inclusive prefix; tile states are 64-bit words {epoch:30 | kind:2 |
// value:32} written and read with RELAXED agent-scope atomics: each word
// carries its own value, so no other data needs ordering (acquire/release
// would add an L2 invalidate / write-back per access — buffer_inv sc1 and
// buffer_wbl2 sc1 — which cost the whole XCD its L2, measured 34 us a call).  The epoch (a per-call
// sequence number) makes states of earlier calls invalid, so nothing is reset
// between calls.  A workgroup's tile is its dispatch-order ticket (lb_ticket,
// common.hpp), not blockIdx.x: a tile only waits on lower tiles, and every
// lower ticket was drawn by a workgroup that is already running, so the chain
// completes whatever order the dispatcher places workgroups in.
// COUNT: the input is not read from memory but computed per item as the
// sampler's per-dst count min(deg(dst[i]), fanout) (init_co_only,
// core/FullyRepGraph.hpp:530-539), with the omit map of sample_gpu_fast_omit
// (core/ntsFastSampler.hpp:711-915) — k_count fused into the scan.
// ---------------------------------------------------------------------------
constexpr uint64_t kTileAgg = 1, kTileIncl = 2;

__device__ __forceinline__ uint64_t tile_word(uint32_t epoch, uint64_t kind, uint32_t v) {
  return ((uint64_t)(epoch & 0x3FFFFFFFu) << 34) | (kind << 32) | v;
}

// The sampler's per-dst counts of the tile's items i = base + k kScanThreads + t:
// min(deg(dst[i]), fanout) (init_co_only, core/FullyRepGraph.hpp:530-539), 0
// for a dst of the omit map (sample_gpu_fast_omit, core/ntsFastSampler.hpp:
// 711-915), whose cache row is recorded in omit_row.  Three rounds of
// independent loads (dst ids, their offsets, the omit map) instead of one
// dependent chain per item.
template <int IT>
__device__ __forceinline__ void count_items(const CountArgs& ca, uint64_t base, uint64_t n,
                                            uint32_t (&x)[IT]) {
  const int t = threadIdx.x;
  uint32_t d[IT];
  uint64_t lo[IT], hi[IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const uint64_t i = base + (uint64_t)k * kScanThreads + t;
    d[k] = i < n ? ca.dst[i] : 0u;
  }
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const uint64_t i = base + (uint64_t)k * kScanThreads + t;
    lo[k] = i < n ? ca.goff[d[k]] : 0u;
    hi[k] = i < n ? ca.goff[d[k] + 1] : 0u;
  }
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const uint32_t deg = (uint32_t)(hi[k] - lo[k]);
    x[k] = ca.fanout < 0 ? deg : min(deg, (uint32_t)ca.fanout);
  }
  if (ca.omit_map) {
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const uint64_t i = base + (uint64_t)k * kScanThreads + t;
      if (i < n) {
        const bool om = ca.omit_map[d[k]] == ca.omit_key;
        if (om) x[k] = 0;
        if (ca.omit_row) ca.omit_row[i] = om ? ca.omit_loc[d[k]] : 0xFFFFFFFFu;
      }
    }
  }
}

// IT items per thread: 16 for the radix-free generic scans; 4 for the count
// scan, whose items are three dependent random loads each — 1,024-item tiles
// put 4x the workgroups on the chip (57 -> 228 at C2's second layer) and keep
// the tile's LDS (4.4 KB) within what a CU has left beside the 144 KB GEMMs.
template <bool COUNT, int IT>
__global__ __launch_bounds__(kScanThreads) void k_scan1(const uint32_t* __restrict__ in,
                                                        uint32_t* __restrict__ out,
                                                        const uint32_t* n_dev, uint64_t n_cap,
                                                        uint64_t* __restrict__ state,
                                                        uint32_t epoch, uint32_t* ticket,
                                                        CountArgs ca) {
  constexpr int kTile = kScanThreads * IT;
  __shared__ uint32_t tile[kTile + kTile / 16];
  __shared__ uint32_t wsum[kScanThreads / kWave];
  __shared__ uint32_t s_prefix;
  const uint32_t ti = lb_ticket(ticket, gridDim.x);
  const int t = threadIdx.x, lane = t & 63;
  uint64_t n;
  uint32_t v_req = 0;
  if (COUNT) {
    v_req = *ca.v_in;
    n = min(v_req, ca.v_cap);
    if (ti == 0 && t == 0) ca.sizes[0] = (uint32_t)n;
  } else {
    n = n_dev ? (uint64_t)*n_dev : n_cap;
  }
  const uint64_t base = (uint64_t)ti * kTile;
  if (base > n) return;  // every tile up to the one holding out[n] runs the chain
  if constexpr (COUNT) {
    uint32_t x[IT];
    count_items(ca, base, n, x);
#pragma unroll
    for (int k = 0; k < IT; ++k) tile[pad_idx(k * kScanThreads + t)] = x[k];
  } else {
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const uint32_t j = k * kScanThreads + t;
      const uint64_t i = base + j;
      tile[pad_idx(j)] = i < n ? in[i] : 0u;
    }
  }
  __syncthreads();
  uint32_t v[IT];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    v[k] = tile[pad_idx(t * IT + k)];
    s += v[k];
  }
  uint32_t agg;
  const uint32_t ex = block_excl_scan(s, wsum, &agg);
  // publish, look back (wave 0, lanes over 64 predecessors at a time)
  if (t < kWave) {
    if (ti == 0) {
      if (t == 0) {
        __hip_atomic_store(state, tile_word(epoch, kTileIncl, agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        s_prefix = 0;
      }
    } else {
      if (t == 0)
        __hip_atomic_store(state + ti, tile_word(epoch, kTileAgg, agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      uint32_t prefix = 0;
      int64_t top = (int64_t)ti - 1;  // highest tile not yet folded in
      for (;;) {
        const int64_t p = top - lane;
        uint64_t w = 0;
        uint32_t kind = 0;
        if (p >= 0) {
          for (;;) {  // this lane's tile has published (under this epoch)
            w = __hip_atomic_load(state + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)(w >> 34) == (epoch & 0x3FFFFFFFu)) break;
            __builtin_amdgcn_s_sleep(1);
          }
          kind = (uint32_t)((w >> 32) & 3u);
        }
        // lanes 0.. up to (and including) the first inclusive one
        const uint64_t inc = __ballot(p >= 0 && kind == kTileIncl);
        const int stop = inc ? __ffsll((long long)inc) - 1 : kWave;
        uint32_t add = (lane <= stop && p >= 0) ? (uint32_t)w : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) add += __shfl_xor(add, o, kWave);
        prefix += add;
        if (inc || top - kWave < 0) break;
        top -= kWave;
      }
      if (t == 0) {
        __hip_atomic_store(state + ti, tile_word(epoch, kTileIncl, prefix + agg),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_prefix = prefix;
      }
    }
  }
  __syncthreads();
  uint32_t run = ex + s_prefix;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    tile[pad_idx(t * IT + k)] = run;
    // COUNT: the dst whose edges cross the edge capacity truncates the layer
    // at its first edge — the selection skips a dst that does not fit whole,
    // so e_size never covers unwritten edge slots (their ids are garbage)
    if (COUNT && run <= ca.e_cap && run + v[k] > ca.e_cap) ca.sizes[1] = run;
    run += v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const uint32_t j = k * kScanThreads + t;
    const uint64_t i = base + j;
    if (i <= n) out[i] = tile[pad_idx(j)];
    if (COUNT && i == n) {  // e_size = co[v], clamped to the edge capacity
      // the overflow flag has ONE writer, this item's thread, for both
      // capacities: a store from another workgroup could land after it
      const uint32_t e = tile[pad_idx(j)];
      if (e <= ca.e_cap) ca.sizes[1] = e;  // (else the crossing dst above wrote it)
      ca.sizes[3] = (v_req > ca.v_cap ? 1u : 0u) | (e > ca.e_cap ? 1u : 0u);
    }
  }
}

static uint32_t next_epoch(nts_hip_ctx* ctx) {
  ctx->scan_epoch = (ctx->scan_epoch + 1) & 0x3FFFFFFFu;
  if (ctx->scan_epoch == 0) ctx->scan_epoch = 1;  // 0: the state words' initial value
  return ctx->scan_epoch;
}
uint32_t scan_next_epoch(nts_hip_ctx* ctx) { return next_epoch(ctx); }

size_t scan1_state_elems(uint64_t n_cap) { return (n_cap / kScanTile + 1 + 63) / 64 * 64; }



int scan1_exclusive(nts_hip_ctx* ctx, const uint32_t* in, uint32_t* out, const uint32_t* n_dev,
                    uint64_t n_cap, hipStream_t stream) {
  const uint64_t nb = n_cap / kScanTile + 1;
  NTS_RET(ensure_scan_state(ctx, scan1_state_elems(n_cap)));
  hipLaunchKernelGGL((k_scan1<false, kScanItems>), dim3((uint32_t)nb), dim3(kScanThreads), 0, stream, in, out,
                     n_dev, n_cap, ctx->scan_state, next_epoch(ctx), scan_ticket(ctx), CountArgs{});
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

// Two-kernel count + scan (NTS_SCAN1=0): per-tile totals of the counts (the
// counts themselves written to co), then k_scan_down over co in place (it
// also writes e_size).  No tile waits on another tile's published state.
// Measured against the single-pass form next to the training stream (one
// MI355X, bench): C2 0.857 vs 0.851 ms/step, C3 0.708 vs 0.699, GPU sampler
// alone 4.84 vs 5.07 G edges/s at C2 — the single-pass form stays the default.
__global__ __launch_bounds__(kScanThreads) void k_count_reduce(CountArgs ca,
                                                               uint32_t* __restrict__ co,
                                                               uint32_t* __restrict__ partials) {
  const int t = threadIdx.x;
  const uint32_t v_req = *ca.v_in;
  const uint64_t n = min(v_req, ca.v_cap);
  if (blockIdx.x == 0 && t == 0) {
    ca.sizes[0] = (uint32_t)n;
    ca.sizes[3] = v_req > ca.v_cap ? 1u : 0u;
  }
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  uint32_t s = 0;
  if (base < n) {
    uint32_t x[kScanItems];
    count_items(ca, base, n, x);
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
      const uint64_t i = base + (uint64_t)k * kScanThreads + t;
      if (i < n) co[i] = x[k];
      s += x[k];
    }
  }
  __shared__ uint32_t wsum[kScanThreads / kWave];
  uint32_t tot;
  (void)block_excl_scan(s, wsum, &tot);
  if (t == 0) partials[blockIdx.x] = tot;
}

size_t count_scan_tmp_elems(uint64_t v_cap) { return scan_tmp_elems<uint32_t>(v_cap) + 64; }

// -DNTS_SCAN1=0: the two-kernel scans for count_scan and the frontier
// compaction (A/B); default the single-pass look-back scans
bool scan1_enabled() {  // compile-time A/B: -DNTS_SCAN1=0
#ifdef NTS_SCAN1
  return NTS_SCAN1 != 0;
#else
  return true;
#endif
}

int count_scan(nts_hip_ctx* ctx, const CountArgs& ca, uint32_t* co, hipStream_t stream,
               uint32_t* tmp) {
  if (!scan1_enabled() && tmp) {
    const uint64_t nb = (uint64_t)ca.v_cap / kScanTile + 1;
    uint32_t* partials = tmp;
    uint32_t* rest = tmp + (nb + 1 + 63) / 64 * 64;
    hipLaunchKernelGGL(k_count_reduce, dim3((uint32_t)nb), dim3(kScanThreads), 0, stream, ca, co,
                       partials);
    NTS_LAUNCH_CHECK();
    if (nb <= kScanDirectTiles) {
      hipLaunchKernelGGL((k_scan_down<uint32_t, true, true>), dim3((uint32_t)nb),
                         dim3(kScanThreads), 0, stream, (const uint32_t*)co, co,
                         (const uint32_t*)ca.sizes, (uint64_t)ca.v_cap, (const uint32_t*)partials,
                         ca.sizes, ca.e_cap);
    } else {
      NTS_RET(scan_exclusive<uint32_t>(partials, partials, nullptr, nb, rest, stream));
      hipLaunchKernelGGL((k_scan_down<uint32_t, false, true>), dim3((uint32_t)nb),
                         dim3(kScanThreads), 0, stream, (const uint32_t*)co, co,
                         (const uint32_t*)ca.sizes, (uint64_t)ca.v_cap, (const uint32_t*)partials,
                         ca.sizes, ca.e_cap);
    }
    NTS_LAUNCH_CHECK();
    return NTS_OK;
  }
  constexpr int kCountItems = 4;
  const uint64_t nb = (uint64_t)ca.v_cap / (kScanThreads * kCountItems) + 1;
  NTS_RET(ensure_scan_state(ctx, (nb + 63) / 64 * 64));
  hipLaunchKernelGGL((k_scan1<true, kCountItems>), dim3((uint32_t)nb), dim3(kScanThreads), 0, stream, nullptr,
                     co, nullptr, (uint64_t)ca.v_cap, ctx->scan_state, next_epoch(ctx), scan_ticket(ctx), ca);
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
// stable LSD radix sort: D-bit digits (D <= 9, passes = ceil(bits / 9)),
// 4096-item tiles.  Per pass: per-tile digit counts (digit-major, row stride
// nb = the capacity's tile count), a scan of each digit's row over the live
// tiles (one workgroup per digit, the row totals to `totals`), then a scatter
// that adds the digits' exclusive prefix over the totals (scanned per
// workgroup in LDS) and in which each wave ranks its 1,024
// contiguous items against a running per-wave digit count in LDS (match-any by
// ballots, no barrier inside the item loop), the tile is reordered by digit in
// LDS and written out in runs (coalesced stores).
// Tiles past the device-side count n exit at once.
// ============================================================================
template <int IT>
__global__ __launch_bounds__(kRadixThreads) void k_radix_hist(const uint32_t* __restrict__ keys,
                                                              const uint32_t* n_dev,
                                                              uint64_t n_cap, uint32_t shift,
                                                              uint32_t mask, uint32_t* hist,
                                                              uint32_t nb) {
  __shared__ uint32_t h[kRadixMaxBins];
  const int t = threadIdx.x;
  const uint32_t bins = mask + 1;
  for (uint32_t d = t; d < bins; d += kRadixThreads) h[d] = 0;
  __syncthreads();
  const uint64_t n = n_dev ? (uint64_t)*n_dev : n_cap;
  const uint64_t base = (uint64_t)blockIdx.x * (kRadixThreads * IT);
  if (base >= n) return;  // past the end: k_radix_rowscan reads only the tiles below n
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const uint64_t i = base + (uint64_t)k * kRadixThreads + t;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & mask], 1u);
  }
  __syncthreads();
  for (uint32_t d = t; d < bins; d += kRadixThreads) hist[(uint64_t)d * nb + blockIdx.x] = h[d];
}

// digit d = blockIdx.x: exclusive scan of hist[d nb .. d nb + live tiles) in
// place, its total to totals[d].  Replaces a device-wide scan of the whole
// bins x nb array (sized by the capacity, most of it zeros past n): no tile
// waits on another, and the grid is the digit count, not the capacity.
__global__ __launch_bounds__(kRadixThreads) void k_radix_rowscan(uint32_t* __restrict__ hist,
                                                                 const uint32_t* n_dev, uint64_t n_cap,
                                                                 uint32_t nb, uint32_t tile,
                                                                 uint32_t* __restrict__ totals) {
  __shared__ uint32_t wsum[kRadixThreads / kWave];
  const int t = threadIdx.x;
  const uint64_t n = n_dev ? (uint64_t)*n_dev : n_cap;
  const uint32_t live = (uint32_t)((n + tile - 1) / tile);  // <= nb
  uint32_t* row = hist + (uint64_t)blockIdx.x * nb;
  constexpr int kPer = 4;  // consecutive entries per thread
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < live; c0 += kRadixThreads * kPer) {
    uint32_t v[kPer], sum = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t j = c0 + t * kPer + k;
      v[k] = j < live ? row[j] : 0u;
      sum += v[k];
    }
    uint32_t tot;
    uint32_t run = carry + block_excl_scan(sum, wsum, &tot);
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t j = c0 + t * kPer + k;
      if (j < live) row[j] = run;
      run += v[k];
    }
    carry += tot;
    __syncthreads();  // wsum is reused by the next chunk
  }
  if (t == 0) totals[blockIdx.x] = carry;
}

template <int IT>
__global__ __launch_bounds__(kRadixThreads) void k_radix_scatter(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out, const uint32_t* n_dev,
    uint64_t n_cap, uint32_t shift, uint32_t dbits, const uint32_t* __restrict__ hist,
    uint32_t nb, const uint32_t* __restrict__ totals, const uint32_t* __restrict__ p1_in,
    uint32_t* __restrict__ p1_out, const uint32_t* __restrict__ p2_in, uint32_t* __restrict__ p2_out) {
  __shared__ RadixTileLds<IT> sm;
  const uint64_t n = n_dev ? (uint64_t)*n_dev : n_cap;
  if ((uint64_t)blockIdx.x * (kRadixThreads * IT) >= n) return;  // whole tile past the end
  const uint32_t bins = 1u << dbits;
  {  // the digits' starts: exclusive scan of the row totals (thread t: digits 2t, 2t + 1)
    static_assert(2 * kRadixThreads == kRadixMaxBins, "two digits per thread");
    const int t = threadIdx.x;
    const uint32_t c0 = 2u * t < bins ? totals[2 * t] : 0u;
    const uint32_t c1 = 2u * t + 1 < bins ? totals[2 * t + 1] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan(c0 + c1, sm.wsum, &tot);
    if (2u * t < bins) sm.gstart[2 * t] = ex;
    if (2u * t + 1 < bins) sm.gstart[2 * t + 1] = ex + c0;
    // (radix_tile_order's first barrier orders these before the reads below)
  }
  uint32_t loc[IT];
  radix_tile_order(sm, keys_in, vals_in, n, shift, dbits, [](uint32_t, uint32_t) {}, [&] {
    for (uint32_t d = threadIdx.x; d < bins; d += kRadixThreads)
      sm.gstart[d] += hist[(uint64_t)d * nb + blockIdx.x];
  }, loc);
  const uint32_t cnt = radix_tile_count<IT>(n), mask = (1u << dbits) - 1u;
  for (uint32_t i = threadIdx.x; i < cnt; i += kRadixThreads) {
    const uint32_t k = sm.sk[i], pos = radix_tile_pos(sm, i, k, shift, mask);
    keys_out[pos] = k;
    if (vals_out) vals_out[pos] = sm.sv[i];
  }
  // payloads (vals_in NULL: the values are the items' indices): read in index
  // order (coalesced), moved into the digit order through sm.sv, written in
  // the keys' runs
  auto payload = [&](const uint32_t* __restrict__ pin, uint32_t* __restrict__ pout) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint64_t wbase = (uint64_t)blockIdx.x * (kRadixThreads * IT) + (uint64_t)w * (IT * kWave);
    uint32_t pv[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const uint64_t i = wbase + (uint64_t)k * kWave + lane;
      pv[k] = i < n ? pin[i] : 0u;
    }
    __syncthreads();  // every read of sm.sv above is done
#pragma unroll
    for (int k = 0; k < IT; ++k)
      if (wbase + (uint64_t)k * kWave + lane < n) sm.sv[loc[k]] = pv[k];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cnt; i += kRadixThreads)
      pout[radix_tile_pos(sm, i, sm.sk[i], shift, mask)] = sm.sv[i];
  };
  if (p1_out) payload(p1_in, p1_out);
  if (p2_out) payload(p2_in, p2_out);
}

static size_t radix_tmp_bytes_t(uint64_t n_cap, uint32_t tile) {
  uint64_t nb = (n_cap + tile - 1) / tile;
  if (nb == 0) nb = 1;
  size_t hist = (size_t)kRadixMaxBins * nb + 1;
  size_t elems = 2 * ((n_cap + 63) / 64 * 64) + (hist + 63) / 64 * 64 + kRadixMaxBins + 64;
  return elems * sizeof(uint32_t);
}

size_t radix_tmp_bytes(uint64_t n_cap) { return radix_tmp_bytes_t(n_cap, kRadixTile); }
size_t radix_pass_tmp_bytes(uint64_t n_cap) { return radix_tmp_bytes_t(n_cap, kRadixThreads * kRadixPassItems); }

static uint32_t* radix_totals(void* tmp, uint64_t n_cap, uint32_t tile) {
  const uint32_t nb = ceil_div(n_cap, tile);
  const uint64_t n_al = (n_cap + 63) / 64 * 64;
  return (uint32_t*)tmp + 2 * n_al + ((uint64_t)kRadixMaxBins * nb + 1 + 63) / 64 * 64;
}

// one pass: digit counts per tile, their per-digit scan, the stable scatter
template <int IT>
static void radix_pass(const uint32_t* ksrc, const uint32_t* vsrc, uint32_t* kdst, uint32_t* vdst,
                       const uint32_t* n_dev, uint64_t n_cap, uint32_t shift, uint32_t dbits,
                       void* tmp, hipStream_t stream, const RadixPayload& pl = RadixPayload{}) {
  constexpr uint32_t tile = kRadixThreads * IT;
  const uint32_t nb = ceil_div(n_cap, tile);
  const uint64_t n_al = (n_cap + 63) / 64 * 64;
  uint32_t* hist = (uint32_t*)tmp + 2 * n_al;
  uint32_t* totals = radix_totals(tmp, n_cap, tile);
  const uint32_t mask = (1u << dbits) - 1u;
  hipLaunchKernelGGL(k_radix_hist<IT>, dim3(nb), dim3(kRadixThreads), 0, stream, ksrc, n_dev, n_cap,
                     shift, mask, hist, nb);
  hipLaunchKernelGGL(k_radix_rowscan, dim3(mask + 1), dim3(kRadixThreads), 0, stream, hist, n_dev,
                     n_cap, nb, tile, totals);
  hipLaunchKernelGGL(k_radix_scatter<IT>, dim3(nb), dim3(kRadixThreads), 0, stream, ksrc, vsrc, kdst,
                     vdst, n_dev, n_cap, shift, dbits, (const uint32_t*)hist, nb,
                     (const uint32_t*)totals, pl.p1_in, pl.p1_out, pl.p2_in, pl.p2_out);
}

int radix_sort_pairs(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* keys_out,
                     uint32_t* vals_out, const uint32_t* n_dev, uint64_t n_cap, uint32_t bits,
                     void* tmp, hipStream_t stream, nts_hip_ctx* ctx) {
  (void)ctx;  // (the device-wide look-back scan's state lived there)
  if (n_cap == 0) return NTS_OK;
  const uint64_t n_al = (n_cap + 63) / 64 * 64;
  uint32_t* ktmp = (uint32_t*)tmp;
  uint32_t* vtmp = ktmp + n_al;
  if (bits < 1) bits = 1;
  const int npass = (int)((bits + kRadixMaxBits - 1) / kRadixMaxBits);
  const uint32_t dbits = (bits + npass - 1) / npass;
  const uint32_t* ksrc = keys_in;
  const uint32_t* vsrc = vals_in;
  for (int p = 0; p < npass; ++p) {
    bool to_out = ((npass - 1 - p) % 2) == 0;
    uint32_t* kdst = to_out ? keys_out : ktmp;
    uint32_t* vdst = to_out ? vals_out : vtmp;
    radix_pass<kRadixItems>(ksrc, vsrc, kdst, vdst, n_dev, n_cap, dbits * p, dbits, tmp, stream);
    NTS_LAUNCH_CHECK();
    ksrc = kdst;
    vsrc = vdst;
  }
  return NTS_OK;
}

int radix_pass_pairs(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* keys_out,
                     uint32_t* vals_out, const uint32_t* n_dev, uint64_t n_cap, uint32_t shift,
                     uint32_t dbits, void* tmp, hipStream_t stream, const uint32_t** totals,
                     const RadixPayload& pl) {
  NTS_CHECK_ARG(dbits >= 1 && dbits <= (uint32_t)kRadixMaxBits, "radix digit of 1..9 bits");
  NTS_CHECK_ARG(n_cap > 0, "empty capacity");
  NTS_CHECK_ARG(!(pl.p1_out || pl.p2_out) || !vals_in, "payloads need index values (vals_in NULL)");
  radix_pass<kRadixPassItems>(keys_in, vals_in, keys_out, vals_out, n_dev, n_cap, shift, dbits, tmp,
                              stream, pl);
  NTS_LAUNCH_CHECK();
  *totals = radix_totals(tmp, n_cap, kRadixThreads * kRadixPassItems);
  return NTS_OK;
}

}  // namespace nts_hip
