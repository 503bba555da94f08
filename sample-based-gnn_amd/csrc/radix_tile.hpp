// One 4096-item tile of a stable LSD radix pass (shared by the generic sort
// in primitives.hip and the sampler's CSR transpose in sampler.hip).
// Internal, not part of the C-ABI.
#pragma once
#include "common.hpp"

namespace nts_hip {

constexpr int kRadixThreads = 256;
constexpr int kRadixItems = 16;  // items per thread of the generic sort's tiles
constexpr int kRadixTile = kRadixThreads * kRadixItems;  // 4096
constexpr int kRadixPassItems = 4;  // radix_pass_pairs' tiles: 1,024 items
constexpr int kRadixMaxBits = 9;
constexpr int kRadixMaxBins = 1 << kRadixMaxBits;

// IT items per thread: tiles of 256 IT items (the generic sort 16; the
// sampler's single CSR pass 4 — four times the workgroups on a layer's ~0.3-1.4
// M edges, each a quarter of the serial ranking chain)
template <int IT>
struct RadixTileLds {
  uint32_t wh[kRadixThreads / kWave][kRadixMaxBins];  // per-wave counts -> offsets
  uint32_t gstart[kRadixMaxBins];  // digit d's global start for this tile
  uint32_t lstart[kRadixMaxBins];  // ... and its start in the tile's digit order
  uint32_t sk[kRadixThreads * IT], sv[kRadixThreads * IT];  // the tile in digit order
  uint32_t wsum[kRadixThreads / kWave];
};

// Tile blockIdx.x of a pass over n items (base = blockIdx.x * 256 IT < n):
// each wave ranks its 64 IT contiguous items against a running per-wave digit
// count in LDS (match-any by ballots, no barrier inside the item loop) and the
// tile is reordered by digit in LDS: on return sm.sk / sm.sv hold it in digit
// order (stable), and item i of that order goes to output position
// radix_tile_pos(sm, i, ...) — consecutive items of a digit's run to
// consecutive positions.  publish(d, count) is told the tile's count of every
// digit first (digit d by thread d % 256), then each thread's gstart() sets
// sm.gstart[d] — where the tile's run of digit d starts in the output — for
// its digits d = t, t + 256 (< bins), their counts in sm.lstart[d].
// vals_in == nullptr: values are the item indices.
// loc[k]: where this thread's item k (index base + 1024 w + 64 k + lane) went
// in the digit order (so payloads read later in index order can follow it).
template <int IT, class Pub, class GS>
__device__ __forceinline__ void radix_tile_order(RadixTileLds<IT>& sm, const uint32_t* __restrict__ keys_in,
                                                 const uint32_t* __restrict__ vals_in, uint64_t n,
                                                 uint32_t shift, uint32_t dbits, Pub&& publish,
                                                 GS&& gstart, uint32_t (&loc)[IT]) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint64_t base = (uint64_t)blockIdx.x * (kRadixThreads * IT);
  const uint32_t mask = (1u << dbits) - 1u, bins = mask + 1;
  for (uint32_t d = t; d < bins; d += kRadixThreads)
#pragma unroll
    for (int ww = 0; ww < kRadixThreads / kWave; ++ww) sm.wh[ww][d] = 0;
  __syncthreads();
  // wave w ranks items base + 64 IT w + 64 k + lane (index order) against its
  // running digit counts
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const uint64_t wbase = base + (uint64_t)w * (IT * kWave);
  uint32_t key[IT], val[IT], rank[IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const uint64_t i = wbase + (uint64_t)k * kWave + lane;
    const bool valid = i < n;
    key[k] = valid ? keys_in[i] : 0u;
    val[k] = valid ? (vals_in ? vals_in[i] : (uint32_t)i) : 0u;
  }
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const bool valid = wbase + (uint64_t)k * kWave + lane < n;
    const uint32_t d = (key[k] >> shift) & mask;
    uint64_t peers = __ballot(valid);
    for (uint32_t b = 0; b < dbits; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    const uint32_t prev = sm.wh[w][d];
    const uint32_t before = (uint32_t)__popcll(peers & lt_mask);
    rank[k] = prev + before;
    if (valid && before == 0) sm.wh[w][d] = prev + (uint32_t)__popcll(peers);
  }
  __syncthreads();
  // per digit: the waves' counts -> their offsets within the digit's slice
  // (wh), the tile's count of the digit (lstart, scanned below) and its
  // start in the output (gstart)
  for (uint32_t d = t; d < bins; d += kRadixThreads) {
    uint32_t run = 0;
#pragma unroll
    for (int ww = 0; ww < kRadixThreads / kWave; ++ww) {
      const uint32_t c = sm.wh[ww][d];
      sm.wh[ww][d] = run;
      run += c;
    }
    sm.lstart[d] = run;
    publish(d, run);
  }
  gstart();  // sm.gstart of this thread's digits (t, t + 256) from their counts in sm.lstart
  __syncthreads();
  {  // exclusive scan of the tile's digit counts: thread t owns digits 2t, 2t + 1
    static_assert(2 * kRadixThreads == kRadixMaxBins, "two digits per thread");
    const uint32_t c0 = 2u * t < bins ? sm.lstart[2 * t] : 0u;
    const uint32_t c1 = 2u * t + 1 < bins ? sm.lstart[2 * t + 1] : 0u;
    uint32_t inc = c0 + c1;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o);
      if (lane >= o) inc += y;
    }
    if (lane == kWave - 1) sm.wsum[w] = inc;
    __syncthreads();
    uint32_t before = 0;
#pragma unroll
    for (int ww = 0; ww < kRadixThreads / kWave; ++ww) before += ww < w ? sm.wsum[ww] : 0u;
    const uint32_t ex = before + inc - (c0 + c1);
    if (2u * t < bins) sm.lstart[2 * t] = ex;
    if (2u * t + 1 < bins) sm.lstart[2 * t + 1] = ex + c0;
  }
  __syncthreads();
  // the tile in digit order through LDS, then handed out in index order:
  // consecutive LDS slots of one digit go to consecutive output positions
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    if (wbase + (uint64_t)k * kWave + lane < n) {
      const uint32_t d = (key[k] >> shift) & mask;
      loc[k] = sm.lstart[d] + sm.wh[w][d] + rank[k];
      sm.sk[loc[k]] = key[k];
      sm.sv[loc[k]] = val[k];
    }
  }
  __syncthreads();
}

// the tile's item count, and the output position of item i of the digit order
template <int IT>
__device__ __forceinline__ uint32_t radix_tile_count(uint64_t n) {
  constexpr uint64_t T = kRadixThreads * IT;
  const uint64_t base = (uint64_t)blockIdx.x * T;
  return (uint32_t)(n - base < T ? n - base : T);
}
template <int IT>
__device__ __forceinline__ uint32_t radix_tile_pos(const RadixTileLds<IT>& sm, uint32_t i, uint32_t key,
                                                   uint32_t shift, uint32_t mask) {
  const uint32_t d = (key >> shift) & mask;
  return sm.gstart[d] + (i - sm.lstart[d]);
}

}  // namespace nts_hip
