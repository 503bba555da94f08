// Multi-hop neighbour sampler, one hop per call, entirely on the device.
//
// Reference semantics (CPU FastSampler::sample_fast, core/ntsFastSampler.hpp:962-1140):
//   per dst d:  num = min(deg(d), fanout)  (fanout < 0 -> deg)      init_co_only (FullyRepGraph.hpp:530-539)
//               deg > fanout : draw uniform positions in [0,deg) by rejection until
//                              `num` distinct ones (unordered_map, :1026-1038)
//               else         : take every neighbour in CSC order (:1040-1048)
//   frontier  : bitmap of sampled ids scanned in ascending order -> `source`,
//               src_index (:1064-1083); row_indices relabelled (:1085-1099)
//   csc_to_csr (core/coocsc.hpp:82-111), WeightCompute (core/coocsc.hpp:301-324)
//
// MI355X design:
//   * one wave per destination; the copy path is a coalesced 64-lane stride,
//     the rejection path draws up to 64 candidates per round and resolves
//     "first `num` distinct in draw order" with ballots (no hash map),
//   * PHILOX mode: every dst owns an independent counter-based stream -> fully
//     parallel and deterministic; MT19937 modes replay the reference's single
//     sequential generator with one wave (bit-exact neighbour sets),
//   * frontier dedup = byte map + popcount scan over V/4096 tiles: ascending
//     `source` without the reference GPU path's O(V) atomics (stage3,
//     cuda/ntsCUDATransferKernel.cuh:1107-1125) and without host round trips,
//   * CSR transpose = stable radix sort of (local src, edge id) -> identical to
//     the reference's serial fill order (ascending dst), atomic-free.
#include "common.hpp"

#include <type_traits>

namespace nts_hip {

constexpr int kSelThreads = 256;
constexpr int kSelWaves = kSelThreads / kWave;
constexpr int kSetCap = 1024;  // max fanout of the rejection path

// ---------------------------------------------------------------------------
// random words
// ---------------------------------------------------------------------------
// Word `idx` of the PHILOX stream of (dst, layer, batch_seq).
__device__ __forceinline__ uint32_t philox_word(uint64_t seed, uint32_t dst, uint32_t layer,
                                                uint64_t batch_seq, uint32_t idx) {
  uint4 c = make_uint4(idx >> 2, dst, layer, (uint32_t)batch_seq);
  uint2 k = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32) ^ (uint32_t)(batch_seq >> 32));
  uint4 r = philox4x32_10(c, k);
  uint32_t j = idx & 3u;
  return j == 0 ? r.x : (j == 1 ? r.y : (j == 2 ? r.z : r.w));
}

// uniform_int_distribution<int>(0, range-1) acceptance test for one 32-bit word.
// Lemire (libstdc++ >= 11, uniform_int_dist.h:246-263): a word is rejected iff
// low32(x*range) < (-range) % range; accepted words yield high32(x*range).
// DIV (libstdc++ <= 10): scaling = 0xFFFFFFFF/range, reject x >= range*scaling,
// value = x / scaling.
struct Draw {
  uint32_t range, thr, scaling, past;
  bool lemire;
  __device__ __forceinline__ void init(uint32_t r, bool lem) {
    range = r;
    lemire = lem;
    thr = (0u - r) % r;
    scaling = 0xFFFFFFFFu / r;
    past = r * scaling;
  }
  __device__ __forceinline__ bool apply(uint32_t x, uint32_t& v) const {
    if (lemire) {
      uint64_t m = (uint64_t)x * range;
      v = (uint32_t)(m >> 32);
      return (uint32_t)m >= thr;
    }
    v = x / scaling;
    return x < past;
  }
};

// ---------------------------------------------------------------------------
// per-layer kernels
// ---------------------------------------------------------------------------
struct SelectArgs {
  const uint64_t* goff;
  const uint32_t* grows;
  const uint32_t* dst;
  const uint32_t* co;
  uint32_t* sizes;  // [0] v, [1] e (count_scan wrote them)
  uint32_t* ans;
  uint32_t* edst;
  uint8_t* marks;
  uint32_t e_cap;
  int fanout;
  uint32_t layer;
  uint64_t batch_seq;
  uint64_t seed;
};

// Copy path: all neighbours of dst i in CSC order (coalesced stride).
__device__ __forceinline__ void copy_all(const SelectArgs& a, uint32_t i, uint64_t beg,
                                         uint32_t deg, uint32_t c, int lane) {
  for (uint32_t k = lane; k < deg; k += kWave) {
    uint32_t g = a.grows[beg + k];
    a.ans[c + k] = g;
    a.edst[c + k] = i;
    a.marks[g] = 1;
  }
}

// Rejection path: the first `need` distinct accepted draws, in draw order.
// `word(j)` returns the j-th word of this dst's stream.  Returns words consumed.
template <typename WordFn>
__device__ __forceinline__ uint32_t select_distinct(const SelectArgs& a, uint32_t i,
                                                    uint64_t beg, uint32_t deg, uint32_t need,
                                                    uint32_t c, int lane, uint32_t* set,
                                                    const Draw& dr, WordFn word) {
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t count = 0, consumed = 0;
  while (count < need) {
    const uint32_t remaining = need - count;
    // round width: fewer candidates when few are missing (cheaper dedup)
    const int R = remaining <= 12 ? 16 : (remaining <= 28 ? 32 : 64);
    uint32_t val = 0;
    bool ok = false;
    if (lane < R) ok = dr.apply(word(consumed + lane), val);
    bool dup = false;
    for (uint32_t j = 0; j < count; ++j) dup |= (set[j] == val);  // LDS broadcast reads
    const uint64_t okmask = __ballot(ok);
    // lane j's draw by v_readlane (a scalar broadcast), not __shfl's
    // ds_bpermute round trip per j
    for (int j = 0; j < R; ++j) {
      uint32_t vj = (uint32_t)__builtin_amdgcn_readlane((int)val, j);
      dup |= (j < lane) && ((okmask >> j) & 1ull) && (vj == val);
    }
    const bool isnew = ok && !dup;
    const uint64_t newmask = __ballot(isnew);
    const uint32_t nnew = __popcll(newmask);
    uint64_t take = newmask;
    if (nnew >= remaining) {
      // keep the first `remaining` new lanes; the stream is consumed up to the last one
      uint64_t m = newmask;
      for (uint32_t t = 1; t < remaining; ++t) m &= m - 1;
      const int last = __ffsll((long long)m) - 1;
      take = newmask & ((last == 63) ? ~0ull : ((2ull << last) - 1ull));
      consumed += (uint32_t)last + 1u;
    } else {
      consumed += (uint32_t)R;
    }
    if ((take >> lane) & 1ull) {
      const uint32_t slot = count + (uint32_t)__popcll(take & lt_mask);
      set[slot] = val;
      const uint32_t pos = c + slot;
      const uint32_t g = a.grows[beg + val];
      a.ans[pos] = g;
      a.edst[pos] = i;
      a.marks[g] = 1;
    }
    count += (uint32_t)__popcll(take);
    __builtin_amdgcn_wave_barrier();
  }
  return consumed;
}

// ---- fanout > kSetCap: distinct positions through an LDS hash set --------
// The reference CPU sampler takes any fanout (core/ntsFastSampler.hpp:1028-1048;
// its GPU path falls back to the first k neighbours past 1024,
// cuda/ntsCUDATransferKernel.cuh:852-881).  Same result as select_distinct —
// the first `need` distinct accepted draws, in draw order — with the kept
// positions in an open-addressing set (key = position + 1, 0 = empty, linear
// probing, capacity a power of two >= 2 x need) instead of a list scanned per
// candidate; repeats inside one 64-word round by lane shuffles.
constexpr uint32_t kBigFanoutMax = 16384;  // hash capacity 32 K words = 128 KB of LDS

__device__ __forceinline__ uint32_t pos_hash(uint32_t v, uint32_t mask) {
  return (v * 0x9E3779B1u) >> 7 & mask;
}
__device__ __forceinline__ bool hset_has(const uint32_t* h, uint32_t mask, uint32_t v) {
  for (uint32_t s = pos_hash(v, mask);; s = (s + 1) & mask) {
    const uint32_t k = h[s];
    if (k == v + 1) return true;
    if (k == 0) return false;
  }
}
__device__ __forceinline__ void hset_put(uint32_t* h, uint32_t mask, uint32_t v) {
  for (uint32_t s = pos_hash(v, mask);; s = (s + 1) & mask) {
    const uint32_t old = atomicCAS(&h[s], 0u, v + 1);
    if (old == 0 || old == v + 1) return;
  }
}

// draws for one dst into out[0 .. need) (positions), whole wave; returns the
// words consumed.  The set (cap words) must be all zeros; it is zeroed again.
template <typename WordFn>
__device__ uint32_t select_distinct_hashed(uint32_t need, uint32_t* hset, uint32_t cap, int lane,
                                           uint32_t deg, uint32_t thr, bool lemire, uint32_t* out,
                                           WordFn word) {
  const uint32_t mask = cap - 1;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t count = 0, consumed = 0;
  while (count < need) {
    const uint32_t remaining = need - count;
    uint32_t val = 0;
    bool ok;
    const uint32_t x = word(consumed + lane);
    if (lemire) {
      const uint64_t m = (uint64_t)x * deg;
      val = (uint32_t)(m >> 32);
      ok = (uint32_t)m >= thr;
    } else {
      val = x / thr;
      ok = x < deg * thr;
    }
    bool dup = ok && hset_has(hset, mask, val);
    const uint64_t okmask = __ballot(ok);
    for (int j = 0; j < kWave; ++j) {
      const uint32_t vj = (uint32_t)__builtin_amdgcn_readlane((int)val, j);
      dup |= (j < lane) && ((okmask >> j) & 1ull) && (vj == val);
    }
    const uint64_t newmask = __ballot(ok && !dup);
    uint64_t take = newmask;
    if ((uint32_t)__popcll(newmask) >= remaining) {
      uint64_t m = newmask;
      for (uint32_t t = 1; t < remaining; ++t) m &= m - 1;
      const int last = __ffsll((long long)m) - 1;
      take = newmask & ((last == 63) ? ~0ull : ((2ull << last) - 1ull));
      consumed += (uint32_t)last + 1u;
    } else {
      consumed += (uint32_t)kWave;
    }
    if ((take >> lane) & 1ull) {
      hset_put(hset, mask, val);
      out[count + (uint32_t)__popcll(take & lt_mask)] = val;
    }
    count += (uint32_t)__popcll(take);
    __syncthreads();  // the puts land before the next round's probes
  }
  for (uint32_t k = lane; k < cap; k += kWave) hset[k] = 0u;
  __syncthreads();
  return consumed;
}

// PHILOX, fanout > kSetCap: one wave per block (the hash set takes the LDS).
// Positions go to ans first (in place), then to neighbour ids.
__global__ __launch_bounds__(kWave) void k_select_philox_big(SelectArgs a, uint32_t cap) {
  extern __shared__ uint32_t hset[];
  const int lane = threadIdx.x;
  for (uint32_t k = lane; k < cap; k += kWave) hset[k] = 0u;
  __syncthreads();
  const uint32_t v = a.sizes[0];
  for (uint32_t i = blockIdx.x; i < v; i += gridDim.x) {
    const uint32_t d = a.dst[i];
    const uint64_t beg = a.goff[d];
    const uint32_t deg = (uint32_t)(a.goff[d + 1] - beg);
    const uint32_t c = a.co[i];
    const uint32_t n = a.co[i + 1] - c;
    if (c + n > a.e_cap) continue;  // capacity overflow (flagged by count_scan)
    if (n == deg) {
      copy_all(a, i, beg, deg, c, lane);
      continue;
    }
    if (n == 0) continue;
    const uint64_t seed = a.seed, bs = a.batch_seq;
    const uint32_t layer = a.layer;
    select_distinct_hashed(n, hset, cap, lane, deg, (0u - deg) % deg, true, a.ans + c,
                           [&](uint32_t j) { return philox_word(seed, d, layer, bs, j); });
    for (uint32_t k = lane; k < n; k += kWave) {
      const uint32_t g = a.grows[beg + a.ans[c + k]];
      a.ans[c + k] = g;
      a.edst[c + k] = i;
      a.marks[g] = 1;
    }
  }
}

// PHILOX: one wave per destination, grid-stride.
__global__ __launch_bounds__(kSelThreads) void k_select_philox(SelectArgs a) {
  __shared__ uint32_t sets[kSelWaves][kSetCap];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t v = a.sizes[0];
  uint32_t* set = sets[w];
  const uint32_t nw = gridDim.x * kSelWaves;
  for (uint32_t i = blockIdx.x * kSelWaves + w; i < v; i += nw) {
    const uint32_t d = a.dst[i];
    const uint64_t beg = a.goff[d];
    const uint32_t deg = (uint32_t)(a.goff[d + 1] - beg);
    const uint32_t c = a.co[i];
    const uint32_t n = a.co[i + 1] - c;
    if (c + n > a.e_cap) continue;  // capacity overflow (flagged by count_scan)
    if (n == deg) {
      copy_all(a, i, beg, deg, c, lane);
    } else if (n > 0) {
      Draw dr;
      dr.init(deg, true);
      const uint64_t seed = a.seed;
      const uint32_t layer = a.layer;
      const uint64_t bs = a.batch_seq;
      select_distinct(a, i, beg, deg, n, c, lane, set, dr, [&](uint32_t j) {
        return philox_word(seed, d, layer, bs, j);
      });
    }
  }
}

// PHILOX for fanout <= 16: four destinations per wave, one 16-lane group each
// (a round of 16 candidates covers a fanout-10 draw; the per-destination chain
// dst -> offsets -> row ids is latency-bound, so four chains per wave in
// flight instead of one).  Same result as k_select_philox: the first `need`
// distinct accepted draws of the destination's stream, in draw order.
constexpr int kGrp = 16;
constexpr int kGrpPerWave = kWave / kGrp;

// dup |= an earlier accepted lane J of the 16-lane group drew val (J < gl):
// lane J of each 16-lane row by a DPP row broadcast (row_newbcast) instead of
// __shfl's ds_bpermute — sampler alone 5.98-6.02 -> 6.04-6.07 G edges/s,
// bit-identical (scripts/ab/r05_ba.sh)
template <int J>
struct GrpDupScan {
  static __device__ __forceinline__ void run(bool& dup, uint32_t val, int gl, uint32_t okm) {
    const uint32_t vj = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)val, 0x150 + J, 0xF, 0xF, false);
    dup |= (J < gl) && ((okm >> J) & 1u) && (vj == val);
    GrpDupScan<J + 1>::run(dup, val, gl, okm);
  }
};
template <>
struct GrpDupScan<kGrp> {
  static __device__ __forceinline__ void run(bool&, uint32_t, int, uint32_t) {}
};

__global__ __launch_bounds__(kSelThreads) void k_select_philox_g16(SelectArgs a) {
  __shared__ uint32_t sets[kSelWaves * kGrpPerWave][kGrp];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int gl = lane & (kGrp - 1), grp = lane >> 4;
  const int gib = w * kGrpPerWave + grp;
  uint32_t* set = sets[gib];
  const uint32_t gshift = kGrp * grp;
  const uint32_t lt16 = (1u << gl) - 1u;
  const uint32_t v = a.sizes[0];
  const uint32_t ng = gridDim.x * kSelWaves * kGrpPerWave;
  for (uint32_t i = blockIdx.x * kSelWaves * kGrpPerWave + gib; i < v; i += ng) {
    const uint32_t d = a.dst[i];
    const uint64_t beg = a.goff[d];
    const uint32_t deg = (uint32_t)(a.goff[d + 1] - beg);
    const uint32_t c = a.co[i];
    const uint32_t n = a.co[i + 1] - c;
    if (c + n > a.e_cap) continue;  // capacity overflow (flagged by count_scan)
    if (n == deg) {
      for (uint32_t k = gl; k < deg; k += kGrp) {
        const uint32_t g = a.grows[beg + k];
        a.ans[c + k] = g;
        a.edst[c + k] = i;
        a.marks[g] = 1;
      }
      continue;
    }
    if (n == 0) continue;
    Draw dr;
    dr.init(deg, true);
    uint32_t count = 0, consumed = 0;
    while (count < n) {  // group-uniform
      const uint32_t remaining = n - count;
      uint32_t val = 0;
      const bool ok = dr.apply(philox_word(a.seed, d, a.layer, a.batch_seq, consumed + gl), val);
      bool dup = false;
      for (uint32_t j = 0; j < count; ++j) dup |= (set[j] == val);
      const uint32_t okm = (uint32_t)(__ballot(ok) >> gshift) & 0xFFFFu;
      GrpDupScan<0>::run(dup, val, gl, okm);
      const bool isnew = ok && !dup;
      const uint32_t newm = (uint32_t)(__ballot(isnew) >> gshift) & 0xFFFFu;
      uint32_t take = newm;
      if ((uint32_t)__popc(newm) >= remaining) {
        uint32_t m = newm;
        for (uint32_t t = 1; t < remaining; ++t) m &= m - 1;
        const int last = __ffs(m) - 1;
        take = newm & ((2u << last) - 1u);
        consumed += (uint32_t)last + 1u;
      } else {
        consumed += kGrp;
      }
      if ((take >> gl) & 1u) {
        const uint32_t slot = count + (uint32_t)__popc(take & lt16);
        set[slot] = val;
        const uint32_t pos = c + slot;
        const uint32_t g = a.grows[beg + val];
        a.ans[pos] = g;
        a.edst[pos] = i;
        a.marks[g] = 1;
      }
      count += (uint32_t)__popc(take);
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// ---- MT19937 (reference stream) -------------------------------------------
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// tempering is invertible: the raw state word back from a tempered word
__device__ __forceinline__ uint32_t mt_untemper(uint32_t y) {
  y ^= y >> 18;
  y ^= (y << 15) & 0xefc60000u;
  uint32_t t = y;
#pragma unroll
  for (int k = 0; k < 4; ++k) t = y ^ ((t << 7) & 0x9d2c5680u);
  y = t;
  t = y;
#pragma unroll
  for (int k = 0; k < 2; ++k) t = y ^ (t >> 11);
  return t;
}

// The stream ring (nts_hip_ctx::mt_ring): word a of the stream since seeding
// at mt_ring[a % kMtRingWords]; block b (624 words, b = 0 the first twist
// after seeding) covers words [624 b, 624 b + 624).
constexpr uint32_t kMtRingBits = 25;
constexpr uint64_t kMtRingWords = 1ull << kMtRingBits;  // 128 MB of words
constexpr uint32_t kMtRingMask = (uint32_t)(kMtRingWords - 1);
constexpr uint64_t kMtPosMask = (1ull << 40) - 1;  // mt_done: position (40 bits) | seq << 40
// a layer's view of the stream: word i = stream word a0 + i, zero past the
// words generated for it (nw)
struct MtWords {
  const uint32_t* ring;
  uint64_t a0;
  uint32_t nw;
  __device__ __forceinline__ uint32_t operator[](uint32_t i) const {
    return i < nw ? ring[(uint32_t)(a0 + i) & kMtRingMask] : 0u;
  }
};
// std::mt19937's state after the stream's first `a` words (a > 0): the raw
// block holding word a - 1 (untempered from the ring) and _M_p = its index + 1
// (624: libstdc++ twists lazily on the next call); whole wave
__device__ __forceinline__ void mt_state_at(const uint32_t* ring, uint64_t a, uint32_t* mt_state,
                                            int lane) {
  const uint64_t last = a - 1, b = last / 624;
  const uint32_t p = (uint32_t)(last - b * 624) + 1u;
  for (int k = lane; k < 624; k += kWave)
    mt_state[k] = mt_untemper(ring[(uint32_t)(b * 624 + k) & kMtRingMask]);
  if (lane == 0) mt_state[624] = p;
}


// The reference draws from ONE sequential generator (random_uniform_int,
// core/ntsFastSampler.hpp:200-205) over the dsts in order, and a dst's word
// count is data dependent (rejections, repeated positions), so the stream
// positions form a serial chain.  Two kernels split the work:
//   k_mt_prep    (parallel) per-dst {c, n, deg, thr}: n = 0 for dsts that draw
//                nothing (copy path, omitted, overflow);
//   k_mt_serial  (ONE wave) resolves only the chain: which stream words each
//                dst consumes, and the positions it keeps (written into `ans`);
//   k_mt_rows    (parallel) positions -> row ids, edge dsts, frontier marks.
// k_mt_serial speculates: the wave is cut into K = 64/G groups of G lanes and
// evaluates K consecutive dsts at once, dst k at the stream position it would
// start at if every dst before it consumed exactly n words (no rejection, no
// repeat).  Within a group the first n distinct accepted draws are found in
// one shot: each accepted lane stores a sentinel, then ds_min's its lane id
// into an LDS table indexed by the drawn position (direct for deg <= TAB,
// hashed above it — a hash collision is detected and sent to the exact path),
// and reads back the earliest lane that drew the same position.  The first
// group always starts at the true position; group k+1 is kept iff groups
// 0..k consumed exactly their n words.  A dst whose draws do not complete
// inside its G-word window goes to the exact full-wave path (rounds of 64
// words, cross-round dedup through `set`).
struct MtInfo {
  uint32_t c, n, deg, thr;  // column offset, draws (0: none), range, Lemire threshold
};

// nn / cstat (chunked resolver, may be null): the draws per dst, and per
// chunk of csz dsts the expected extra words (repeats) and their
// variance: drawing the k-th distinct of `deg` positions takes a geometric
// number of words with success (deg - k) / deg — mean extra k / (deg - k),
// variance k deg / (deg - k)^2 (rejections, p < deg / 2^32, neglected).
__global__ void k_mt_prep(const uint64_t* __restrict__ goff, const uint32_t* __restrict__ dst,
                          const uint32_t* __restrict__ co, uint32_t* sizes, uint32_t e_cap,
                          int lemire, uint4* __restrict__ info, uint32_t* __restrict__ nn,
                          float2* __restrict__ cstat, uint32_t csz, const uint64_t* done,
                          uint64_t* a0p) {
  const uint32_t v = sizes[0];
  // the layer's first stream word, for the kernels after this one (the
  // resolver moves mt_done on)
  if (a0p && blockIdx.x == 0 && threadIdx.x == 0) *a0p = *done & kMtPosMask;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < v; i += gridDim.x * blockDim.x) {
    const uint32_t d = dst[i];
    const uint32_t deg = (uint32_t)(goff[d + 1] - goff[d]);
    const uint32_t c = co[i];
    const uint32_t n = co[i + 1] - c;
    const bool draw = n > 0 && n < deg && (uint64_t)c + n <= e_cap;
    uint32_t thr = 0;
    if (draw) thr = lemire ? (0u - deg) % deg : 0xFFFFFFFFu / deg;  // DIV: `scaling`
    info[i] = make_uint4(c, draw ? n : 0u, deg, thr);
    if (nn) {
      nn[i] = draw ? n : 0u;
      if (draw) {
        float m = 0.f, var = 0.f;
        const float fd = (float)deg;
        for (uint32_t k = 1; k < n; ++k) {
          const float r = fd - (float)k;
          m += (float)k / r;
          var += (float)k * fd / (r * r);
        }
        atomicAdd(&cstat[i / csz].x, m);
        atomicAdd(&cstat[i / csz].y, var);
      }
    }
  }
}

// The word source of the MT19937 walks: the stream ring (the layer's words,
// generated ahead by k_mt_ring_gen) or words staged in LDS; word r at
// tw[(fa + r) & fmask] for r < fnw, 0 past them.  q0: the next word's index.
struct MtStream {
  const uint32_t* tw;
  uint32_t q0;
  uint64_t fa = 0;
  uint32_t fmask = ~0u, fnw = ~0u;
  __device__ __forceinline__ uint32_t word(uint32_t r) const {
    return r < fnw ? tw[(uint32_t)(fa + r) & fmask] : 0u;
  }
};

__device__ __forceinline__ bool mt_apply(uint32_t x, uint32_t deg, uint32_t thr, bool lemire,
                                         uint32_t& v) {
  if (lemire) {
    const uint64_t m = (uint64_t)x * deg;
    v = (uint32_t)(m >> 32);
    return (uint32_t)m >= thr;
  }
  v = x / thr;                 // thr = scaling
  return x < deg * thr;        // past = range * scaling
}

// Exact path, whole wave: the first n distinct accepted draws of one dst in
// rounds of up to 64 words; positions -> ans[c + slot].
__device__ void mt_exact(MtStream& s, uint32_t* set, uint32_t* ans, uint32_t c, uint32_t n,
                         uint32_t deg, uint32_t thr, bool lemire, int lane) {
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t count = 0;
  while (count < n) {
    if (s.q0 >= s.fnw) {  // past the generated stream: sticky, the caller reports it
      s.q0 = s.fnw + 1;
      break;
    }
    const uint32_t remaining = n - count;
    const int R = remaining <= 12 ? 16 : (remaining <= 28 ? 32 : 64);
    uint32_t val = 0;
    bool ok = false;
    if (lane < R) ok = mt_apply(s.word(s.q0 + lane), deg, thr, lemire, val);
    bool dup = false;
    for (uint32_t j = 0; j < count; ++j) dup |= (set[j] == val);
    const uint64_t okmask = __ballot(ok);
    for (int j = 0; j < R; ++j) {
      const uint32_t vj = (uint32_t)__builtin_amdgcn_readlane((int)val, j);
      dup |= (j < lane) && ((okmask >> j) & 1ull) && (vj == val);
    }
    const bool isnew = ok && !dup;
    const uint64_t newmask = __ballot(isnew);
    uint64_t take = newmask;
    if ((uint32_t)__popcll(newmask) >= remaining) {
      uint64_t m = newmask;
      for (uint32_t t = 1; t < remaining; ++t) m &= m - 1;
      const int last = __ffsll((long long)m) - 1;
      take = newmask & ((last == 63) ? ~0ull : ((2ull << last) - 1ull));
      s.q0 += (uint32_t)last + 1u;
    } else {
      s.q0 += (uint32_t)R;
    }
    if ((take >> lane) & 1ull) {
      const uint32_t slot = count + (uint32_t)__popcll(take & lt_mask);
      set[slot] = val;
      ans[c + slot] = val;
    }
    count += (uint32_t)__popcll(take);
    __syncthreads();
  }
}

constexpr uint32_t kMtTab = 16384;  // LDS dedup table entries (all groups)
constexpr uint32_t kMtTaken = 0xFFFFFFFEu;  // exact path: position already kept

// Exact path for deg <= kMtTab, whole wave: the table is direct-mapped by
// position over all groups' regions.  Per round of 64 words: a position is
// new iff it is accepted, not marked kept by an earlier round, and no earlier
// lane of the round drew it (sentinel + ds_min of lane ids, as the fast
// path).  Kept positions are marked, and unmarked when the dst is done, so
// the table holds no marks between dsts.
__device__ void mt_exact_tab(MtStream& s, uint32_t* tab, uint32_t* out, uint32_t n, uint32_t deg,
                             uint32_t thr, bool lemire, int lane) {
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t count = 0;
  while (count < n) {
    if (s.q0 >= s.fnw) {  // past the generated stream: sticky, the caller reports it
      s.q0 = s.fnw + 1;
      break;
    }
    const uint32_t remaining = n - count;
    uint32_t val = 0;
    bool ok = mt_apply(s.word(s.q0 + lane), deg, thr, lemire, val);
    if (ok) ok = tab[val] != kMtTaken;
    if (ok) tab[val] = 0xFFFFFFFFu;
    if (ok) atomicMin(&tab[val], (uint32_t)lane);
    const bool isnew = ok && tab[val] == (uint32_t)lane;
    const uint64_t newmask = __ballot(isnew);
    uint64_t take = newmask;
    if ((uint32_t)__popcll(newmask) >= remaining) {
      uint64_t m = newmask;
      for (uint32_t t = 1; t < remaining; ++t) m &= m - 1;
      const int last = __ffsll((long long)m) - 1;
      take = newmask & ((last == 63) ? ~0ull : ((2ull << last) - 1ull));
      s.q0 += (uint32_t)last + 1u;
    } else {
      s.q0 += (uint32_t)kWave;
    }
    if ((take >> lane) & 1ull) {
      tab[val] = kMtTaken;
      out[count + (uint32_t)__popcll(take & lt_mask)] = val;
    }
    count += (uint32_t)__popcll(take);
  }
  __syncthreads();  // out (LDS or global) written before it is read back
  for (uint32_t k = lane; k < n; k += kWave) tab[out[k]] = 0u;
  __syncthreads();
}

// Exact path for deg > kMtTab and n > kSetCap: the kept positions in `tab`
// used as an open-addressing set (select_distinct_hashed's), n <= kMtTab / 2.
__device__ void mt_exact_hashed(MtStream& s, uint32_t* tab, uint32_t* out, uint32_t n,
                                uint32_t deg, uint32_t thr, bool lemire, int lane) {
  const uint32_t mask = kMtTab - 1;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (uint32_t k = lane; k < kMtTab; k += kWave) tab[k] = 0u;
  __syncthreads();
  uint32_t count = 0;
  while (count < n) {
    if (s.q0 >= s.fnw) {  // past the generated stream: sticky, the caller reports it
      s.q0 = s.fnw + 1;
      break;
    }
    const uint32_t remaining = n - count;
    uint32_t val = 0;
    const bool ok = mt_apply(s.word(s.q0 + lane), deg, thr, lemire, val);
    bool dup = ok && hset_has(tab, mask, val);
    const uint64_t okmask = __ballot(ok);
    for (int j = 0; j < kWave; ++j) {
      const uint32_t vj = (uint32_t)__builtin_amdgcn_readlane((int)val, j);
      dup |= (j < lane) && ((okmask >> j) & 1ull) && (vj == val);
    }
    const uint64_t newmask = __ballot(ok && !dup);
    uint64_t take = newmask;
    if ((uint32_t)__popcll(newmask) >= remaining) {
      uint64_t m = newmask;
      for (uint32_t t = 1; t < remaining; ++t) m &= m - 1;
      const int last = __ffsll((long long)m) - 1;
      take = newmask & ((last == 63) ? ~0ull : ((2ull << last) - 1ull));
      s.q0 += (uint32_t)last + 1u;
    } else {
      s.q0 += (uint32_t)kWave;
    }
    if ((take >> lane) & 1ull) {
      hset_put(tab, mask, val);
      out[count + (uint32_t)__popcll(take & lt_mask)] = val;
    }
    count += (uint32_t)__popcll(take);
    __syncthreads();
  }
  for (uint32_t k = lane; k < kMtTab; k += kWave) tab[k] = 0u;
  __syncthreads();
}

constexpr uint32_t kMtInfo = 2048;  // per-dst info staged in LDS
constexpr uint32_t kMtPos = 8192;   // kept positions staged in LDS before the flush
// chunked resolver (fanout <= 32): dsts per chunk, at most kMtChunk — a
// layer of up to kMtSmallV dsts is cut into kMtChunkSmall-dst chunks, one of
// up to kMtMaxChunks x kMtChunkMid into kMtChunkMid-dst chunks: a window
// table's lanes walk fewer dsts each and more chunks fill the CUs (C2 with
// --rng mt, scripts/ab/r04_n.sh: 4.60 ms/step at 64 / 256, 4.50 at 32 / 128,
// 4.80 at 64 / 64 — the resolver's chain over the chunks grows; 5.29 with
// 256 everywhere; round 5, with the tables at 8 / 6 waves per SIMD,
// scripts/ab/r05_aj.sh: mid 96 / 128 / 192 -> 3.63 / 3.59-3.61 / 3.57,
// small 24 / 32 / 48 -> 3.56-3.58 / 3.59-3.61 / 3.60); words staged per chunk
#ifndef NTS_MT_CHUNK_MID  // (A/B builds)
#define NTS_MT_CHUNK_MID 192
#endif
#ifndef NTS_MT_CHUNK_SMALL
#define NTS_MT_CHUNK_SMALL 32
#endif
constexpr uint32_t kMtChunk = 256;
constexpr uint32_t kMtChunkMid = NTS_MT_CHUNK_MID;
constexpr uint32_t kMtChunkSmall = NTS_MT_CHUNK_SMALL;
constexpr uint32_t kMtSmallV = 32768;
constexpr uint32_t kMtStage = 12288;

// The hot loop issues no vector-memory instruction: on gfx9 one vmcnt counter
// covers loads and stores, so a loop-carried global load (the next dsts'
// info) would wait for every position store of the iteration before it.
// Per-dst info arrives in 2048-dst chunks and kept positions leave in
// ~7 K-word flushes, both through LDS.
// FLAT (the chunked resolver's replay, one block per chunk of kMtChunk dsts):
// the chunk's exact entry word is known (k_mtp_resolve), its words come from
// the bulk-generated stream (staged in LDS when they fit), and no generator
// state is kept.
struct MtChunked {
  const uint32_t* ring;     // the stream ring (nts_hip_ctx::mt_ring)
  const uint64_t* a0p;      // FLAT: the layer's first stream word (k_mt_prep copied it)
  uint64_t gen_hi;          // stream words generated for the layer (absolute)
  const uint32_t* base;     // FLAT: [v + 1] exclusive scan of the draws n
  const uint32_t* entries;  // FLAT: [chunks + 1] extra words consumed before each chunk
  uint64_t* done;           // !FLAT: mt_done (the layer starts at its position, ends there)
  uint32_t seq;             // !FLAT: the layer's sequence number
  uint32_t* ovf;            // !FLAT: sizes[3] (bit 2: the generated stream fell short)
  uint32_t csz = kMtChunk;  // FLAT: dsts per chunk (<= kMtChunk)
};

template <int G, bool FLAT>
__global__ __launch_bounds__(kWave) void k_mt_serial(const uint4* __restrict__ info,
                                                     const uint32_t* sizes,
                                                     uint32_t* __restrict__ ans,
                                                     uint32_t* mt_state, int lemire_i, int dbg,
                                                     MtChunked ch) {
  constexpr int K = kWave / G;
  uint64_t st_it = 0, st_ex = 0, st_cyc_ex = 0, st_commit = 0;
  const uint64_t st_t0 = __builtin_readcyclecounter();
  constexpr uint32_t TAB = kMtTab / K;
  constexpr uint64_t GM = (G == 64) ? ~0ull : ((1ull << (G & 63)) - 1ull);
  constexpr uint32_t NINF = FLAT ? kMtChunk : kMtInfo;
  __shared__ uint32_t wl[FLAT ? kMtStage : 1];  // FLAT: the chunk's words staged
  __shared__ uint32_t tab[kMtTab];
  __shared__ uint32_t set[kSetCap];
  __shared__ uint4 inf[NINF];
  __shared__ uint32_t pbuf[kMtPos];
  const int lane = threadIdx.x;
  const int grp = lane / G, gl = lane % G;
  const bool lemire = lemire_i != 0;
  uint32_t vv = sizes[0], i0 = 0;
  MtStream s{nullptr, 0u};
  uint64_t a0 = 0;
  if constexpr (FLAT) {
    i0 = blockIdx.x * ch.csz;
    if (i0 >= vv) return;
    vv = min(vv, i0 + ch.csz);
    a0 = *ch.a0p;
    const MtWords W{ch.ring, a0, (uint32_t)(ch.gen_hi - a0)};
    const uint32_t e0 = ch.base[i0] + ch.entries[blockIdx.x];
    const uint32_t nw = ch.base[vv] + ch.entries[blockIdx.x + 1] - e0;
    if (nw <= kMtStage) {
      for (uint32_t k = lane; k < nw; k += kWave) wl[k] = W[e0 + k];
      s.tw = wl;
      // the chunk consumes exactly its nw words when the layer's stream is
      // whole; when it fell short the walks stop there (past wl a walk read
      // LDS garbage and, through the flat pointer, left the LDS aperture)
      s.fnw = nw;
    } else {  // (rare) read the chunk's words in place
      s.tw = ch.ring;
      s.fa = a0 + e0;
      s.fmask = kMtRingMask;
      s.fnw = W.nw > e0 ? W.nw - e0 : 0u;
    }
  } else {  // the whole layer, from the stream position after the last MT layer
    a0 = *ch.done & kMtPosMask;
    s.tw = ch.ring;
    s.fa = a0;
    s.fmask = kMtRingMask;
    s.fnw = (uint32_t)(ch.gen_hi - a0);
  }
  for (uint32_t k = lane; k < kMtTab; k += kWave) tab[k] = 0u;  // no stale kMtTaken marks
  const uint32_t v = vv;
  const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
  uint32_t ibase = i0;  // inf[k] = info[ibase + k]
  for (uint32_t k = lane; k < NINF && i0 + k < v; k += kWave) inf[k] = info[i0 + k];
  __syncthreads();
  uint32_t cbase = inf[0].x, chi = cbase;  // pbuf[k] -> ans[cbase + k]; chi: end of the kept range
  __syncthreads();
  uint32_t i = i0;
  while (i < v) {
    if (i + K > ibase + NINF) {  // next info chunk
      __syncthreads();
      ibase = i;
      for (uint32_t k = lane; k < NINF && ibase + k < v; k += kWave) inf[k] = info[ibase + k];
      __syncthreads();
    }
    const uint32_t ci = inf[i - ibase].x;
    if (ci - cbase + kSetCap + kWave > kMtPos) {  // flush kept positions
      __syncthreads();
      for (uint32_t k = lane; k < chi - cbase; k += kWave) ans[cbase + k] = pbuf[k];
      cbase = ci;
      __syncthreads();
    }
    // the K dsts i .. i+K-1, speculative start of each
    uint4 mine = (i + grp < v) ? inf[i - ibase + grp] : zero;
    uint32_t n_k[K];
    uint32_t my_sp = s.q0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      n_k[k] = __builtin_amdgcn_readlane(mine.y, k * G);
      if (k < grp) my_sp += n_k[k];
    }
    const uint32_t deg = mine.z;
    const bool active = mine.y > 0;
    uint32_t val = 0;
    bool ok = false;
    if (active) ok = mt_apply(s.word(my_sp + gl), deg, mine.w, lemire, val);
    const uint32_t slot_idx = (uint32_t)grp * TAB + (deg <= TAB ? val : (val & (TAB - 1)));
    if (ok) tab[slot_idx] = 0xFFFFFFFFu;
    if (ok) atomicMin(&tab[slot_idx], (uint32_t)gl);
    const uint32_t w = ok ? tab[slot_idx] : (uint32_t)gl;
    bool dup = w != (uint32_t)gl;
    uint64_t collm = 0;
    if (__ballot(dup && deg > TAB)) {  // hashed: the earlier lane may hold another position
      const uint32_t wv = __shfl(val, grp * G + (int)(w & (G - 1)), kWave);
      const bool coll = dup && deg > TAB && wv != val;
      collm = __ballot(coll);
    }
    // rank of each new lane among its group's new lanes; the lane of rank
    // n-1 ends the dst's draws (its word is the last one consumed)
    const uint64_t newm = __ballot(ok && !dup);
    const uint64_t gnew = (newm >> (grp * G)) & GM;
    const uint32_t rank = (uint32_t)__popcll(gnew & ((1ull << gl) - 1ull));
    const bool isnew = ok && !dup;
    const uint64_t lastm = __ballot(isnew && rank + 1 == mine.y);
    // per group, at its first lane: committable (its n-th new draw inside the
    // window, no hash collision; or nothing to draw) and clean (consumed
    // exactly n words, so the next group's speculative start was right)
    const uint64_t gl_last = (lastm >> (grp * G)) & GM;
    const bool can = mine.y == 0 || (gl_last != 0 && ((collm >> (grp * G)) & GM) == 0);
    const uint32_t cons = gl_last ? (uint32_t)__ffsll((long long)gl_last) : 0u;  // last + 1
    const bool clean = can && (mine.y == 0 || cons == mine.y);
    const bool inb = i + grp < v;
    constexpr uint64_t LEAD = (G == 16) ? 0x0001000100010001ull
                                        : ((G == 32) ? 0x0000000100000001ull : 1ull);
    const uint64_t canm = __ballot(gl == 0 && inb && can) & LEAD;
    const uint64_t dirtym = ~__ballot(gl == 0 && inb && clean) & LEAD;
    // first group that is not clean (or past v): groups before it commit,
    // and it commits too when committable
    const int f = dirtym ? (__ffsll((long long)dirtym) - 1) / G : K;
    const uint32_t commit = (uint32_t)f + ((f < K && ((canm >> (f * G)) & 1ull)) ? 1u : 0u);
    // words consumed: the speculative start of the last committed group
    // (relative) + its own consumption
    uint32_t adv = 0;
    if (commit) {
      const int lc = (int)commit - 1;
      adv = __builtin_amdgcn_readlane(my_sp, lc * G) - s.q0 +
            __builtin_amdgcn_readlane(mine.y == 0 ? 0u : cons, lc * G);
    }
    if (isnew && rank < mine.y && (uint32_t)grp < commit) pbuf[mine.x - cbase + rank] = val;
    // column offsets ascend with the dst, so the last committed dst ends the
    // kept range (copy-path ranges inside it are rewritten by k_mt_rows)
    if (commit) chi = __builtin_amdgcn_readlane(mine.x + mine.y, (commit - 1) * G);
    s.q0 += adv;
    i += commit;
    ++st_it;
    st_commit += commit;
    if (commit == 0) {  // dst i: exact path
      const uint64_t te = __builtin_readcyclecounter();
      ++st_ex;
      const uint4 fi = inf[i - ibase];
      if (fi.y <= kSetCap) {
        if (fi.z <= kMtTab)
          mt_exact_tab(s, tab, pbuf + (fi.x - cbase), fi.y, fi.z, fi.w, lemire, lane);
        else
          mt_exact(s, set, pbuf + (fi.x - cbase), 0, fi.y, fi.z, fi.w, lemire, lane);
        chi = fi.x + fi.y;
      } else {  // fanout > kSetCap: flush, then straight to the global positions
        __syncthreads();
        for (uint32_t k = lane; k < chi - cbase && chi > cbase; k += kWave) ans[cbase + k] = pbuf[k];
        if (fi.z <= kMtTab)
          mt_exact_tab(s, tab, ans + fi.x, fi.y, fi.z, fi.w, lemire, lane);
        else
          mt_exact_hashed(s, tab, ans + fi.x, fi.y, fi.z, fi.w, lemire, lane);
        cbase = chi = fi.x + fi.y;
      }
      ++i;
      st_cyc_ex += __builtin_readcyclecounter() - te;
    }
  }
  if (dbg && lane == 0 && (!FLAT || blockIdx.x == 0))
    printf("[mt G=%d%s] v=%u it=%llu commit=%llu exact=%llu cyc=%llu cyc_exact=%llu\n", G,
           FLAT ? " chunk0" : "", v - i0,
           (unsigned long long)st_it, (unsigned long long)st_commit, (unsigned long long)st_ex,
           (unsigned long long)(__builtin_readcyclecounter() - st_t0),
           (unsigned long long)st_cyc_ex);
  __syncthreads();
  for (uint32_t k = lane; k < chi - cbase && chi > cbase; k += kWave) ans[cbase + k] = pbuf[k];
  if constexpr (!FLAT) {
    // the stream position after the layer, and the generator state as
    // std::mt19937 holds it there
    const uint32_t used = s.q0;
    if (used > s.fnw) {  // the generated stream fell short: the host reports it
      if (lane == 0) atomicOr(ch.ovf, 4u);
      return;
    }
    if (lane == 0) *ch.done = ((a0 + used) & kMtPosMask) | ((uint64_t)ch.seq << 40);
    if (used > 0) mt_state_at(ch.ring, a0 + used, mt_state, lane);
  }
}

// ---- chunked MT19937 resolver (fanout <= 32) -----------------------------
// The single wave above walks the whole layer.  Here the layer's words are
// generated in bulk first (the stream does not depend on the data), the dsts
// are cut into chunks of kMtChunk, and for every chunk and every plausible
// number of extra words consumed before it (a window of +-4 sigma around the
// expected count) one lane walks the chunk and records the count after it —
// a table per chunk.  One wave then chains the tables (Delta_{k+1} =
// T_k[Delta_k]; a Delta outside the window is walked out serially), and each
// chunk is replayed from its exact entry word by k_mt_serial<FLAT>.  Every
// position is the one the sequential generator yields.
constexpr uint32_t kMtWmax = 2048;  // window entries per chunk
constexpr uint32_t kMtChunkedMinV = 4096;  // dst capacity from which a layer is chunked

// words consumed by one dst whose draws start at word p (lane-private):
// n when its first n words are accepted and pairwise distinct, else the
// sequential count; `lst` holds up to NMAX distinct positions of this lane.
template <int NMAX>
__device__ __forceinline__ uint32_t lane_consume(const MtWords& W, uint32_t p, uint32_t n, uint32_t deg,
                                                 uint32_t thr, bool lemire, uint32_t* lst,
                                                 uint32_t lstride) {
  uint32_t val[NMAX];
  bool clean = true;
#pragma unroll
  for (int t = 0; t < NMAX; ++t) {
    if ((uint32_t)t < n) {
      const uint32_t q = p + t;
      clean &= mt_apply(W[q], deg, thr, lemire, val[t]);
    }
  }
#pragma unroll
  for (int a = 1; a < NMAX; ++a)
#pragma unroll
    for (int b = 0; b < a; ++b)
      if ((uint32_t)a < n) clean &= val[a] != val[b];
  if (clean) return n;
  // the sequential walk, its words fetched 16 at a time (one memory latency
  // per 16 words, not per word: a dst whose degree is close to n needs many)
  uint32_t cnt = 0, q = p, end = p;
  while (cnt < n) {
    // past the words generated for the layer (a short stream, which the
    // layer reports): stop — past nw every word reads 0, and a walk there
    // would run to the 2^20 guard for every dst behind it
    if (q >= W.nw) break;
    uint32_t buf[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) buf[j] = W[q + j];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      uint32_t x;
      if (cnt < n && mt_apply(buf[j], deg, thr, lemire, x)) {
        bool dup = false;
        for (uint32_t k = 0; k < cnt; ++k) dup |= lst[k * lstride] == x;
        if (!dup) {
          lst[(cnt++) * lstride] = x;
          end = q + j + 1;
        }
      }
    }
    q += 16;
    if (q - p > 1u << 20) break;  // (unreachable for deg > n) keep every lane finite
  }
  // (a walk cut short ends at or past nw, so the layer's end does too)
  return (cnt >= n ? end : max(q, p + n)) - p;
}

// words consumed by one dst whose draws start at the first of the NW words in
// `cur` (lane-private, registers only): the index after the n-th distinct
// accepted draw, or 0 when it lies past the NW words (then lane_consume walks
// the stream).  A draw is new iff it is accepted and no earlier accepted draw
// has its value — the reference's rejection loop (ntsFastSampler.hpp:1026-1038).
template <int NW>
__device__ __forceinline__ uint32_t regs_consume(const uint32_t (&cur)[NW], uint32_t n,
                                                 uint32_t deg, uint32_t thr, bool lemire) {
  constexpr uint32_t kRej = 0xFFFFFFFFu;  // a rejected word (positions are < deg)
  uint32_t val[NW];
  uint32_t cnt = 0, used = 0;
#pragma unroll
  for (int t = 0; t < NW; ++t) {
    // n is the same for every lane (one dst per wave step): past the first n
    // words, stop as soon as every lane has its n-th distinct draw
    if ((uint32_t)t >= n && __ballot(used == 0) == 0) break;
    uint32_t x;
    val[t] = mt_apply(cur[t], deg, thr, lemire, x) ? x : kRej;
    bool dup = val[t] == kRej;
#pragma unroll
    for (int b = 0; b < t; ++b) dup |= val[b] == val[t];
    cnt += dup ? 0u : 1u;
    used = (used == 0 && cnt == n) ? (uint32_t)t + 1u : used;
  }
  return used;
}

// regs_consume on words already applied (the accepted position, or
// 0xFFFFFFFF for a rejected word) in an LDS window: word t at u[t].  (Each
// union word's distance back to its previous equal, computed once per wave
// and read by the lanes instead of their pairwise compares, measured slower:
// 6.0 vs 2.3 ms for the C2 bottom layer's tables — a chain of LDS reads per
// word.)
template <int NW>
__device__ __forceinline__ uint32_t window_consume(const uint32_t* u, uint32_t n) {
  constexpr uint32_t kRej = 0xFFFFFFFFu;
  uint32_t val[NW];
  uint32_t cnt = 0, used = 0;
#pragma unroll
  for (int t = 0; t < NW; ++t) {
    if ((uint32_t)t >= n && __ballot(used == 0) == 0) break;
    val[t] = u[t];
    bool dup = val[t] == kRej;
#pragma unroll
    for (int b = 0; b < t; ++b) dup |= val[b] == val[t];
    cnt += dup ? 0u : 1u;
    used = (used == 0 && cnt == n) ? (uint32_t)t + 1u : used;
  }
  return used;
}

// The stream ring's generator: nblk more 624-word blocks of the stream after
// the raw block in `raw` (block blk0 - 1), tempered into the ring at words
// 624 blk0 ...; `raw` is left holding the last one.  One workgroup (a twist is
// three dependent pieces of 227 / 227 / 170 words); it runs on the ring's side
// stream, ahead of the layers that read the words (mt_ring_prepare).  (A
// one-wave form with the block in registers and the twist operands moved by
// lane rotations measured slower: 1.92 vs 1.47 ms per C2 bottom layer.)
constexpr int kGenThreads = 256;
__global__ __launch_bounds__(kGenThreads) void k_mt_ring_gen(uint32_t* __restrict__ raw,
                                                            uint32_t* __restrict__ ring,
                                                            uint64_t blk0, uint32_t nblk) {
  __shared__ uint32_t blk[2][624];
  const int t = threadIdx.x;
  for (int k = t; k < 624; k += kGenThreads) blk[0][k] = raw[k];
  __syncthreads();
  const uint32_t U = 0x80000000u, L = 0x7fffffffu, A = 0x9908b0dfu;
  for (uint32_t b = 0; b < nblk; ++b) {
    const uint32_t* cur = blk[b & 1];
    uint32_t* nxt = blk[(b + 1) & 1];
    // _M_gen_rand in three dependent pieces: [0,227) from the current block,
    // [227,454) and [454,624) from the words just made
    if (t < 227) {
      const uint32_t y = (cur[t] & U) | (cur[t + 1] & L);
      nxt[t] = cur[t + 397] ^ (y >> 1) ^ ((y & 1u) ? A : 0u);
    }
    __syncthreads();
    if (t < 227) {
      const int k = t + 227;
      const uint32_t y = (cur[k] & U) | (cur[k + 1] & L);
      nxt[k] = nxt[k - 227] ^ (y >> 1) ^ ((y & 1u) ? A : 0u);
    }
    __syncthreads();
    if (t < 170) {
      const int k = t + 454;
      const uint32_t y = (cur[k] & U) | ((k < 623 ? cur[k + 1] : nxt[0]) & L);
      nxt[k] = nxt[k - 227] ^ (y >> 1) ^ ((y & 1u) ? A : 0u);
    }
    __syncthreads();
    const uint64_t w0 = (blk0 + b) * 624;
    for (int k = t; k < 624; k += kGenThreads)
      ring[(uint32_t)(w0 + k) & kMtRingMask] = mt_temper(nxt[k]);
  }
  __syncthreads();
  for (int k = t; k < 624; k += kGenThreads) raw[k] = blk[nblk & 1][k];
}

// the window tables: block (x, k) = entries lo_k + 256 x + t of chunk k
template <int NMAX>
__global__ __launch_bounds__(256) void k_mtp_tables(const uint4* __restrict__ info,
                                                   const uint32_t* __restrict__ base,
                                                   const uint32_t* sizes, const float2* cstat,
                                                   const uint32_t* __restrict__ ring,
                                                   const uint64_t* a0p, uint64_t gen_hi,
                                                   int lemire_i, uint32_t csz,
                                                   uint2* __restrict__ win,
                                                   uint32_t* __restrict__ tabs) {
  __shared__ uint4 inf[kMtChunk];
  __shared__ uint32_t bs[kMtChunk];
#ifdef NTS_MT_LDS_LST  // (A/B build: the fallback walk's list in LDS, NMAX words a lane)
  __shared__ uint32_t lst[NMAX * 256];
#endif
  __shared__ float red[2][4];
  __shared__ uint32_t uu[4][2][192];  // per wave: the union windows of two dsts
  const int t = threadIdx.x;
  const uint32_t k = blockIdx.y, v = sizes[0];
  const uint32_t i0 = k * csz;
  if (i0 >= v) return;
  const uint32_t i1 = min(v, i0 + csz);
  float m = 0.f, var = 0.f;
  for (uint32_t j = t; j < k; j += 256) {
    m += cstat[j].x;
    var += cstat[j].y;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    m += __shfl_down(m, o, kWave);
    var += __shfl_down(var, o, kWave);
  }
  if ((t & 63) == 0) {
    red[0][t >> 6] = m;
    red[1][t >> 6] = var;
  }
  for (uint32_t j = t; j < i1 - i0; j += 256) {
    inf[j] = info[i0 + j];
    bs[j] = base[i0 + j];
  }
  __syncthreads();
  const float mm = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  const float vv = red[1][0] + red[1][1] + red[1][2] + red[1][3];
// the window's half-width in sigmas (compile-time A/B; a Delta outside its
// window, ~0.3 % of the chunks at 3, is walked out by the resolver): C2 --rng
// mt 3.57-3.59 / 3.57-3.58 / 3.52-3.55 ms/step at 4 / 3.5 / 3 (r05_ax.sh)
#ifndef NTS_MT_SIGMA
#define NTS_MT_SIGMA 3.f
#endif
  const float h = ceilf(NTS_MT_SIGMA * sqrtf(vv)) + 8.f;
  const uint32_t lo = (uint32_t)fmaxf(0.f, floorf(mm - h));
  const uint32_t wn = min(kMtWmax, (uint32_t)(mm + h - (float)lo) + 1u);
  if (blockIdx.x == 0 && t == 0) win[k] = make_uint2(lo, wn);
  // waves whose entries all lie past the window leave (no block barrier
  // below): the last block of a window is ~half idle otherwise (3.60-3.62 ->
  // 3.57-3.59 ms/step, r05_ax.sh)
#ifdef NTS_MT_BLOCK_EXIT  // (A/B build: whole blocks only)
  if (blockIdx.x * 256u >= wn) return;
#else
  if (blockIdx.x * 256u + (uint32_t)(t & ~63) >= wn) return;
#endif
  const uint32_t slot = blockIdx.x * 256u + t;
  const uint64_t a0 = *a0p;
  const MtWords W{ring, a0, (uint32_t)(gen_hi - a0)};
  const bool lemire = lemire_i != 0;
  uint32_t dl = lo + slot;
  // The wave's lanes walk the dst with nearby starts (consecutive Deltas,
  // drifting apart by their extra words): the union of their words, kU from
  // the smallest start, is fetched once per wave (three words a lane) and
  // accepted / mapped to positions once, into LDS; each lane reads its window
  // from there.  The next drawing dst's union is fetched while this one is
  // checked, based at this step's smallest Delta (Deltas only grow).  A wave
  // whose starts spread wider than the union reads its own words.
#ifndef NTS_MT_NWX
#define NTS_MT_NWX 8  // words past the n-th in a lane's window (A/B, r04_o: 4 / 6 / 8 / 12 -> 4.20 / 3.95 / 3.91 / 3.89 ms)
#endif
  constexpr int NW = NMAX + NTS_MT_NWX;
  constexpr int kU = 192;
  const int wvi = t >> 6, ln = t & 63;
  // wave minimum / maximum (every lane active here): DPP moves within each
  // 16-lane row, then the four rows' values by v_readlane — a few VALU
  // cycles instead of six dependent ds_bpermute round trips per call (two
  // calls per dst step)
  auto row16 = [](uint32_t x, auto op) {
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false));
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false));
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false));
    x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false));
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 0);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)x, 16);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)x, 32);
    const uint32_t r3 = (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
    return op(op(r0, r1), op(r2, r3));
  };
  auto wmin = [&](uint32_t x) { return row16(x, [](uint32_t p, uint32_t q) { return min(p, q); }); };
  auto wmax = [&](uint32_t x) { return row16(x, [](uint32_t p, uint32_t q) { return max(p, q); }); };
  uint32_t rw[kU / kWave];
  auto load_union = [&](uint32_t P) {
#pragma unroll
    for (int q = 0; q < kU / kWave; ++q) rw[q] = W[P + ln + kWave * q];
  };
  auto store_union = [&](int buf, const uint4& f) {
#pragma unroll
    for (int q = 0; q < kU / kWave; ++q) {
      uint32_t x;
      uu[wvi][buf][ln + kWave * q] = mt_apply(rw[q], f.z, f.w, lemire, x) ? x : 0xFFFFFFFFu;
    }
  };
  const uint32_t cnt = i1 - i0;
  auto next_draw = [&](uint32_t j) {
    while (j < cnt && inf[j].y == 0) ++j;
    return j;
  };
  uint32_t j = next_draw(0);
  int buf = 0;
  uint32_t P0 = j < cnt ? bs[j] + wmin(dl) : 0u;
  if (j < cnt) {
    load_union(P0);
    store_union(0, inf[j]);
  }
  while (j < cnt) {
    const uint4 f = inf[j];
    const uint32_t p = bs[j] + dl;
    const uint32_t jn = next_draw(j + 1);
    const uint32_t P0n = jn < cnt ? bs[jn] + wmin(dl) : 0u;
    if (jn < cnt) load_union(P0n);
    uint32_t used;
    if (wmax(p) + NW - P0 <= (uint32_t)kU) {  // (p >= P0: Deltas only grow)
      used = window_consume<NW>(&uu[wvi][buf][p - P0], f.y);
    } else {
      uint32_t cur[NW];
#pragma unroll
      for (int q = 0; q < NW; ++q) cur[q] = W[p + q];
      used = regs_consume<NW>(cur, f.y, f.z, f.w, lemire);
    }
    if (used == 0) {
#ifdef NTS_MT_LDS_LST
      used = lane_consume<NMAX>(W, p, f.y, f.z, f.w, lemire, lst + t, 256);
#else
      // the rare sequential walk keeps its list in private memory (scratch):
      // in LDS it cost NMAX KiB a block and capped the kernel at 7 (NMAX 10)
      // or 4 (NMAX 25) waves per SIMD
      uint32_t plst[NMAX];
      asm volatile("" ::"v"(plst) : "memory");  // (its address escapes: scratch, not registers)
      used = lane_consume<NMAX>(W, p, f.y, f.z, f.w, lemire, plst, 1);
#endif
    }
    dl += used - f.y;
    if (jn < cnt) store_union(buf ^ 1, inf[jn]);
    P0 = P0n;
    buf ^= 1;
    j = jn;
  }
  if (slot < wn) tabs[(uint64_t)k * kMtWmax + slot] = dl;
}

// chain the tables: entries[k] = extra words before chunk k (one wave).  The
// windows of the next kRing chunks are fetched ahead into LDS by LDS DMA
// (16 B per lane per instruction; no other vector-memory op in the loop, so
// the hand-counted vmcnt below is exact).  A Delta outside its chunk's window
// is walked out by lane 0.  Also leaves the generator state after the layer.
constexpr int kRing = 5;
constexpr uint32_t kMtMaxChunks = 4096;  // the host keeps v_cap <= kMtMaxChunks * csz
constexpr int kRingOps = kMtWmax * 4 / (16 * kWave);  // LDS-DMA instructions per window

__device__ __forceinline__ void glds16(const void* src, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}

template <int NMAX>
__global__ __launch_bounds__(kWave) void k_mtp_resolve(const uint4* __restrict__ info,
                                                      const uint32_t* __restrict__ base,
                                                      const uint32_t* sizes,
                                                      const uint32_t* __restrict__ sring,
                                                      const uint64_t* a0p, uint64_t gen_hi,
                                                      int lemire_i, uint32_t csz,
                                                      const uint2* __restrict__ win,
                                                      const uint32_t* __restrict__ tabs,
                                                      uint32_t* __restrict__ entries,
                                                      uint64_t* __restrict__ done, uint32_t seq,
                                                      uint32_t* __restrict__ mt_state,
                                                      uint32_t* __restrict__ ovf,
                                                      uint32_t* __restrict__ nfallback) {
  __shared__ __attribute__((aligned(16))) uint32_t ring[kRing][kMtWmax];
  __shared__ uint32_t ent[kMtMaxChunks];
  __shared__ uint2 wins[kMtMaxChunks];
  __shared__ uint32_t lst[NMAX];
  const int lane = threadIdx.x;
  const uint32_t v = sizes[0];
  const uint32_t nch = min((v + csz - 1) / csz, kMtMaxChunks);
  for (uint32_t k = lane; k < nch; k += kWave) wins[k] = win[k];  // before any LDS DMA
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const bool lemire = lemire_i != 0;
  const uint64_t a0 = *a0p;
  const MtWords W{sring, a0, (uint32_t)(gen_hi - a0)};
  const uint32_t nw = W.nw;
  auto fetch = [&](uint32_t k) {  // window of chunk min(k, nch - 1) -> ring slot k % kRing
    const uint32_t kk = nch ? min(k, nch - 1) : 0u;
    const char* src = reinterpret_cast<const char*>(tabs + (uint64_t)kk * kMtWmax);
    const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)ring[k % kRing];
#pragma unroll
    for (int q = 0; q < kRingOps; ++q) glds16(src + 1024 * q + 16 * lane, dst + 1024 * q);
  };
  for (uint32_t k = 0; k < (uint32_t)kRing; ++k) fetch(k);
  uint32_t dl = 0, fallbacks = 0;
  for (uint32_t k = 0; k < nch; ++k) {
    ent[k] = dl;  // (lane-uniform store)
    // the window of chunk k landed: (kRing - 1) windows issued after it
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kRing - 1) * kRingOps) : "memory");
    const uint2 w = wins[k];
    if (dl >= w.x && dl < w.x + w.y) {
      dl = ring[k % kRing][dl - w.x];
    } else {  // outside the window: walk the chunk
      ++fallbacks;
      uint32_t d2 = dl;
      if (lane == 0) {
        const uint32_t i0 = k * csz, i1 = min(v, i0 + csz);
        for (uint32_t j = i0; j < i1; ++j) {
          const uint4 f = info[j];
          if (f.y == 0) continue;
          d2 += lane_consume<NMAX>(W, base[j] + d2, f.y, f.z, f.w, lemire, lst, 1) - f.y;
        }
      }
      dl = __builtin_amdgcn_readfirstlane(d2);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();  // the slot is read before it is refilled
    fetch(k + kRing);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (uint32_t k = lane; k < nch; k += kWave) entries[k] = ent[k];
  if (lane == 0) {
    entries[nch] = dl;
    if (dl + base[v] > nw) *ovf |= 4u;  // the stream generated fell short
    *nfallback = fallbacks;
  }
  // the stream position after the layer, and the generator state there
  // (only when the words consumed are inside the generated stream: the host
  // reports a short stream)
  const uint32_t used = base[v] + dl;
  if (used > nw) return;
  if (lane == 0) *done = ((a0 + used) & kMtPosMask) | ((uint64_t)seq << 40);
  if (used > 0) mt_state_at(sring, a0 + used, mt_state, lane);
}

// positions -> neighbour ids (16-lane group per dst); copy-path dsts take
// every neighbour in CSC order (core/ntsFastSampler.hpp:1040-1048)
__global__ __launch_bounds__(kSelThreads) void k_mt_rows(SelectArgs a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int gl = lane & (kGrp - 1), grp = lane >> 4;
  const uint32_t v = a.sizes[0];
  const uint32_t ng = gridDim.x * kSelWaves * kGrpPerWave;
  for (uint32_t i = blockIdx.x * kSelWaves * kGrpPerWave + w * kGrpPerWave + grp; i < v; i += ng) {
    const uint32_t d = a.dst[i];
    const uint64_t beg = a.goff[d];
    const uint32_t deg = (uint32_t)(a.goff[d + 1] - beg);
    const uint32_t c = a.co[i];
    const uint32_t n = a.co[i + 1] - c;
    if ((uint64_t)c + n > a.e_cap) continue;
    const bool copy = n == deg;
    for (uint32_t k = gl; k < n; k += kGrp) {
      // (positions are < deg; the clamp only keeps the reads inside the
      // graph when a short stream left stale words in ans — that layer is
      // reported short and sampled again)
      const uint32_t g = a.grows[beg + (copy ? k : min(a.ans[c + k], deg - 1))];
      a.ans[c + k] = g;
      a.edst[c + k] = i;
      a.marks[g] = 1;
    }
  }
}

// ---- frontier compaction --------------------------------------------------
constexpr int kMarkThreads = 256;
constexpr int kMarkTile = kMarkThreads * 16;  // 4096 vertices per block
constexpr uint32_t kMarkDirectTiles = 2048;     // k_mark_write sums the tile counts itself

__device__ __forceinline__ uint32_t count16(uint4 m) {
  // marks are 0/1 bytes -> popcount of each word counts set bytes
  return __popc(m.x) + __popc(m.y) + __popc(m.z) + __popc(m.w);
}

__global__ __launch_bounds__(kMarkThreads) void k_mark_count(const uint8_t* __restrict__ marks,
                                                             uint32_t* blk) {
  const uint4 m = reinterpret_cast<const uint4*>(marks)[(uint64_t)blockIdx.x * kMarkThreads +
                                                        threadIdx.x];
  uint32_t c = count16(m);
  // wave reduce + block reduce
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, kWave);
  __shared__ uint32_t ws[kMarkThreads / kWave];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int i = 0; i < kMarkThreads / kWave; ++i) s += ws[i];
    blk[blockIdx.x] = s;
  }
}

// Single-pass frontier compaction (the default): each 4096-vertex tile counts
// its marks, takes its offset by decoupled look-back over the tiles before it
// (lookback_exclusive) and writes `source` / `src_index` in ascending vertex
// order — k_mark_count + k_mark_write in one launch.  Clears the marks it
// read; the last tile writes src_size (and the s_cap overflow flag, this
// kernel's only writer of it).
__global__ __launch_bounds__(kMarkThreads) void k_mark_fused(
    uint8_t* __restrict__ marks, uint32_t nblk, uint64_t n_vertices, uint32_t s_cap,
    uint32_t* __restrict__ source, uint32_t* __restrict__ src_index, uint32_t* sizes,
    uint64_t* __restrict__ state, uint32_t epoch, uint32_t* ticket) {
  const uint32_t tile = lb_ticket(ticket, nblk);
  const uint64_t tid = (uint64_t)tile * kMarkThreads + threadIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __shared__ uint32_t ws[kMarkThreads / kWave];
  __shared__ uint32_t s_prefix;
  const uint4 m = reinterpret_cast<const uint4*>(marks)[tid];
  if (m.x | m.y | m.z | m.w) reinterpret_cast<uint4*>(marks)[tid] = make_uint4(0u, 0u, 0u, 0u);
  const uint32_t c = count16(m);
  uint32_t inc = c;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += y;
  }
  if (lane == 63) ws[w] = inc;
  __syncthreads();
  uint32_t agg = 0, off = 0;
  for (int i = 0; i < kMarkThreads / kWave; ++i) {
    off += i < w ? ws[i] : 0u;
    agg += ws[i];
  }
  if (w == 0) {
    const uint32_t pre = lookback_exclusive(state, tile, epoch, agg);
    if (lane == 0) s_prefix = pre;
  }
  __syncthreads();
  uint32_t pos = s_prefix + off + inc - c;
  if (tile == nblk - 1 && threadIdx.x == 0) {
    const uint32_t total = s_prefix + agg;
    sizes[2] = min(total, s_cap);
    if (total > s_cap) atomicOr(&sizes[3], 2u);
  }
  if (c == 0) return;
  const uint32_t words[4] = {m.x, m.y, m.z, m.w};
  const uint64_t v0 = tid * 16;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if ((words[q] >> (8 * b)) & 0xffu) {
        const uint64_t vtx = v0 + q * 4 + b;
        if (vtx < n_vertices && pos < s_cap) {
          source[pos] = (uint32_t)vtx;
          src_index[vtx] = pos;
        }
        ++pos;
      }
    }
  }
}

// Also clears the byte map it consumed, so the next layer starts from zeros
// without a memset (the map is zeroed once when allocated).
// DIRECT: blk holds the per-tile counts and each block sums the ones before
// its tile (and block 0 all of them, for src_size) — no scan kernel between
// k_mark_count and this one; otherwise blk is the scanned offsets [nblk + 1].
template <bool DIRECT>
__global__ __launch_bounds__(kMarkThreads) void k_mark_write(
    uint8_t* __restrict__ marks, const uint32_t* __restrict__ blk, uint32_t nblk,
    uint64_t n_vertices, uint32_t s_cap, uint32_t* __restrict__ source,
    uint32_t* __restrict__ src_index, uint32_t* sizes) {
  const uint64_t tid = (uint64_t)blockIdx.x * kMarkThreads + threadIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __shared__ uint32_t ws[kMarkThreads / kWave];
  __shared__ uint32_t bo[2];
  if (DIRECT) {
    // fixed-order sums: tiles before this one, and (block 0) all tiles
    uint32_t a = 0, b = 0;
    for (uint32_t i = threadIdx.x; i < nblk; i += kMarkThreads) {
      const uint32_t v = blk[i];
      a += i < blockIdx.x ? v : 0u;
      b += v;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_down(a, o, kWave);
      b += __shfl_down(b, o, kWave);
    }
    __shared__ uint32_t wa[kMarkThreads / kWave], wb[kMarkThreads / kWave];
    if (lane == 0) { wa[w] = a; wb[w] = b; }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t sa = 0, sb = 0;
      for (int i = 0; i < kMarkThreads / kWave; ++i) { sa += wa[i]; sb += wb[i]; }
      bo[0] = sa;
      bo[1] = sb;
    }
  } else if (threadIdx.x == 0) {
    bo[0] = blk[blockIdx.x];
    bo[1] = blk[nblk];
  }
  const uint4 m = reinterpret_cast<const uint4*>(marks)[tid];
  if (m.x | m.y | m.z | m.w) reinterpret_cast<uint4*>(marks)[tid] = make_uint4(0u, 0u, 0u, 0u);
  const uint32_t c = count16(m);
  uint32_t inc = c;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    uint32_t y = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += y;
  }
  if (lane == 63) ws[w] = inc;
  __syncthreads();
  uint32_t off = bo[0];
  for (int i = 0; i < w; ++i) off += ws[i];
  uint32_t pos = off + inc - c;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint32_t s = bo[1];
    sizes[2] = min(s, s_cap);
    if (s > s_cap) atomicOr(&sizes[3], 2u);
  }
  if (c == 0) return;
  const uint32_t words[4] = {m.x, m.y, m.z, m.w};
  const uint64_t v0 = tid * 16;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if ((words[q] >> (8 * b)) & 0xffu) {
        const uint64_t vtx = v0 + q * 4 + b;
        if (vtx < n_vertices && pos < s_cap) {
          source[pos] = (uint32_t)vtx;
          src_index[vtx] = pos;
        }
        ++pos;
      }
    }
  }
}

// ---- relabel + weights ------------------------------------------------------
__device__ __forceinline__ float norm_degree(uint32_t out_src, uint32_t in_dst) {
  // 1 / ((float)std::sqrt(out) * (float)std::sqrt(in)), nts_norm_degree
  // (core/ntsBaseOp.hpp:652-657): std::sqrt of an integer is the double sqrt.
  const float a = (float)sqrt((double)out_src);
  const float b = (float)sqrt((double)in_dst);
  return 1.0f / (a * b);
}

// up_cnt != nullptr (UP_DEGREE): count the sampled edges per local src
// instead of computing the weights (k_up_weight does, once counted).
// MEAN divides by the dst's full-graph in-degree (the CPU sampler,
// core/ntsFastSampler.hpp:1111-1113); MEAN_SAMPLED by its sampled edge count
// (the reference GPU kernel get_mean_weight, cuda/ntsCUDATransferKernel.cuh:319-342,
// which its GPU toolkits never reach: SURVEY Appendix B-5).
struct RelabelArgs {
  const uint32_t* ans;
  const uint32_t* edst;
  const uint32_t* dst;
  const uint32_t* src_index;
  const uint32_t* out_deg;
  const uint32_t* in_deg;
  const uint32_t* co;
  const uint32_t* sizes;
  int weight_type;
  uint32_t* ri;
  float* wf;
  uint32_t* up_cnt;
  uint32_t* pub;  // the layer's last kernel: nts_sampcsc_dev::sizes_host, else NULL
};

// the layer's sizes words into the caller's host-mapped copy, from the layer's
// last kernel (every sizes word is final by then): replaces a per-batch D2H
// copy, a blit kernel of its own on the sampler stream
__device__ __forceinline__ void publish_sizes(const uint32_t* sizes, uint32_t* pub) {
  if (pub && blockIdx.x == 0 && threadIdx.x < 4) pub[threadIdx.x] = sizes[threadIdx.x];
}

__device__ __forceinline__ uint32_t relabel_one(const RelabelArgs& a, uint32_t k) {
  const uint32_t g = a.ans[k];
  const uint32_t r = a.src_index[g];
  a.ri[k] = r;
  if (a.up_cnt) {
    atomicAdd(a.up_cnt + r, 1u);
  } else if (a.weight_type != NTS_WEIGHT_NONE) {
    const uint32_t dg = a.dst[a.edst[k]];
    const uint32_t ind = a.in_deg[dg];
    float w = norm_degree(a.out_deg[g], ind);
    if (a.weight_type == NTS_WEIGHT_MEAN) w = w / (float)ind;
    if (a.weight_type == NTS_WEIGHT_MEAN_SAMPLED) w = w / (float)(a.co[a.edst[k] + 1] - a.co[a.edst[k]]);
    a.wf[k] = w;
  }
  return r;
}

__global__ void k_relabel(RelabelArgs a) {
  publish_sizes(a.sizes, a.pub);
  const uint32_t e = a.sizes[1];
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < e; k += gridDim.x * blockDim.x)
    relabel_one(a, k);
}

// UP_DEGREE weights: out = sampled edges of the src (counted by k_relabel),
// in = sampled edges of the dst (its CSC segment)
__global__ void k_up_weight(const uint32_t* __restrict__ ri, const uint32_t* __restrict__ edst,
                            const uint32_t* __restrict__ co, const uint32_t* __restrict__ cnt,
                            const uint32_t* sizes, int weight_type, float* __restrict__ wf,
                            uint32_t* pub) {
  publish_sizes(sizes, pub);
  const uint32_t e = sizes[1];
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < e; k += gridDim.x * blockDim.x) {
    const uint32_t d = edst[k];
    const uint32_t ind = co[d + 1] - co[d];
    float w = norm_degree(cnt[ri[k]], ind);
    if (weight_type == NTS_WEIGHT_MEAN || weight_type == NTS_WEIGHT_MEAN_SAMPLED)
      w = w / (float)ind;  // the dst's sampled count is its UP_DEGREE in-degree
    wf[k] = w;
  }
}

// merged src/dst frontier (GAT): every dst is a source too
__global__ void k_mark_dst(const uint32_t* __restrict__ dst, const uint32_t* sizes,
                           uint8_t* __restrict__ marks) {
  const uint32_t v = sizes[0];
  for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < v; d += gridDim.x * blockDim.x)
    marks[dst[d]] = 1;
}
__global__ void k_dst_local(const uint32_t* __restrict__ dst, const uint32_t* __restrict__ src_index,
                            const uint32_t* sizes, uint32_t* __restrict__ dl) {
  const uint32_t v = sizes[0];
  for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < v; d += gridDim.x * blockDim.x)
    dl[d] = src_index[dst[d]];
}

// ---- CSR transpose in two halves -------------------------------------------
// First half (radix_pass_pairs): ONE stable radix pass on the high H bits of
// the local src, so each bucket of 2^L consecutive sources holds its edges
// contiguously, in edge order.  Second half, k_csr_bucket: one workgroup per
// bucket finishes the transpose in LDS — per-wave counts of the low L bits
// (the bucket's row counts: the row offsets come out of their scan), then each
// wave re-reads its quarter of the bucket in order and ranks every edge
// against a running per-(wave, row) position (match-any by ballots), so a
// row's edges land in edge order: the stable order of the reference's serial
// fill (core/coocsc.hpp:82-111), as the two-pass radix sort + k_csr_finalize
// gave.  Replaces the second radix pass (its counts, digit scans and 8-byte
// scatter) and the finalize's separate read of the sorted pairs.
constexpr int kCsrBucketThreads = 1024;  // 16 waves: short in-order chains per bucket
constexpr int kCsrBucketWaves = kCsrBucketThreads / kWave;
constexpr int kCsrBucketIt = 4;  // 64-edge groups per lane in flight

template <int L>
__global__ __launch_bounds__(kCsrBucketThreads) void k_csr_bucket(
    const uint32_t* __restrict__ skey, const uint32_t* __restrict__ seid,
    const uint32_t* __restrict__ totals, const uint32_t* __restrict__ sdst,
    const uint32_t* __restrict__ swf, const uint32_t* sizes, uint32_t* __restrict__ ro,
    uint32_t* __restrict__ ci, float* __restrict__ wb, uint32_t* __restrict__ ceid, uint32_t* pub) {
  constexpr uint32_t R = 1u << L, RPT = R > kCsrBucketThreads ? R / kCsrBucketThreads : 1;
  __shared__ uint32_t wh[kCsrBucketWaves][R];  // per-wave row counts -> running positions
  __shared__ uint32_t wsum[kCsrBucketWaves];
  publish_sizes(sizes, pub);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t b = blockIdx.x, s = sizes[2], r0 = b << L;
  if (r0 > s) return;  // (block-uniform) no row of this bucket, nor ro[s]
  // the bucket's start: the items of the buckets before it
  uint32_t part = 0;
  for (uint32_t i = t; i < b; i += kCsrBucketThreads) part += totals[i];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) part += __shfl_xor(part, o, kWave);
  if (lane == 0) wsum[w] = part;
  for (uint32_t d = t; d < R; d += kCsrBucketThreads)
#pragma unroll
    for (int ww = 0; ww < kCsrBucketWaves; ++ww) wh[ww][d] = 0;
  __syncthreads();
  uint32_t bstart = 0;
#pragma unroll
  for (int ww = 0; ww < kCsrBucketWaves; ++ww) bstart += wsum[ww];
  const uint32_t cnt = totals[b];
  const uint32_t q0 = (uint32_t)((uint64_t)cnt * w / kCsrBucketWaves);
  const uint32_t q1 = (uint32_t)((uint64_t)cnt * (w + 1) / kCsrBucketWaves);
  const uint32_t* kb = skey + bstart;
  const uint32_t* eb = seid + bstart;
  const uint32_t* db = sdst + bstart;
  const uint32_t* fb = swf ? swf + bstart : nullptr;
  // (1) wave w counts the rows of its quarter
  for (uint32_t i = q0 + lane; i < q1; i += kWave) atomicAdd(&wh[w][kb[i] & (R - 1)], 1u);
  __syncthreads();  // (also: every wave has read wsum)
  // (2) thread t owns rows t RPT .. +RPT-1: per-wave exclusive offsets, the
  // rows' counts scanned over the block -> row offsets and absolute positions
  uint32_t rc[RPT], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < RPT; ++k) {
    const uint32_t d = t * RPT + k;
    uint32_t run = 0;
    if (d < R) {
#pragma unroll
      for (int ww = 0; ww < kCsrBucketWaves; ++ww) {
        const uint32_t c = wh[ww][d];
        wh[ww][d] = run;
        run += c;
      }
    }
    rc[k] = run;
    sum += run;
  }
  uint32_t inc = sum;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += y;
  }
  __syncthreads();  // wsum reused
  if (lane == kWave - 1) wsum[w] = inc;
  __syncthreads();
  uint32_t base = bstart + inc - sum;
#pragma unroll
  for (int ww = 0; ww < kCsrBucketWaves; ++ww) base += ww < w ? wsum[ww] : 0u;
#pragma unroll
  for (uint32_t k = 0; k < RPT; ++k) {
    const uint32_t d = t * RPT + k;
    if (d < R) {
      if (r0 + d <= s) ro[r0 + d] = base;
#pragma unroll
      for (int ww = 0; ww < kCsrBucketWaves; ++ww) wh[ww][d] += base;
    }
    base += rc[k];
  }
  __syncthreads();
  // (3) each wave walks its share in order, kCsrBucketIt groups of 64 at a
  // time (the loads first, then the ranks in group order); the dst ids and
  // forward weights came through the radix pass beside the edge ids
  // (payloads gathered within each 4096-edge tile), so every read here is
  // sequential
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (uint32_t i0 = q0; i0 < q1; i0 += kCsrBucketIt * kWave) {
    uint32_t key[kCsrBucketIt], eid[kCsrBucketIt], dv[kCsrBucketIt];
    float fv[kCsrBucketIt];
#pragma unroll
    for (int g = 0; g < kCsrBucketIt; ++g) {
      const uint32_t i = i0 + g * kWave + lane;
      const bool ok = i < q1;
      key[g] = ok ? kb[i] : 0u;
      eid[g] = ok && ceid ? eb[i] : 0u;
      dv[g] = ok ? db[i] : 0u;
      fv[g] = ok && wb && fb ? __uint_as_float(fb[i]) : 0.f;
    }
#pragma unroll
    for (int g = 0; g < kCsrBucketIt; ++g) {
      const bool ok = i0 + g * kWave + lane < q1;
      const uint32_t d = key[g] & (R - 1);
      uint64_t peers = __ballot(ok);
#pragma unroll
      for (int bb = 0; bb < L; ++bb) {
        const bool bit = (d >> bb) & 1u;
        const uint64_t m = __ballot(bit);
        peers &= bit ? m : ~m;
      }
      const uint32_t prev = wh[w][d];
      const uint32_t before = (uint32_t)__popcll(peers & lt);
      if (ok && before == 0) wh[w][d] = prev + (uint32_t)__popcll(peers);
      if (ok) {
        const uint32_t pos = prev + before;
        ci[pos] = dv[g];
        if (ceid) ceid[pos] = eid[g];
        if (wb) wb[pos] = fv[g];
      }
    }
  }
}

// ---- CSR from sorted (local src, edge id) ----------------------------------
__global__ void k_csr_finalize(const uint32_t* __restrict__ skey, const uint32_t* __restrict__ seid,
                               const uint32_t* __restrict__ edst, const float* __restrict__ wf,
                               const uint32_t* sizes, uint32_t* __restrict__ ro,
                               uint32_t* __restrict__ ci, float* __restrict__ wb,
                               uint32_t* __restrict__ ceid, uint32_t* pub) {
  publish_sizes(sizes, pub);
  const uint32_t e = sizes[1];
  const uint32_t s = sizes[2];
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < e; j += gridDim.x * blockDim.x) {
    const uint32_t key = skey[j];
    const uint32_t eid = seid[j];
    ci[j] = edst[eid];
    if (ceid) ceid[j] = eid;
    if (wb) wb[j] = wf ? wf[eid] : 0.0f;
    if (j == 0 || skey[j - 1] != key) {
      // rows between the previous key and this one are empty (cannot happen for
      // a frontier built from the edges, kept for robustness)
      const uint32_t prev = (j == 0) ? 0u : skey[j - 1] + 1u;
      for (uint32_t r = prev; r <= key; ++r) ro[r] = j;
    }
    if (j == e - 1)
      for (uint32_t r = key + 1; r <= s; ++r) ro[r] = e;
  }
  if (e == 0 && blockIdx.x == 0 && threadIdx.x == 0)
    for (uint32_t r = 0; r <= s; ++r) ro[r] = 0;
}

}  // namespace nts_hip

namespace nts_hip {

// ---- the stream ring, host side ----------------------------------------------
// Words are generated in launches of up to kMtGenChunk blocks on the ring's
// own stream, each followed by an event; a layer waits on the event that
// covers its words.  Bound on the words a layer may consume: its w_cap (a
// layer past it reports a short stream, sizes[3] bit 2).  The host keeps the
// position read back after the last finished MT layer (mt_done, copied to
// pinned memory after each layer) plus the bounds of the layers issued since,
// generates up to that sum plus two layers' bounds ahead, and never more than
// the ring holds beyond the oldest word a pending layer can still read.
constexpr uint32_t kMtGenChunk = 4096;  // ~2.7 ms of generation per launch

static int mt_ring_ensure(nts_hip_ctx* ctx) {
  if (ctx->mt_ring) return NTS_OK;
  // first MT layer since the context was created: the generator starts from
  // the seeded state (no MT layer has moved it)
  NTS_HIP_TRY(hipMalloc(&ctx->mt_ring, kMtRingWords * sizeof(uint32_t)));
  NTS_HIP_TRY(hipMalloc(&ctx->mt_gen_raw, 624 * sizeof(uint32_t)));
  NTS_HIP_TRY(hipMalloc(&ctx->mt_done, sizeof(uint64_t)));
  NTS_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ctx->mt_done_host), sizeof(uint64_t),
                            hipHostMallocDefault));
  // the generator (one workgroup per launch) on a high-priority stream: its
  // launches are dispatched ahead of queued table / training blocks
  int lo_prio = 0, hi_prio = 0;
  NTS_HIP_TRY(hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio));
  NTS_HIP_TRY(hipStreamCreateWithPriority(&ctx->mt_gen_stream, hipStreamNonBlocking, hi_prio));
  return mt_ring_reset(ctx);
}

int mt_ring_reset(nts_hip_ctx* ctx) {
  if (!ctx->mt_ring) return NTS_OK;
  NTS_HIP_TRY(hipStreamSynchronize(ctx->mt_gen_stream));
  NTS_HIP_TRY(hipStreamSynchronize(ctx->stream));
  NTS_HIP_TRY(hipMemcpyAsync(ctx->mt_gen_raw, ctx->mt_state, 624 * sizeof(uint32_t),
                             hipMemcpyDeviceToDevice, ctx->stream));
  NTS_HIP_TRY(hipMemsetAsync(ctx->mt_done, 0, sizeof(uint64_t), ctx->stream));
  NTS_HIP_TRY(hipStreamSynchronize(ctx->stream));
  *ctx->mt_done_host = 0;
  ctx->mt_gen_blocks = 0;
  ctx->mt_seq = 0;
  ctx->mt_pos_done = 0;
  ctx->mt_seq_done = 0;
  ctx->mt_pending.clear();
  for (auto& e : ctx->mt_gen_evs) ctx->mt_ev_pool.push_back(e.second);
  ctx->mt_gen_evs.clear();
  return NTS_OK;
}

void mt_ring_free(nts_hip_ctx* ctx) {
  if (ctx->mt_gen_stream) (void)hipStreamSynchronize(ctx->mt_gen_stream);
  for (auto& e : ctx->mt_gen_evs) (void)hipEventDestroy(e.second);
  for (auto ev : ctx->mt_ev_pool) (void)hipEventDestroy(ev);
  ctx->mt_gen_evs.clear();
  ctx->mt_ev_pool.clear();
  if (ctx->mt_gen_stream) (void)hipStreamDestroy(ctx->mt_gen_stream);
  if (ctx->mt_ring) (void)hipFree(ctx->mt_ring);
  if (ctx->mt_gen_raw) (void)hipFree(ctx->mt_gen_raw);
  if (ctx->mt_done) (void)hipFree(ctx->mt_done);
  if (ctx->mt_done_host) (void)hipHostFree(ctx->mt_done_host);
  ctx->mt_gen_stream = nullptr;
  ctx->mt_ring = ctx->mt_gen_raw = nullptr;
  ctx->mt_done = ctx->mt_done_host = nullptr;
}

static void mt_ring_readback(nts_hip_ctx* ctx) {
  const uint64_t snap = __atomic_load_n(ctx->mt_done_host, __ATOMIC_ACQUIRE);
  const uint32_t sseq = (uint32_t)(snap >> 40);
  if (sseq == ctx->mt_seq_done) return;
  ctx->mt_seq_done = sseq;
  ctx->mt_pos_done = snap & kMtPosMask;
  auto& p = ctx->mt_pending;  // layers up to sseq are in mt_pos_done now
  p.erase(p.begin(), std::find_if(p.begin(), p.end(), [&](const std::pair<uint32_t, uint64_t>& e) {
            return ((sseq - e.first) & 0xFFFFFFu) >= (1u << 23);  // e.first > sseq (24-bit order)
          }));
}

int mt_ring_prepare(nts_hip_ctx* ctx, uint64_t w_bound, hipStream_t st, uint64_t* gen_hi,
                    uint32_t* seq) {
  NTS_RET(mt_ring_ensure(ctx));
  mt_ring_readback(ctx);
  auto upper_now = [&] {
    uint64_t u = ctx->mt_pos_done + w_bound;
    for (auto& e : ctx->mt_pending) u += e.second;
    return u;
  };
  // through the block holding the last word the layer may read, + one block
  uint64_t need = upper_now() / 624 + 2;
  auto ring_cap = [&] {  // blocks the generator may reach without overwriting
    const uint64_t oldest = ctx->mt_pos_done >= 624 ? ctx->mt_pos_done - 624 : 0;
    return (oldest + kMtRingWords) / 624;
  };
  if (need > ring_cap()) {  // too far ahead of what has been read back: wait for the layers
    NTS_HIP_TRY(hipStreamSynchronize(st));
    mt_ring_readback(ctx);
    need = upper_now() / 624 + 2;
    NTS_CHECK_ARG(need <= ring_cap(), "MT19937: a layer's word bound exceeds the stream ring");
  }
  ctx->mt_seq = (ctx->mt_seq + 1) & 0xFFFFFFu;
  if (ctx->mt_seq == 0) ctx->mt_seq = 1;  // (0: nothing done yet)
  *seq = ctx->mt_seq;
  ctx->mt_pending.push_back({ctx->mt_seq, w_bound});
  const uint64_t target = std::min(need + 2 * (w_bound / 624 + 1), ring_cap());
  while (ctx->mt_gen_blocks < target) {
    const uint32_t n = (uint32_t)std::min<uint64_t>(target - ctx->mt_gen_blocks, kMtGenChunk);
    hipLaunchKernelGGL(k_mt_ring_gen, dim3(1), dim3(kGenThreads), 0, ctx->mt_gen_stream,
                       ctx->mt_gen_raw, ctx->mt_ring, ctx->mt_gen_blocks, n);
    NTS_LAUNCH_CHECK();
    ctx->mt_gen_blocks += n;
    hipEvent_t ev;
    if (!ctx->mt_ev_pool.empty()) {
      ev = ctx->mt_ev_pool.back();
      ctx->mt_ev_pool.pop_back();
    } else {
      NTS_HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    NTS_HIP_TRY(hipEventRecord(ev, ctx->mt_gen_stream));
    ctx->mt_gen_evs.push_back({ctx->mt_gen_blocks, ev});
  }
  // wait for the first launch that covers the layer's words; launches before
  // it are complete then too (one stream), so their events go back to the pool
  auto& evs = ctx->mt_gen_evs;
  size_t i = 0;
  while (i + 1 < evs.size() && evs[i].first < need) ++i;
  NTS_HIP_TRY(hipStreamWaitEvent(st, evs[i].second, 0));
  *gen_hi = evs[i].first * 624;
  for (size_t k = 0; k < i; ++k) ctx->mt_ev_pool.push_back(evs[k].second);
  evs.erase(evs.begin(), evs.begin() + i);
  return NTS_OK;
}

uint64_t mt_word_bound(uint64_t e_cap, int fanout, double scale) {
  if (fanout <= 0) return 131072;  // (no draws: every neighbour taken)
  double h = 0.0;  // H_{f+1} - 1
  for (int k = 2; k <= fanout + 1; ++k) h += 1.0 / k;
  const double per_edge = (double)(fanout + 1) * h / fanout;
  const double w = ((double)e_cap * per_edge * 1.05 + 131072.0) * scale;
  return std::max<uint64_t>((uint64_t)std::ceil(w), 1024);
}

// The ring restarted from the generator state in ctx->mt_state (raw block B
// holding the last word consumed, _M_p = p): ring block 0 = B tempered (word
// p is the next to read), the generator continues from B (block 1 = twist(B)).
__global__ __launch_bounds__(256) void k_mt_rebase(const uint32_t* __restrict__ st,
                                                  uint32_t* __restrict__ ring,
                                                  uint32_t* __restrict__ raw,
                                                  uint64_t* __restrict__ done) {
  for (int k = threadIdx.x; k < 624; k += 256) {
    ring[k] = mt_temper(st[k]);
    raw[k] = st[k];
  }
  if (threadIdx.x == 0) *done = (uint64_t)st[624];  // position p, layer seq 0
}

int mt_ring_rebase(nts_hip_ctx* ctx) {
  NTS_RET(mt_ring_ensure(ctx));
  NTS_HIP_TRY(hipStreamSynchronize(ctx->mt_gen_stream));
  NTS_HIP_TRY(hipStreamSynchronize(ctx->stream));
  hipLaunchKernelGGL(k_mt_rebase, dim3(1), dim3(256), 0, ctx->stream, ctx->mt_state, ctx->mt_ring,
                     ctx->mt_gen_raw, ctx->mt_done);
  NTS_LAUNCH_CHECK();
  uint32_t p = 624;
  NTS_HIP_TRY(hipMemcpyAsync(&p, ctx->mt_state + 624, sizeof(uint32_t), hipMemcpyDeviceToHost,
                             ctx->stream));
  NTS_HIP_TRY(hipStreamSynchronize(ctx->stream));
  NTS_CHECK_ARG(p >= 1 && p <= 624, "MT19937 state: position out of range");
  *ctx->mt_done_host = p;
  ctx->mt_gen_blocks = 1;
  ctx->mt_seq = 0;
  ctx->mt_pos_done = p;
  ctx->mt_seq_done = 0;
  ctx->mt_pending.clear();
  for (auto& e : ctx->mt_gen_evs) ctx->mt_ev_pool.push_back(e.second);
  ctx->mt_gen_evs.clear();
  return NTS_OK;
}

// after a layer's last MT kernel: its end position back to the host (pinned)
int mt_ring_finish(nts_hip_ctx* ctx, hipStream_t st) {
  NTS_HIP_TRY(hipMemcpyAsync(ctx->mt_done_host, ctx->mt_done, sizeof(uint64_t),
                             hipMemcpyDeviceToHost, st));
  return NTS_OK;
}

}  // namespace nts_hip

using namespace nts_hip;

extern "C" int nts_hip_sample_layer(nts_hip_ctx* ctx, const nts_graph_dev* g, int fanout,
                                    int layer, uint64_t batch_seq, int rng_mode,
                                    int weight_type, nts_sampcsc_dev* o) {
  NTS_CHECK_ARG(ctx && g && o, "NULL argument");
  NTS_CHECK_ARG(g->column_offset && g->row_indices, "graph not on device");
  NTS_CHECK_ARG((o->destination || o->v_cap == 0) && o->v_size && o->column_offset &&
                    o->row_indices &&
                    o->sample_ans && o->edge_dst && o->source && o->sizes,
                "missing sampCSC buffer");
  const bool up_degree = (weight_type & NTS_WEIGHT_UP_DEGREE) != 0;
  weight_type &= 0xF;
  NTS_CHECK_ARG(weight_type >= NTS_WEIGHT_SUM && weight_type <= NTS_WEIGHT_MEAN_SAMPLED,
                "weight_type");
  NTS_CHECK_ARG(weight_type == NTS_WEIGHT_NONE || (o->edge_weight_forward && g->in_degree &&
                                                   g->out_degree),
                "weights requested without buffers/degrees");
  const bool up = up_degree && weight_type != NTS_WEIGHT_NONE;
  NTS_CHECK_ARG(rng_mode >= NTS_RNG_PHILOX && rng_mode <= NTS_RNG_MT19937_DIV, "rng_mode");
  NTS_CHECK_ARG(fanout <= (int)kBigFanoutMax, "fanout above 16384 (the distinct-position hash set)");
  NTS_CHECK_ARG(rng_mode == NTS_RNG_PHILOX || fanout <= (int)(kMtTab / 2),
                "MT19937 modes: fanout above 8192 (the exact path's hash set)");
  NTS_CHECK_ARG(g->n_vertices <= 0xFFFFFFFFull, "vertex count exceeds uint32 ids");
  const bool csr = o->row_offset != nullptr;
  NTS_CHECK_ARG(!csr || o->column_indices, "CSR requested without column_indices");
  NTS_CHECK_ARG(!o->omit_row || (o->omit_map && o->omit_loc), "omit_row needs omit_map + omit_loc");
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const uint64_t V = g->n_vertices;
  NTS_RET(ensure_vertices(ctx, V));
  const uint32_t nblk_marks = ceil_div(V, kMarkTile);

  // scratch layout (u32 words)
  auto al = [](uint64_t x) { return (x + 63) / 64 * 64; };
  const uint64_t scan_co = al(count_scan_tmp_elems(o->v_cap) + 1);
  const uint64_t blk = al(nblk_marks + 1);
  const uint64_t scan_blk = al(scan_tmp_elems<uint32_t>(nblk_marks) + 1);
  const uint64_t sort_k = csr ? al(o->e_cap) : 0, sort_v = sort_k;
  const uint64_t sort_p = csr ? 2 * al(o->e_cap) : 0;  // k_csr_bucket's payloads
  const size_t sort_tmp =
      csr ? std::max(radix_tmp_bytes(o->e_cap), radix_pass_tmp_bytes(o->e_cap)) : 0;
  const uint64_t up_n = up ? al(o->s_cap) : 0;
  // MT19937 modes: per-dst info; the chunked resolver (fanout 1..32) adds the
  // draws' scan, chunk stats, the bulk word stream + raw blocks, the window
  // tables and the chunk entries
  const bool mt_serial_env = getenv("NTS_MT_SERIAL") != nullptr;  // (read per call: tests A/B)
  // (small layers stay on the single walker: the tables' cost grows with the
  // layer's length times its window, while the walker's chain is short; the
  // C2 seed layer (10,000 dsts, fanout 25) is chunked: 8.9 vs 11.4 ms/step
  // with every layer chunked vs the walker for it, r04)
  const bool mt_chunked_env = getenv("NTS_MT_CHUNKED") != nullptr;
  const uint32_t mt_csz = o->v_cap <= kMtSmallV                            ? kMtChunkSmall
                          : o->v_cap <= (uint64_t)kMtMaxChunks * kMtChunkMid ? kMtChunkMid
                                                                             : kMtChunk;
  const bool mt_chunked = rng_mode != NTS_RNG_PHILOX && !mt_serial_env && fanout >= 1 &&
                          fanout <= 32 && (uint64_t)o->v_cap <= (uint64_t)kMtMaxChunks * mt_csz &&
                          (mt_chunked_env || o->v_cap >= kMtChunkedMinV);
  const uint64_t nch_cap = (uint64_t)o->v_cap / mt_csz + 1;
  // the words a layer may read (the stream generated ahead for it): a dst of
  // degree d > f takes d (H_d - H_{d-f}) draws on average to collect f
  // distinct positions (coupon collector), one word per draw (Lemire / DIV
  // rejections < 2^-16); per sampled edge that peaks at d = f + 1, (f+1)
  // (H_{f+1} - 1) / f (f = 10: 2.22, 25: 2.97, 32: 3.18), so the bound
  // covers every degree profile's mean with 5 % and 131,072 words to spare
  // (the per-dst spread is ~sqrt(f) draws: invisible past a few dsts)
  const uint64_t w_cap = mt_word_bound(o->e_cap, fanout, ctx->mt_budget_scale);
  const uint64_t mt_info_n = rng_mode != NTS_RNG_PHILOX ? al((uint64_t)o->v_cap * 4) : 0;
  const uint64_t mt_base_n = mt_chunked ? al((uint64_t)o->v_cap + 1) : 0;
  const uint64_t mt_stat_n = mt_chunked ? al(2 * nch_cap) : 0;
  const uint64_t mt_win_n = mt_chunked ? al(2 * nch_cap) : 0;
  const uint64_t mt_tab_n = mt_chunked ? al(nch_cap * kMtWmax) : 0;
  const uint64_t mt_ent_n = mt_chunked ? al(nch_cap + 1) : 0;
  const uint64_t mt_misc_n = mt_chunked ? 64 : 0;
  const uint64_t mt_n = mt_info_n + mt_base_n + mt_stat_n + mt_win_n + mt_tab_n + mt_ent_n +
                        mt_misc_n;
  const size_t need = (scan_co + blk + scan_blk + sort_k + sort_v + sort_p + up_n + mt_n) *
                          sizeof(uint32_t) + sort_tmp + 256;
  NTS_RET(ensure_scratch(ctx, need));
  uint32_t* w0 = (uint32_t*)ctx->scratch;
  uint32_t* t_scan_co = w0;
  uint32_t* t_blk = t_scan_co + scan_co;
  uint32_t* t_scan_blk = t_blk + blk;
  uint32_t* t_skey = t_scan_blk + scan_blk;
  uint32_t* t_seid = t_skey + sort_k;
  uint32_t* t_sdst = t_seid + sort_v;
  uint32_t* t_swf = t_sdst + sort_p / 2;
  uint32_t* t_up = t_sdst + sort_p;
  uint32_t* t_mt = t_up + up_n;  // MT19937 modes: per-dst MtInfo (16-byte aligned)
  void* t_sort = (void*)(t_mt + mt_n);

  const uint32_t gv = std::max(1u, std::min(ceil_div(o->v_cap, 256), kMaxGrid));
  const uint32_t ge = std::max(1u, std::min(ceil_div(o->e_cap, 256), kMaxGrid));

  // 1) per-dst counts -> column_offset, v_size, e_size (count + scan)
  {
    CountArgs ca;
    ca.goff = g->column_offset;
    ca.dst = o->destination;
    ca.v_in = o->v_size;
    ca.v_cap = o->v_cap;
    ca.fanout = fanout;
    ca.sizes = o->sizes;
    ca.e_cap = o->e_cap;
    ca.omit_map = o->omit_map;
    ca.omit_key = o->omit_key;
    ca.omit_loc = o->omit_loc;
    ca.omit_row = o->omit_row;
    NTS_RET(count_scan(ctx, ca, o->column_offset, st, t_scan_co));
  }

  // 2) selection (marks the frontier; the byte map is all zeros here: it is
  // zeroed when allocated and k_mark_write clears what each layer set)
  SelectArgs a;
  a.goff = g->column_offset;
  a.grows = g->row_indices;
  a.dst = o->destination;
  a.co = o->column_offset;
  a.sizes = o->sizes;
  a.ans = o->sample_ans;
  a.edst = o->edge_dst;
  a.marks = ctx->marks;
  a.e_cap = o->e_cap;
  a.fanout = fanout;
  a.layer = (uint32_t)layer;
  a.batch_seq = batch_seq;
  a.seed = ctx->seed;
  if (rng_mode == NTS_RNG_PHILOX) {
    if (fanout >= 0 && fanout <= kGrp) {
      const uint32_t gs =
          std::max(1u, std::min(ceil_div(o->v_cap, kSelWaves * kGrpPerWave), 4096u));
      hipLaunchKernelGGL(k_select_philox_g16, dim3(gs), dim3(kSelThreads), 0, st, a);
    } else if (fanout < 0 || fanout <= kSetCap) {
      const uint32_t gs = std::max(1u, std::min(ceil_div(o->v_cap, kSelWaves), 4096u));
      hipLaunchKernelGGL(k_select_philox, dim3(gs), dim3(kSelThreads), 0, st, a);
    } else {
      uint32_t cap = 1;
      while (cap < 2u * (uint32_t)fanout) cap <<= 1;
      const size_t lds = (size_t)cap * sizeof(uint32_t);
      NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_select_philox_big),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      const uint32_t gs = std::max(1u, std::min(o->v_cap, 2048u));
      hipLaunchKernelGGL(k_select_philox_big, dim3(gs), dim3(kWave), lds, st, a, cap);
    }
  } else {
    const int lem = rng_mode == NTS_RNG_MT19937_LEMIRE ? 1 : 0;
#ifdef NTS_MT_DEBUG  // (debug builds: -DNTS_MT_DEBUG=1)
    constexpr int mt_dbg = NTS_MT_DEBUG;
#else
    constexpr int mt_dbg = 0;
#endif
    uint4* info = reinterpret_cast<uint4*>(t_mt);
    // the stream words this layer may read are generated (ahead, on the
    // ring's side stream) before its kernels run
    uint64_t gen_hi = 0;
    uint32_t seq = 0;
    NTS_RET(mt_ring_prepare(ctx, w_cap, st, &gen_hi, &seq));
    if (mt_chunked) {
      uint32_t* base = t_mt + mt_info_n;
      float2* cstat = reinterpret_cast<float2*>(base + mt_base_n);
      uint2* win = reinterpret_cast<uint2*>(base + mt_base_n + mt_stat_n);
      uint32_t* tabs = base + mt_base_n + mt_stat_n + mt_win_n;
      uint32_t* entries = tabs + mt_tab_n;
      uint32_t* misc = entries + mt_ent_n;  // [1] fallbacks, [2..3] the layer's first stream word
      uint64_t* a0p = reinterpret_cast<uint64_t*>(misc + 2);
      NTS_HIP_TRY(hipMemsetAsync(cstat, 0, mt_stat_n * sizeof(uint32_t), st));
      hipLaunchKernelGGL(k_mt_prep, dim3(gv), dim3(256), 0, st, g->column_offset, o->destination,
                         o->column_offset, o->sizes, o->e_cap, lem, info, base, cstat, mt_csz,
                         (const uint64_t*)ctx->mt_done, a0p);
      NTS_LAUNCH_CHECK();
      NTS_RET(scan1_exclusive(ctx, base, base, o->sizes, o->v_cap, st));
      const dim3 tgrid(kMtWmax / 256, (uint32_t)nch_cap);
      const MtChunked chunked{ctx->mt_ring, a0p, gen_hi, base, entries, nullptr, 0u, nullptr,
                              mt_csz};
      // the tables' and resolver's draw bound NMAX at the layer's fanout
      // class: each lane's window holds NMAX + 8 words in registers (C2 with
      // --rng mt: 4.49 ms/step with 16 / 32 for fanouts 10 / 25, 4.17 with 12 /
      // 32, 3.91 with 10 / 25)
      auto run = [&](auto nmax, auto g) -> int {
        constexpr int NM = decltype(nmax)::value, G = decltype(g)::value;
        hipLaunchKernelGGL(k_mtp_tables<NM>, tgrid, dim3(256), 0, st, info, base, o->sizes, cstat,
                           ctx->mt_ring, a0p, gen_hi, lem, mt_csz, win, tabs);
        NTS_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_mtp_resolve<NM>, dim3(1), dim3(kWave), 0, st, info, base, o->sizes,
                           ctx->mt_ring, a0p, gen_hi, lem, mt_csz, win, tabs, entries, ctx->mt_done,
                           seq, ctx->mt_state, o->sizes + 3, misc + 1);
        NTS_LAUNCH_CHECK();
        hipLaunchKernelGGL((k_mt_serial<G, true>), dim3((uint32_t)nch_cap), dim3(kWave), 0, st, info,
                           o->sizes, o->sample_ans, nullptr, lem, mt_dbg, chunked);
        return NTS_OK;
      };
      using I16 = std::integral_constant<int, 16>;
      using I32 = std::integral_constant<int, 32>;
      if (fanout <= 10) NTS_RET(run(std::integral_constant<int, 10>{}, I16{}));
      else if (fanout <= 12) NTS_RET(run(std::integral_constant<int, 12>{}, I16{}));
      else if (fanout <= 16) NTS_RET(run(I16{}, I16{}));
      else if (fanout <= 25) NTS_RET(run(std::integral_constant<int, 25>{}, I32{}));
      else NTS_RET(run(I32{}, I32{}));
      NTS_LAUNCH_CHECK();
      NTS_RET(mt_ring_finish(ctx, st));
      const uint32_t gs = std::max(1u, std::min(ceil_div(o->v_cap, kSelWaves * kGrpPerWave), 4096u));
      hipLaunchKernelGGL(k_mt_rows, dim3(gs), dim3(kSelThreads), 0, st, a);
      NTS_LAUNCH_CHECK();
      goto frontier;
    }
    hipLaunchKernelGGL(k_mt_prep, dim3(gv), dim3(256), 0, st, g->column_offset, o->destination,
                       o->column_offset, o->sizes, o->e_cap, lem, info, nullptr, nullptr, 1u,
                       nullptr, nullptr);
    NTS_LAUNCH_CHECK();
    const MtChunked whole{ctx->mt_ring, nullptr, gen_hi, nullptr, nullptr, ctx->mt_done, seq,
                          o->sizes + 3};
    if (fanout >= 0 && fanout <= 16)
      hipLaunchKernelGGL((k_mt_serial<16, false>), dim3(1), dim3(kWave), 0, st, info, o->sizes,
                         o->sample_ans, ctx->mt_state, lem, mt_dbg, whole);
    else if (fanout >= 0 && fanout <= 32)
      hipLaunchKernelGGL((k_mt_serial<32, false>), dim3(1), dim3(kWave), 0, st, info, o->sizes,
                         o->sample_ans, ctx->mt_state, lem, mt_dbg, whole);
    else
      hipLaunchKernelGGL((k_mt_serial<64, false>), dim3(1), dim3(kWave), 0, st, info, o->sizes,
                         o->sample_ans, ctx->mt_state, lem, mt_dbg, whole);
    NTS_LAUNCH_CHECK();
    NTS_RET(mt_ring_finish(ctx, st));
    const uint32_t gs = std::max(1u, std::min(ceil_div(o->v_cap, kSelWaves * kGrpPerWave), 4096u));
    hipLaunchKernelGGL(k_mt_rows, dim3(gs), dim3(kSelThreads), 0, st, a);
  }
  NTS_LAUNCH_CHECK();

frontier:
  if (o->dst_local_id) {
    hipLaunchKernelGGL(k_mark_dst, dim3(gv), dim3(256), 0, st, o->destination, o->sizes,
                       ctx->marks);
    NTS_LAUNCH_CHECK();
  }

  // 3) frontier: ascending compaction of the byte map — single pass up to
  // kMarkFusedMaxTiles tiles (C2's 57), else (and with the two-kernel scans,
  // NTS_SCAN1=0) count + write: at products' 598 tiles the look-back chain
  // took 23 us a layer against 5 + 9 for the pair (scripts/r05_c3tr.sh)
  constexpr uint32_t kMarkFusedMaxTiles = 256;
  if (scan1_enabled() && nblk_marks <= kMarkFusedMaxTiles) {
    NTS_RET(ensure_scan_state(ctx, scan1_state_elems((uint64_t)nblk_marks * 4096)));
    hipLaunchKernelGGL(k_mark_fused, dim3(nblk_marks), dim3(kMarkThreads), 0, st, ctx->marks,
                       nblk_marks, V, o->s_cap, o->source, ctx->src_index, o->sizes,
                       ctx->scan_state, scan_next_epoch(ctx), scan_ticket(ctx));
    NTS_LAUNCH_CHECK();
  } else {
    hipLaunchKernelGGL(k_mark_count, dim3(nblk_marks), dim3(kMarkThreads), 0, st, ctx->marks,
                       t_blk);
    NTS_LAUNCH_CHECK();
    if (nblk_marks <= kMarkDirectTiles) {  // up to 8M vertices: no scan kernel
      hipLaunchKernelGGL(k_mark_write<true>, dim3(nblk_marks), dim3(kMarkThreads), 0, st,
                         ctx->marks, t_blk, nblk_marks, V, o->s_cap, o->source, ctx->src_index,
                         o->sizes);
    } else {
      NTS_RET(scan_exclusive<uint32_t>(t_blk, t_blk, nullptr, nblk_marks, t_scan_blk, st));
      hipLaunchKernelGGL(k_mark_write<false>, dim3(nblk_marks), dim3(kMarkThreads), 0, st,
                         ctx->marks, t_blk, nblk_marks, V, o->s_cap, o->source, ctx->src_index,
                         o->sizes);
    }
    NTS_LAUNCH_CHECK();
  }

  if (o->dst_local_id) {
    hipLaunchKernelGGL(k_dst_local, dim3(gv), dim3(256), 0, st, o->destination, ctx->src_index,
                       o->sizes, o->dst_local_id);
    NTS_LAUNCH_CHECK();
  }

  // 4) relabel to local ids + forward weights
  RelabelArgs ra{o->sample_ans,      o->edge_dst, o->destination, ctx->src_index,
                 g->out_degree,      g->in_degree, o->column_offset, o->sizes,
                 weight_type,        o->row_indices, o->edge_weight_forward,
                 up ? t_up : nullptr, (up || csr) ? nullptr : o->sizes_host};
  if (up) NTS_HIP_TRY(hipMemsetAsync(t_up, 0, up_n * sizeof(uint32_t), st));
  hipLaunchKernelGGL(k_relabel, dim3(ge), dim3(256), 0, st, ra);
  NTS_LAUNCH_CHECK();
  if (up) {
    hipLaunchKernelGGL(k_up_weight, dim3(ge), dim3(256), 0, st, o->row_indices, o->edge_dst,
                       o->column_offset, t_up, o->sizes, weight_type, o->edge_weight_forward,
                       csr ? nullptr : o->sizes_host);
    NTS_LAUNCH_CHECK();
  }

  // 5) CSR transpose (stable in edge order = ascending local dst): radix sort
  // of (local src, edge id), then the CSR arrays.  Measured and dropped in
  // round 4 (C2, per layer): fusing the relabel with the first pass's digit
  // counts (20 vs 11 + 8 us: a tile per block is fewer threads for its random
  // gathers), the CSR writes into the last pass (45 vs 16 + 20 us), and the
  // later passes' tile offsets by a per-digit decoupled look-back (48-91 us)
  // or counted by the pass before with atomics (65 vs 16 us).
  if (csr) {
    const uint32_t bits = ceil_log2((uint64_t)o->s_cap + 1);
#ifndef NTS_CSR_RADIX2  // (A/B build: the two-pass radix sort + k_csr_finalize)
    if (bits >= 11 && bits <= 19) {
      // one radix pass on the high H bits, then k_csr_bucket per 2^L sources
      const uint32_t H = std::min(9u, bits - 6), L = bits - H;
      const uint32_t* totals = nullptr;
      const bool wpl = weight_type != NTS_WEIGHT_NONE && o->edge_weight_backward;
      RadixPayload pl;
      pl.p1_in = o->edge_dst;
      pl.p1_out = t_sdst;
      if (wpl) {
        pl.p2_in = reinterpret_cast<const uint32_t*>(o->edge_weight_forward);
        pl.p2_out = t_swf;
      }
      // (the edge ids only where the CSR's edge-id map is asked for: GAT)
      NTS_RET(radix_pass_pairs(o->row_indices, nullptr, t_skey, o->csr_edge_id ? t_seid : nullptr,
                               o->sizes + 1, o->e_cap, L, H, t_sort, st, &totals, pl));
      const uint32_t* swf = wpl ? t_swf : nullptr;
#define NTS_CSR_BUCKET(LL)                                                                        \
  hipLaunchKernelGGL(k_csr_bucket<LL>, dim3(1u << H), dim3(kCsrBucketThreads), 0, st, t_skey,   \
                     t_seid, totals, t_sdst, swf, o->sizes, o->row_offset, o->column_indices,   \
                     o->edge_weight_backward, o->csr_edge_id, o->sizes_host)
      switch (L) {
        case 6: NTS_CSR_BUCKET(6); break;
        case 7: NTS_CSR_BUCKET(7); break;
        case 8: NTS_CSR_BUCKET(8); break;
        case 9: NTS_CSR_BUCKET(9); break;
        default: NTS_CSR_BUCKET(10); break;
      }
#undef NTS_CSR_BUCKET
      NTS_LAUNCH_CHECK();
      return NTS_OK;
    }
#endif
    NTS_RET(radix_sort_pairs(o->row_indices, nullptr, t_skey, t_seid, o->sizes + 1, o->e_cap,
                             bits, t_sort, st, ctx));
    hipLaunchKernelGGL(k_csr_finalize, dim3(ge), dim3(256), 0, st, t_skey, t_seid, o->edge_dst,
                       weight_type == NTS_WEIGHT_NONE ? nullptr : o->edge_weight_forward,
                       o->sizes, o->row_offset, o->column_indices, o->edge_weight_backward,
                       o->csr_edge_id, o->sizes_host);
    NTS_LAUNCH_CHECK();
  }
  return NTS_OK;
}

extern "C" int nts_hip_mt_budget_scale(nts_hip_ctx* ctx, double scale) {
  NTS_CHECK_ARG(ctx, "ctx is NULL");
  NTS_CHECK_ARG(scale > 0.0 && scale < 1e6, "scale must be > 0");
  ctx->mt_budget_scale = scale;
  return NTS_OK;
}

extern "C" int nts_hip_mt_checkpoint(nts_hip_ctx* ctx, uint32_t* dev_state625) {
  NTS_CHECK_ARG(ctx && dev_state625, "NULL argument");
  NTS_HIP_TRY(hipMemcpyAsync(dev_state625, ctx->mt_state, 625 * sizeof(uint32_t),
                             hipMemcpyDeviceToDevice, ctx->stream));
  return NTS_OK;
}

extern "C" int nts_hip_mt_rewind(nts_hip_ctx* ctx, const uint32_t* dev_state625) {
  NTS_CHECK_ARG(ctx && dev_state625, "NULL argument");
  if (ctx->mt_gen_stream) NTS_HIP_TRY(hipStreamSynchronize(ctx->mt_gen_stream));
  NTS_HIP_TRY(hipStreamSynchronize(ctx->stream));
  NTS_HIP_TRY(hipMemcpyAsync(ctx->mt_state, dev_state625, 625 * sizeof(uint32_t),
                             hipMemcpyDeviceToDevice, ctx->stream));
  return mt_ring_rebase(ctx);
}
