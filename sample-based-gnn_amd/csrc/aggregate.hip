// Sampled aggregation (CSC gather SpMM, CSR transpose gather, atomic scatter),
// row/label gathers and the fused Adam step.
//
// The aggregation is HBM-bound (~2 flop/B).  Layout: X/Y row-major
// fp32 [rows, ld]; one wave-group (LPD lanes) per destination row, each lane
// owning NCH vectors of VEC floats of the row; neighbour rows are fetched 4
// edges ahead so every lane keeps 4*NCH independent loads in flight.  The sum
// runs in CSC edge order as acc + x*w with contraction disabled: bit-identical
// to the reference's MiniBatchFuseOp/nts_comp (core/ntsBaseOp.hpp:546-562,
// `_mm256_add_ps(_mm256_mul_ps(source,w),destination)`) for the same sampCSC.
#include "common.hpp"

#pragma clang fp contract(off)

namespace nts_hip {

template <int VEC>
struct VT;
template <>
struct VT<1> {
  using T = float;
  __device__ static __forceinline__ T zero() { return 0.f; }
  __device__ static __forceinline__ T madd(T a, T x, float w) { return a + x * w; }
  __device__ static __forceinline__ T scale(T x, float w) { return x * w; }
  __device__ static __forceinline__ void st_nt(T* p, T v) { __builtin_nontemporal_store(v, p); }
  __device__ static __forceinline__ void st_part(T* p, T v, uint32_t) { st_nt(p, v); }
};
template <>
struct VT<2> {
  using T = float2;
  __device__ static __forceinline__ T zero() { return make_float2(0.f, 0.f); }
  __device__ static __forceinline__ T madd(T a, T x, float w) {
    return make_float2(a.x + x.x * w, a.y + x.y * w);
  }
  __device__ static __forceinline__ T scale(T x, float w) { return make_float2(x.x * w, x.y * w); }
  __device__ static __forceinline__ void st_nt(T* p, T v) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 u = {v.x, v.y};
    __builtin_nontemporal_store(u, reinterpret_cast<f2*>(p));
  }
  __device__ static __forceinline__ void st_part(T* p, T v, uint32_t) {  // 1 of 2 valid
    __builtin_nontemporal_store(v.x, reinterpret_cast<float*>(p));
  }
};
template <>
struct VT<4> {
  using T = float4;
  __device__ static __forceinline__ T zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ static __forceinline__ T madd(T a, T x, float w) {
    return make_float4(a.x + x.x * w, a.y + x.y * w, a.z + x.z * w, a.w + x.w * w);
  }
  __device__ static __forceinline__ T scale(T x, float w) {
    return make_float4(x.x * w, x.y * w, x.z * w, x.w * w);
  }
  __device__ static __forceinline__ void st_nt(T* p, T v) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    f4 u = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(u, reinterpret_cast<f4*>(p));
  }
  __device__ static __forceinline__ void st_part(T* p, T v, uint32_t nvalid) {  // 1..3 valid
    float* q = reinterpret_cast<float*>(p);
    __builtin_nontemporal_store(v.x, q);
    if (nvalid > 1) __builtin_nontemporal_store(v.y, q + 1);
    if (nvalid > 2) __builtin_nontemporal_store(v.z, q + 2);
  }
};

constexpr int kAggThreads = 256;

// y[d, :] = sum_{e in [off[d], off[d+1])} w[e] * x[row(e), :]
// row(e) = MAP ? map[idx[e]] : idx[e];  w == nullptr -> weight 1.
// Per destination the LPD-lane group loads up to LPD edges' (row, weight) at
// once — one lane per edge, the map lookup included — and then fetches the
// neighbour rows U at a time (row ids broadcast by __shfl, the tail batch
// predicated), so a row costs off -> idx/map -> ceil(deg/U) row rounds of
// memory latency instead of two dependent loads per U edges plus a serial
// remainder.  The sum order is still the CSC edge order.
//
// TIER (two-tier feature table, load_feature_gpu_cache semantics,
// core/ntsFastSampler.hpp:263-317): x is the HBM cache of the hottest rows
// and tier.cmap[g] its slot for global row g, or kNotCached, in which case the
// row is read from the host-pinned table tier.host (zero-copy over the host
// link).  The per-edge id carries the tier in bit 31 (vertex ids < 2^31).
// host_local: the non-cached rows were staged by local src id (tier.host is
// then an HBM buffer [src_size, ldh], see nts_hip_stage_uncached_rows)
struct Tier {
  const uint32_t* cmap;
  const float* host;
  uint64_t ldh;
  int host_local;
};
constexpr uint32_t kNotCached = 0xFFFFFFFFu;
constexpr uint32_t kHostBit = 0x80000000u;

// MODE: what the gather computes around the weighted sum (MAP/TIER only with kAggPlain)
//   kAggPlain: y = A x
//   kAggAct:   y = dropout(relu(A x), p) — vertexForward's activation in the
//              epilogue, keep bits keyed exactly like the GEMM epilogue of
//              nts_hip_gemm_relu_dropout_f32 (dropout_words(row, col, seed, offset))
//   kAggMask:  y = A (x ⊙ [mx > 0] · scale) — that activation's backward fused
//              into the row loads (mx = the forward activation, same shape as x)
//   kAggPostMask: y = (A x) ⊙ [mx > 0] · scale with mx indexed by the OUTPUT
//              row (the activation backward applied to the gathered sum: the
//              graph-op backward feeding a transform-first bottom layer)
//   kAggColmax: kAggPlain, and per block the column maxima of |y| over the
//     block's output rows into row blockIdx.x of ax.cm_out (the f16
//     pair-table TN GEMM's per-chunk column scales, nts_hip_spmm_csr_bwd_colmax)
enum { kAggPlain = 0, kAggAct = 1, kAggMask = 2, kAggPostMask = 3, kAggColmax = 4 };
struct AggExtra {
  const float* mx = nullptr;
  uint64_t ldm = 0;
  float scale = 1.f;
  uint32_t keep_threshold = 0;
  uint64_t seed = 0, offset = 0;
  // per-block column maxima of the output (nts_hip_spmm_csr_bwd_colmax):
  // cm_out[b * F + col] = max over block b's rows d of |rs(d) y[d, col]|, float
  // bits, rs(d) = cm_rs[cm_map[d]] (cm_map NULL: cm_rs[d]; cm_rs NULL: 1)
  uint32_t* cm_out = nullptr;
  const float* cm_rs = nullptr;
  const uint32_t* cm_map = nullptr;
  // the activation's keep mask as bits (nts_hip_act_bits_words): kAggAct
  // writes them beside its output (bits_out), kAggPostMask reads them instead
  // of the output's rows (bits_in); ldb words per row
  uint32_t* bits_out = nullptr;
  const uint32_t* bits_in = nullptr;
  uint64_t ldb = 0;
};

// Mask bits of a float4 row on LPD >= 32 lanes (one chunk of NCH float4 a
// lane): word (h NCH + c) 4 + q of a row holds, at bit b, whether component q
// of chunk c of lane 32 h + b is > 0 (h = 0 for 32-lane groups)
// (nts_hip_act_bits_words: (LPD / 32) NCH 4 words a row)

template <int VEC>
__device__ __forceinline__ float& vcomp(typename VT<VEC>::T& v, int q) {
  return reinterpret_cast<float*>(&v)[q];
}
template <int VEC>
__device__ __forceinline__ float vcomp(const typename VT<VEC>::T& v, int q) {
  return reinterpret_cast<const float*>(&v)[q];
}

// acc[c] += sum over the edges [beg, end) in edge order of w[e] * row(e)[col],
// col = c0 + sl + c * LPD (one LPD-lane group, see k_spmm_gather)
// pre: the row's first chunk of edge ids / weights was loaded by the caller
// (lane sl: entry beg + sl, raw id before MAP/TIER) — one row ahead, so that
// the chain per row is the row loads alone
template <int VEC, int LPD, int NCH, bool MAP, int U, bool TIER, int MODE>
__device__ __forceinline__ void gather_edges(typename VT<VEC>::T (&acc)[NCH], uint32_t beg,
                                             uint32_t end, uint32_t c0, int sl,
                                             const uint32_t* __restrict__ idx,
                                             const float* __restrict__ w,
                                             const float* __restrict__ x, uint64_t ldx,
                                             const uint32_t* __restrict__ map, uint32_t nv,
                                             const Tier& tier, const AggExtra& ax,
                                             bool pre = false, uint32_t pre_r = 0,
                                             float pre_w = 0.f) {
  using V = VT<VEC>;
  using T = typename V::T;
  for (uint32_t cb = beg; cb < end; cb += LPD) {
    const uint32_t ne = min(end - cb, (uint32_t)LPD);
    uint32_t my_r = 0;
    float my_w = 0.f;
    if ((uint32_t)sl < ne) {  // streamed once: do not keep in cache
      if (pre && cb == beg) {
        my_r = pre_r;
        my_w = pre_w;
      } else {
        my_r = __builtin_nontemporal_load(idx + cb + sl);
        my_w = w ? __builtin_nontemporal_load(w + cb + sl) : 1.0f;
      }
      const uint32_t loc = my_r;
      if (MAP) my_r = map[my_r];
      if (TIER) {
        const uint32_t slot = tier.cmap[my_r];
        my_r = slot != kNotCached ? slot : ((tier.host_local ? loc : my_r) | kHostBit);
      }
    }
    for (uint32_t j0 = 0; j0 < ne; j0 += U) {
      T xv[U][NCH];
      T mv[MODE == kAggMask ? U : 1][MODE == kAggMask ? NCH : 1];
      float ww[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int src = (int)(j0 + j) & (LPD - 1);
        const uint32_t r = (uint32_t)__shfl((int)my_r, src, LPD);
        ww[j] = __shfl(my_w, src, LPD);
        const bool ok = j0 + j < ne;
        const T* xrow = reinterpret_cast<const T*>(
            TIER && (r & kHostBit) ? tier.host + (uint64_t)(r & ~kHostBit) * tier.ldh
                                   : x + (uint64_t)r * ldx);
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const uint32_t col = c0 + sl + c * LPD;
          xv[j][c] = (ok && col < nv) ? xrow[col] : V::zero();
        }
        if constexpr (MODE == kAggMask) {
          const T* mrow = reinterpret_cast<const T*>(ax.mx + (uint64_t)r * ax.ldm);
#pragma unroll
          for (int c = 0; c < NCH; ++c) {
            const uint32_t col = c0 + sl + c * LPD;
            mv[j][c] = (ok && col < nv) ? mrow[col] : V::zero();
          }
        }
      }
      if constexpr (MODE == kAggMask) {  // dZ = dX ⊙ [X > 0] · scale
#pragma unroll
        for (int j = 0; j < U; ++j)
#pragma unroll
          for (int c = 0; c < NCH; ++c)
#pragma unroll
            for (int q = 0; q < VEC; ++q) {
              float& g = vcomp<VEC>(xv[j][c], q);
              g = vcomp<VEC>(mv[j][c], q) > 0.f ? g * ax.scale : 0.f;
            }
      }
#pragma unroll
      for (int j = 0; j < U; ++j)
        if (j0 + j < ne) {
#pragma unroll
          for (int c = 0; c < NCH; ++c) acc[c] = V::madd(acc[c], xv[j][c], ww[j]);
        }
    }
  }
}

// epilogue of one output row: activation (kAggAct) and the store
template <int VEC, int LPD, int NCH, int MODE>
__device__ __forceinline__ void store_row(typename VT<VEC>::T (&acc)[NCH], uint32_t d, uint32_t c0,
                                          int sl, uint32_t nv, uint32_t last_valid,
                                          float* __restrict__ y, uint64_t ldy, const AggExtra& ax) {
  using V = VT<VEC>;
  using T = typename V::T;
  if constexpr (MODE == kAggAct) {  // relu + inverted dropout, mask never stored
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const uint32_t f0 = (c0 + sl + c * LPD) * VEC;  // first float column
#pragma unroll
      for (int q2 = 0; q2 < (VEC + 1) / 2; ++q2) {
        uint4 rnd = make_uint4(0u, 0u, 0u, 0u);
        if (ax.keep_threshold) rnd = dropout_words((uint64_t)d, f0 + 2 * q2, ax.seed, ax.offset);
        const uint32_t wd = (d & 3) == 0 ? rnd.x : (d & 3) == 1 ? rnd.y : (d & 3) == 2 ? rnd.z : rnd.w;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (2 * q2 + h >= VEC) break;
          const uint32_t col = f0 + 2 * q2 + h;
          float& v = vcomp<VEC>(acc[c], 2 * q2 + h);
          v = (dropout_bits(wd, col) >= ax.keep_threshold && v > 0.f) ? v * ax.scale : 0.f;
        }
      }
    }
    if constexpr (VEC == 4 && LPD >= 32) {
      if (ax.bits_out) {  // (uniform) the row's keep mask, one ballot per component
        const int hw = (threadIdx.x & 63) >> 5;
        uint32_t* brow = ax.bits_out + (uint64_t)d * ax.ldb + (LPD == 64 ? hw : 0) * NCH * 4;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          uint32_t wq[4];
#pragma unroll
          for (int q = 0; q < 4; ++q)
            wq[q] = (uint32_t)(__ballot(vcomp<VEC>(acc[c], q) > 0.f) >> (32 * hw));
          if ((threadIdx.x & 31) == 0)
            *reinterpret_cast<uint4*>(brow + 4 * c) = make_uint4(wq[0], wq[1], wq[2], wq[3]);
        }
      }
    }
  }
  if constexpr (MODE == kAggPostMask) {  // dZ = dX ⊙ [X > 0] · scale, X row d
    bool bits = false;
    if constexpr (VEC == 4 && LPD >= 32) {
      if (ax.bits_in) {  // (uniform) the keep mask as bits
        bits = true;
        const uint4* brow = reinterpret_cast<const uint4*>(ax.bits_in + (uint64_t)d * ax.ldb) +
                            (LPD == 64 ? (sl >> 5) : 0) * NCH;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const uint4 b4 = brow[c];
          const uint32_t wq[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float& v = vcomp<VEC>(acc[c], q);
            v = ((wq[q] >> (sl & 31)) & 1u) ? v * ax.scale : 0.f;
          }
        }
      }
    }
    if (!bits) {
      const T* mrow = reinterpret_cast<const T*>(ax.mx + (uint64_t)d * ax.ldm);
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const uint32_t col = c0 + sl + c * LPD;
        if (col < nv) {
          const T m = mrow[col];
#pragma unroll
          for (int q = 0; q < VEC; ++q) {
            float& v = vcomp<VEC>(acc[c], q);
            v = vcomp<VEC>(m, q) > 0.f ? v * ax.scale : 0.f;
          }
        }
      }
    }
  }
  T* yrow = reinterpret_cast<T*>(y + (uint64_t)d * ldy);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {  // output rows are not re-read here: keep them
    const uint32_t col = c0 + sl + c * LPD;  // out of the cache that serves x rows
    if (col + 1 < nv || (col + 1 == nv && last_valid == (uint32_t)VEC)) {
      V::st_nt(yrow + col, acc[c]);
    } else if (col + 1 == nv) {  // partial last vector: only the valid floats
      V::st_part(yrow + col, acc[c], last_valid);
    }
  }
}

// COOP (the CSR transposes, whose rows are as long as a source is popular —
// hundreds of edges for the hubs of a power-law graph against ~6 on average):
// a row longer than kLongRow(U) edges is not summed by its own lane group,
// which would serialise ~len/U rounds of memory latency and set the whole
// launch's time; the block's GPB groups each sum a contiguous GPB-th of its
// edges (in edge order) and the partial sums are added in group order through
// LDS.  Deterministic; rows up to kLongRow edges keep the serial edge order
// (bit-identical to MiniBatchFuseOp::backward's), longer rows are summed as
// GPB in-order pieces.  A group takes at most kCoopRows rows (grid >=
// ceil(n_cap / (GPB kCoopRows))): the block's long rows fit its list.
template <int U>
constexpr uint32_t kLongRow() { return 4 * U; }
constexpr uint32_t kCoopRows = 16;

// Row software pipeline of k_spmm_gather (compile-time A/B builds, `make
// variant`): 0 none, 1 the next row's offsets, 2 the offsets two rows ahead
// and the first id/weight chunk one row ahead; and the waves-per-SIMD floor of
// its single-chunk instances (0: the compiler's choice).  Measured at C2 size
// (scripts/micro_agg.py, r04): bottom fwd / CSR bwd 103.7 / 121.7 us with 0,
// 105.9 / 130.5 with 1, 102.3 / 130.6 with 2, 114.4 / 152.1 with 2 and a
// floor of 6 waves (spills) — the prefetch registers cost a wave per SIMD
// (occupancy 6 -> 5) and the gather needs the waves more than the shorter
// chain, so 0 stays
#ifndef NTS_AGG_PF
#define NTS_AGG_PF 0
#endif
#ifndef NTS_AGG_WPE
#define NTS_AGG_WPE 0
#endif
constexpr int kAggPf = NTS_AGG_PF;
constexpr int kAggWpe = NTS_AGG_WPE == 0 ? 1 : NTS_AGG_WPE;

template <int VEC, int LPD, int NCH, bool MAP, int U, bool TIER, int MODE = kAggPlain,
          bool COOP = false>
__global__ __launch_bounds__(kAggThreads) __attribute__((amdgpu_waves_per_eu(NCH == 1 ? kAggWpe : 1))) void k_spmm_gather(
    const uint32_t* __restrict__ off, const uint32_t* __restrict__ idx,
    const float* __restrict__ w, const uint32_t* n_dev, uint32_t n_cap,
    const float* __restrict__ x, uint64_t ldx, const uint32_t* __restrict__ map, uint32_t nv,
    float* __restrict__ y, uint64_t ldy, uint32_t last_valid, Tier tier, AggExtra ax) {
  using V = VT<VEC>;
  using T = typename V::T;
  static_assert(MODE == kAggPlain || (!MAP && !TIER), "activation modes gather local rows only");
  constexpr bool CM = MODE == kAggColmax;
  constexpr int EM = CM ? kAggPlain : MODE;  // the gather and store proper
  const uint32_t n = n_dev ? min(*n_dev, n_cap) : n_cap;
  constexpr int GPB = kAggThreads / LPD;
  const int grp = threadIdx.x / LPD, sl = threadIdx.x % LPD;
  __shared__ uint32_t long_rows[COOP ? GPB * kCoopRows : 1];
  __shared__ uint32_t n_long;
  if (COOP) {
    if (threadIdx.x == 0) n_long = 0;
    __syncthreads();
  }
  // kAggColmax: the block's column maxima in LDS (float bits; non-negative
  // floats order as their bits), one LDS atomic per lane and column per row
  const uint32_t ncol = (nv - 1) * VEC + last_valid;
  __shared__ uint32_t smax[CM ? 512 : 1];
  if constexpr (CM) {
    for (uint32_t c = threadIdx.x; c < ncol; c += kAggThreads) smax[c] = 0u;
    __syncthreads();
  }
  auto colmax_row = [&](const T (&acc)[NCH], uint32_t c0, uint32_t d) {
    // the row's scale (a power of two: the product is exact unless it leaves
    // the float range)
    const float rsd = ax.cm_rs ? ax.cm_rs[ax.cm_map ? ax.cm_map[d] : d] : 1.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        const uint32_t col = (c0 + sl + c * LPD) * VEC + q;
        if (col < ncol)
          atomicMax(&smax[col], __float_as_uint(fabsf(vcomp<VEC>(acc[c], q) * rsd)));
      }
  };
  // software pipeline over the group's rows: the offsets two rows ahead and
  // the first chunk of edge ids / weights one row ahead are loaded while this
  // row is gathered (the chain per row off -> ids -> rows becomes the rows)
  const uint32_t stride = gridDim.x * GPB;
  auto first_chunk = [&](uint32_t b, uint32_t e, uint32_t& r, float& wt) {
    r = 0;
    wt = 0.f;
    if ((uint32_t)sl < e - b) {
      r = __builtin_nontemporal_load(idx + b + sl);
      wt = w ? __builtin_nontemporal_load(w + b + sl) : 1.0f;
    }
  };
#ifdef NTS_AGG_XCD
  // (A/B build: XCD-aware block order — the blocks one XCD runs, b % 8 under
  // round-robin placement, take one contiguous eighth of the dsts, so each
  // XCD's L2 sees one dst range's sources; bijective for any grid)
  uint32_t bid = blockIdx.x;
  if constexpr (!CM) {
    const uint32_t q8 = gridDim.x / 8, r8 = gridDim.x % 8, x8 = blockIdx.x % 8;
    bid = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + blockIdx.x / 8;
  }
  uint32_t d = bid * GPB + grp;
#else
  uint32_t d = blockIdx.x * GPB + grp;
#endif
  uint32_t beg = 0, end = 0, beg1 = 0, end1 = 0, pr = 0;
  float pw = 0.f;
  if (kAggPf >= 1 && d < n) {
    beg = off[d];
    end = off[d + 1];
  }
  if (kAggPf >= 2 && d + stride < n) {
    beg1 = off[d + stride];
    end1 = off[d + stride + 1];
  }
  if (kAggPf >= 2) first_chunk(beg, end, pr, pw);
  for (; d < n; d += stride) {
    uint32_t cbeg, cend, cpr = 0;
    float cpw = 0.f;
    if constexpr (kAggPf == 0) {
      cbeg = off[d];
      cend = off[d + 1];
    } else if constexpr (kAggPf == 1) {
      cbeg = beg;
      cend = end;
      if (d + stride < n) {
        beg = off[d + stride];
        end = off[d + stride + 1];
      }
    } else {
      uint32_t beg2 = 0, end2 = 0, pr1, dn2 = d + 2 * stride;
      float pw1;
      if (dn2 < n) {
        beg2 = off[dn2];
        end2 = off[dn2 + 1];
      }
      first_chunk(beg1, end1, pr1, pw1);
      cbeg = beg;
      cend = end;
      cpr = pr;
      cpw = pw;
      beg = beg1;
      end = end1;
      beg1 = beg2;
      end1 = end2;
      pr = pr1;
      pw = pw1;
    }
    if (COOP && cend - cbeg > kLongRow<U>()) {  // summed by the whole block below
      if (sl == 0) long_rows[atomicAdd(&n_long, 1u)] = d;
      continue;
    }
    for (uint32_t c0 = 0; c0 < nv; c0 += LPD * NCH) {
      T acc[NCH];
#pragma unroll
      for (int c = 0; c < NCH; ++c) acc[c] = V::zero();
      // kAggPostMask: the output row's mask is known before the edges are —
      // load it first, so its latency overlaps the gather instead of following it
      T pm[MODE == kAggPostMask ? NCH : 1];
      uint4 pb[MODE == kAggPostMask && VEC == 4 && LPD >= 32 ? NCH : 1];
      if constexpr (MODE == kAggPostMask) {
        bool bits = false;
        if constexpr (VEC == 4 && LPD >= 32) {
          if (ax.bits_in) {  // (uniform) the keep mask as bits
            bits = true;
            const uint4* brow = reinterpret_cast<const uint4*>(ax.bits_in + (uint64_t)d * ax.ldb) +
                                (LPD == 64 ? (sl >> 5) : 0) * NCH;
#pragma unroll
            for (int c = 0; c < NCH; ++c) pb[c] = brow[c];
          }
        }
        if (!bits) {
          const T* mrow = reinterpret_cast<const T*>(ax.mx + (uint64_t)d * ax.ldm);
#pragma unroll
          for (int c = 0; c < NCH; ++c) {
            const uint32_t col = c0 + sl + c * LPD;
            pm[c] = col < nv ? mrow[col] : V::zero();
          }
        }
      }
      gather_edges<VEC, LPD, NCH, MAP, U, TIER, EM>(acc, cbeg, cend, c0, sl, idx, w, x, ldx, map,
                                                      nv, tier, ax, kAggPf >= 2, cpr, cpw);
      if constexpr (MODE == kAggPostMask) {  // same arithmetic as store_row's
        bool bits = false;
        if constexpr (VEC == 4 && LPD >= 32) {
          if (ax.bits_in) {
            bits = true;
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
              const uint32_t wq[4] = {pb[c].x, pb[c].y, pb[c].z, pb[c].w};
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                float& v = vcomp<VEC>(acc[c], q);
                v = ((wq[q] >> (sl & 31)) & 1u) ? v * ax.scale : 0.f;
              }
            }
          }
        }
        if (!bits) {
#pragma unroll
          for (int c = 0; c < NCH; ++c)
#pragma unroll
            for (int q = 0; q < VEC; ++q) {
              float& v = vcomp<VEC>(acc[c], q);
              v = vcomp<VEC>(pm[c], q) > 0.f ? v * ax.scale : 0.f;
            }
        }
      }
      store_row<VEC, LPD, NCH, MODE == kAggPostMask ? kAggPlain : EM>(acc, d, c0, sl, nv,
                                                                      last_valid, y, ldy, ax);
      if constexpr (CM) colmax_row(acc, c0, d);
    }
  }
  if constexpr (COOP) {
    __shared__ T part[GPB * LPD * NCH];
    __syncthreads();
    const uint32_t nl = n_long;  // the order rows are handled in does not matter
    for (uint32_t i = 0; i < nl; ++i) {
      const uint32_t d = long_rows[i];
      const uint32_t beg = off[d], end = off[d + 1], len = end - beg;
      const uint32_t pb = beg + (uint32_t)(((uint64_t)len * grp) / GPB);
      const uint32_t pe = beg + (uint32_t)(((uint64_t)len * (grp + 1)) / GPB);
      for (uint32_t c0 = 0; c0 < nv; c0 += LPD * NCH) {
        T acc[NCH];
#pragma unroll
        for (int c = 0; c < NCH; ++c) acc[c] = V::zero();
        gather_edges<VEC, LPD, NCH, MAP, U, TIER, EM>(acc, pb, pe, c0, sl, idx, w, x, ldx, map,
                                                        nv, tier, ax);
#pragma unroll
        for (int c = 0; c < NCH; ++c) part[(grp * NCH + c) * LPD + sl] = acc[c];
        __syncthreads();
        if (grp == 0) {
#pragma unroll
          for (int c = 0; c < NCH; ++c) {
            T s = part[c * LPD + sl];
            for (int g = 1; g < GPB; ++g) {
              const T q = part[(g * NCH + c) * LPD + sl];
#pragma unroll
              for (int k = 0; k < VEC; ++k) vcomp<VEC>(s, k) = vcomp<VEC>(s, k) + vcomp<VEC>(q, k);
            }
            acc[c] = s;
          }
          store_row<VEC, LPD, NCH, EM>(acc, d, c0, sl, nv, last_valid, y, ldy, ax);
          if constexpr (CM) colmax_row(acc, c0, d);
        }
        __syncthreads();
      }
    }
  }
  if constexpr (CM) {  // the block's maxima -> its row of the per-block buffer
    __syncthreads();
    uint32_t* row = ax.cm_out + (uint64_t)blockIdx.x * ncol;
    for (uint32_t c = threadIdx.x; c < ncol; c += kAggThreads) row[c] = smax[c];
  }
}

// g_in[idx[e], :] += w[e] * g_out[d, :]   (float atomics, order not deterministic)
template <int VEC, int LPD>
__global__ __launch_bounds__(kAggThreads) void k_spmm_scatter_atomic(
    const uint32_t* __restrict__ off, const uint32_t* __restrict__ idx,
    const float* __restrict__ w, const uint32_t* n_dev, uint32_t n_cap,
    const float* __restrict__ g, uint64_t ldg, uint32_t nv, float* __restrict__ gin,
    uint64_t ldgi) {
  using V = VT<VEC>;
  using T = typename V::T;
  const uint32_t n = n_dev ? min(*n_dev, n_cap) : n_cap;
  constexpr int GPB = kAggThreads / LPD;
  const int grp = threadIdx.x / LPD, sl = threadIdx.x % LPD;
  for (uint32_t d = blockIdx.x * GPB + grp; d < n; d += gridDim.x * GPB) {
    const uint32_t beg = off[d], end = off[d + 1];
    const T* grow = reinterpret_cast<const T*>(g + (uint64_t)d * ldg);
    for (uint32_t col = sl; col < nv; col += LPD) {
      const T gv = grow[col];
      for (uint32_t e = beg; e < end; ++e) {
        const float we = w ? w[e] : 1.0f;
        const T v = V::scale(gv, we);
        float* dst = gin + (uint64_t)idx[e] * ldgi + (uint64_t)col * VEC;
        const float* vs = reinterpret_cast<const float*>(&v);
#pragma unroll
        for (int k = 0; k < VEC; ++k) unsafeAtomicAdd(dst + k, vs[k]);
      }
    }
  }
}

// out[i,:] = table[index[i],:]; TIER: table is the HBM cache, rows whose
// tier.cmap entry is kNotCached come from the host-pinned tier.host
// (zero_copy_feature_move_gpu_cache + gather_feature_from_gpu_cache,
// cuda/ntsCUDATransferKernel.cuh:154-183, in one pass).
// STAGE (with TIER): only the rows that are not cached are copied, out row i
// = host row index[i]; cached rows of `out` are left untouched.
template <int VEC, int LPD, bool TIER, bool STAGE = false>
__global__ __launch_bounds__(kAggThreads) void k_gather_rows(const float* __restrict__ table,
                                                            uint64_t ldt,
                                                            const uint32_t* __restrict__ index,
                                                            const uint32_t* n_dev, uint32_t n_cap,
                                                            uint32_t nv, float* __restrict__ out,
                                                            uint64_t ldo, Tier tier) {
  using T = typename VT<VEC>::T;
  const uint32_t n = n_dev ? min(*n_dev, n_cap) : n_cap;
  constexpr int GPB = kAggThreads / LPD;
  const int grp = threadIdx.x / LPD, sl = threadIdx.x % LPD;
  for (uint32_t i = blockIdx.x * GPB + grp; i < n; i += gridDim.x * GPB) {
    const uint32_t g = index[i];
    const uint32_t slot = TIER ? tier.cmap[g] : g;
    if (STAGE && slot != kNotCached) continue;  // group-uniform
    const T* src = reinterpret_cast<const T*>(
        TIER && slot == kNotCached ? tier.host + (uint64_t)g * tier.ldh
                                   : table + (uint64_t)slot * ldt);
    T* dst = reinterpret_cast<T*>(out + (uint64_t)i * ldo);
    for (uint32_t c = sl; c < nv; c += LPD) dst[c] = src[c];
  }
}

// out = g ⊙ [x > 0] · scale — the backward of dropout(relu(.)) given its
// output x (relu zeroes and dropped elements are exactly the zeros of x)
__global__ void k_act_backward(const float4* __restrict__ g, const float4* __restrict__ x,
                               float4* __restrict__ out, uint64_t n4, float scale) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const float4 a = g[i], b = x[i];
    out[i] = make_float4(b.x > 0.f ? a.x * scale : 0.f, b.y > 0.f ? a.y * scale : 0.f,
                         b.z > 0.f ? a.z * scale : 0.f, b.w > 0.f ? a.w * scale : 0.f);
  }
}
__global__ void k_act_backward_2d(const float* __restrict__ g, uint64_t ldg,
                                  const float* __restrict__ x, uint64_t ldx, float* __restrict__ out,
                                  uint64_t ldo, uint32_t rows, uint32_t F, float scale) {
  const uint64_t n = (uint64_t)rows * F;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = i / F, c = i % F;
    out[r * ldo + c] = x[r * ldx + c] > 0.f ? g[r * ldg + c] * scale : 0.f;
  }
}

__global__ void k_gather_labels(const int64_t* __restrict__ labels,
                                const uint32_t* __restrict__ index, const uint32_t* n_dev,
                                uint32_t n_cap, int64_t* __restrict__ out) {
  const uint32_t n = n_dev ? min(*n_dev, n_cap) : n_cap;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    out[i] = labels[index[i]];
}

// Adam, element-wise in the exact operation order of the reference's torch
// expressions (core/NtsScheduler.hpp:863-880 and :937-945).
__global__ void k_adam(float* __restrict__ W, const float* __restrict__ G, float* __restrict__ M,
                       float* __restrict__ Vv, uint64_t n, float alpha, float beta1, float beta2,
                       float eps, float wd, float beta1_t, float beta2_t, int bias_correction) {
  const float omb1 = 1.0f - beta1, omb2 = 1.0f - beta2;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const float w = W[i];
    if (bias_correction) {
      // W_g = W_gradient + weight_decay * S
      const float wg = G[i] + wd * w;
      const float m = beta1 * M[i] + omb1 * wg;
      const float v = beta2 * Vv[i] + omb2 * (wg * wg);
      M[i] = m;
      Vv[i] = v;
      const float mt = m / (1.0f - beta1_t);
      const float vt = v / (1.0f - beta2_t);
      W[i] = w - (alpha * mt) / (sqrtf(vt) + eps);
    } else {
      // W_g = W * weight_decay + W.grad();  V = b2*V + (1-b2)*W_g*W_g
      const float wg = w * wd + G[i];
      const float m = beta1 * M[i] + omb1 * wg;
      const float v = beta2 * Vv[i] + (omb2 * wg) * wg;
      M[i] = m;
      Vv[i] = v;
      W[i] = w - (alpha * m) / (sqrtf(v) + eps);
    }
  }
}

#ifdef NTS_WITH_AGG_LDS  // negative result (2.5 TB/s of rows vs 6.7 in registers): variant builds only
// ---------------------------------------------------------------------------
// LDS-staged aggregation of 128- and 256-float rows (k_agg_lds): the same sums as
// k_spmm_gather (per output row, its edges in edge order, acc + x * w with
// contraction off — bit-identical for every row k_spmm_gather sums serially;
// the long CSR rows it splits into pieces are summed serially here, i.e. in
// MiniBatchFuseOp's order), but the neighbour rows are gathered into LDS by
// LDS DMA (global_load_lds_dwordx4, per-lane row bases) instead of registers:
// the gather form MI355X_MICROARCH.md measures at 7.4-8.6 TB/s against
// 5.5-5.8 for register gathers (§ Indexed rows: gather into LDS).
//
// Block = an id loader wave, a row loader wave and 4 consumer waves (8 groups
// of 32 lanes, one float4 of the row per lane, two for 256-float rows).
// Output rows are cut into parts of R <= kLdsR rows; block b takes parts b,
// b + G, ... and streams each part's edges in 16 KB stages (kLdsSE rows of 128
// floats, or 16 of 256) through a ring of kLdsNS LDS slots:
//   id loader   per stage: the stage's row ids, weights and its part's
//               offsets by LDS DMA into an id ring, 8 stages ahead (the id
//               loads' latency never sits in front of a row DMA)
//   row loader  per stage: once its ids are in and its slot is free (stage
//               k - NS consumed), 16 row DMAs; stage k-2 is marked full when
//               it lands — three stages in flight.  Each loader issues only
//               its own LDS DMAs, so its vmcnt counts are static.
//   groups      group g owns rows pR + g + 8 j of part p, sums each row's
//               edges that fall in the stage, stores a row when its last edge
//               is in, and carries a row that continues into the next stage.
// Output modes as k_spmm_gather's: plain, relu/dropout epilogue (kAggAct),
// post-mask (kAggPostMask), column maxima per part (kAggColmax; part p's
// maxima row = max over its rows of |rs(row) y|, the TN GEMM's operand
// scales), all written by store_row.
constexpr int kLdsR = 128;                       // output rows per part
constexpr int kLdsSE = 32;                       // edges (rows of x) per stage
constexpr int kLdsNS = 4;                        // ring slots
constexpr int kLdsCons = 4;                      // consumer waves
constexpr int kLdsThreads = kWave * (kLdsCons + 2);  // + row loader + id loader
constexpr int kLdsID = 12;                       // id-ring entries (stages ahead of the rows)
constexpr int kLdsIdAhead = 8;                   // id loads in flight (3 LDS DMAs each)
constexpr int kLdsRowB = 512;                    // 128 floats
constexpr int kLdsMaxParts = 64;                 // parts per block (lane-held bounds)
constexpr int kLdsCmSlots = 8;                   // colmax part ring
constexpr int kLdsF = 128;                       // floats per row

struct LdsAggShared {
  float4 rows[kLdsNS][kLdsSE * 32];              // 64 KB: 16 KB per slot (32 or 16 rows)
  uint32_t full[kLdsNS], freed[kLdsNS];          // row slots: stages landed / waves done
  // id ring (kLdsID stages, filled kLdsIdAhead stages ahead by the id loader's
  // LDS DMAs): per stage [0, 32) row ids, [32, 64) weights, [64, 192) the
  // part's offsets off[pR + j]; its descriptor and the part's edge end
  uint32_t ids[kLdsID][64 + kLdsR];
  uint4 meta[kLdsID];                            // {part, sb, se, flags | total << 8}
  uint32_t pend[kLdsID];                         // off[min(pR + R, n)]
  uint32_t ids_ready;                            // stages whose id entries landed
  uint32_t cm[kLdsCmSlots][kLdsF];               // kAggColmax: part maxima ring
  uint32_t cm_cnt[kLdsCmSlots];
};

// 16 (or 4) bytes per lane from `src` to LDS (wave-uniform base `lds`) + 16 (4)
// * lane.  Inline asm: the compiler neither counts these loads nor waits for
// them — the loader's s_waitcnt vmcnt(N) are the only waits, with N counted by
// hand (every load the loader issues is one of these).
__device__ __forceinline__ void glds16a(const void* src, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}
__device__ __forceinline__ void glds4a(const void* src, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)p;
}
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// bounded spin (a hang would take the GPU with it): gives up after ~2^22 polls
__device__ __forceinline__ void lds_wait_ge(const uint32_t* p, uint32_t v) {
  for (uint32_t it = 0; lds_ld(p) < v && it < (1u << 22); ++it) __builtin_amdgcn_s_sleep(1);
  asm volatile("" ::: "memory");
}

template <int MODE, int NCH>
__global__ __launch_bounds__(kLdsThreads) void k_agg_lds(
    const uint32_t* __restrict__ off, const uint32_t* __restrict__ idx,
    const float* __restrict__ w, const uint32_t* n_dev, uint32_t n_cap,
    const float* __restrict__ x, uint64_t ldx, float* __restrict__ y, uint64_t ldy, uint32_t R,
    AggExtra ax) {
  constexpr bool CM = MODE == kAggColmax;
  constexpr int EM = CM ? kAggPlain : MODE;
  constexpr int RF4 = 32 * NCH;         // float4s per row (128 or 256 floats)
  constexpr int SE = kLdsSE / NCH;      // rows per stage (16 KB)
  static_assert(!CM || NCH == 1, "column maxima: 128-float rows");
  __shared__ LdsAggShared sh;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t n = n_dev ? min(*n_dev, n_cap) : n_cap;
  const uint32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t parts = (n + R - 1) / R;
  const uint32_t parts_cap = (n_cap + R - 1) / R;
  const uint32_t my_parts = parts > b ? (parts - b + G - 1) / G : 0u;  // <= kLdsMaxParts (host)
  for (int i = tid; i < kLdsNS; i += kLdsThreads) {
    sh.full[i] = 0u;
    sh.freed[i] = 0u;
  }
  if (tid == 0) sh.ids_ready = 0u;
  if (CM) {
    for (int i = tid; i < kLdsCmSlots * kLdsF; i += kLdsThreads) (&sh.cm[0][0])[i] = 0u;
    for (int i = tid; i < kLdsCmSlots; i += kLdsThreads) sh.cm_cnt[i] = 0u;
    // parts past the live rows: zero maxima (as k_spmm_gather's per-block rows)
    for (uint32_t p = parts + (b + G - parts % G) % G; p < parts_cap; p += G)
      for (int c = tid; c < kLdsF; c += kLdsThreads) ax.cm_out[(uint64_t)p * kLdsF + c] = 0u;
  }
  __syncthreads();
  if (my_parts == 0) return;

  // stage k consumed by every consumer wave
  auto consumed = [&](uint32_t k) {
    return lds_ld(&sh.freed[k % kLdsNS]) >= (uint32_t)kLdsCons * (k / kLdsNS + 1);
  };
  if (wv == kLdsCons + 1) {
    // ---------------- id loader ----------------
    // lane i holds part i's edge bounds and stage count; per stage three LDS
    // DMAs (ids | weights, the part's offsets) into id-ring entry k % kLdsID,
    // kLdsIdAhead stages in flight; entry k is refilled once stage k - kLdsID
    // is consumed.  (The only vector-memory ops of this wave: counted waits.)
    uint32_t pe0 = 0, pe1 = 0, nst = 0;
    if ((uint32_t)lane < my_parts) {
      const uint32_t p = b + (uint32_t)lane * G;
      pe0 = off[(uint64_t)p * R];
      pe1 = off[min((uint64_t)(p + 1) * R, (uint64_t)n)];
      nst = max(1u, (pe1 - pe0 + SE - 1) / SE);
    }
    uint32_t total = nst;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o);
    const uint32_t lids = lds_u32(&sh.ids[0][0]);
    uint32_t cur_i = 0, cur_s = 0;  // cursor: part, stage within the part
    for (uint32_t k = 0; k < total + kLdsIdAhead - 1; ++k) {
      if (k < total) {
        const int q = (int)(k % kLdsID);
        if (k >= (uint32_t)kLdsID)
          for (uint32_t it = 0; !consumed(k - kLdsID) && it < (1u << 22); ++it) __builtin_amdgcn_s_sleep(1);
        const uint32_t i = cur_i;
        const uint32_t e0 = __shfl(pe0, (int)i), e1 = __shfl(pe1, (int)i), ns = __shfl(nst, (int)i);
        const uint32_t sb = e0 + cur_s * SE, se = min(sb + SE, e1);
        if (lane == 0) {
          sh.meta[q] = make_uint4(b + i * G, sb, se,
                                  (cur_s == 0 ? 1u : 0u) | (cur_s + 1 == ns ? 2u : 0u) | (total << 8));
          sh.pend[q] = e1;
        }
        if (++cur_s == ns) {
          cur_s = 0;
          ++cur_i;
        }
        const uint32_t e = sb + (uint32_t)(lane & 31);
        const uint32_t ec = e < se ? e : sb < se ? sb : 0u;
        const void* src = lane < 32 || !w ? (const void*)(idx + ec) : (const void*)(w + ec);
        glds4a(src, lids + (uint32_t)(q * (64 + kLdsR) * 4));
        const uint64_t p = b + i * G;
        glds4a(off + min(p * R + lane, (uint64_t)n), lids + (uint32_t)((q * (64 + kLdsR) + 64) * 4));
        glds4a(off + min(p * R + 64 + lane, (uint64_t)n), lids + (uint32_t)((q * (64 + kLdsR) + 128) * 4));
      }
      // entry k - (kLdsIdAhead - 1) landed: younger are the 3 (kLdsIdAhead - 1)
      // loads of the stages after it (fewer at the end: then wait for all)
      if (k + 1 >= (uint32_t)kLdsIdAhead) {
        if (k < total) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(3 * (kLdsIdAhead - 1)) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) lds_st(&sh.ids_ready, min(k + 2 - kLdsIdAhead, total));
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) lds_st(&sh.ids_ready, total);
    return;
  }
  if (wv == kLdsCons) {
    // ---------------- row loader ----------------
    // per stage 16 LDS DMAs of 1 KB into row slot k % kLdsNS once its ids are
    // in and stage k - kLdsNS is consumed; stage k-2 is marked full when it
    // lands (younger: the 32 DMAs of k-1 and k), three stages in flight
    const uint32_t lrows = lds_u32(&sh.rows[0][0]);
    uint32_t total = 1;
    for (uint32_t k = 0; k < total; ++k) {
      const uint32_t slot = k % kLdsNS;
      const int q = (int)(k % kLdsID);
      lds_wait_ge(&sh.ids_ready, k + 1);
      if (k >= (uint32_t)kLdsNS) lds_wait_ge(&sh.freed[slot], (uint32_t)kLdsCons * (k / kLdsNS));
      const uint4 mt = sh.meta[q];
      total = mt.w >> 8;
      const uint32_t nrow = mt.z - mt.y;
      const uint32_t id = sh.ids[q][lane & 31];
      const uint32_t id0 = __shfl(id, 0);
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) {
        const int fl4 = 64 * jj + lane, r = fl4 / RF4, c16 = fl4 % RF4;
        uint32_t rid = __shfl(id, r);
        rid = (uint32_t)r < nrow ? rid : (nrow ? id0 : 0u);
        const char* src = reinterpret_cast<const char*>(x + (uint64_t)rid * ldx) + 16 * c16;
        glds16a(src, lrows + (uint32_t)(slot * kLdsSE * kLdsRowB + 1024 * jj));
      }
      if (k >= 2) {
        asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
        lds_st(&sh.full[(k - 2) % kLdsNS], k - 1);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (uint32_t k = total > 2 ? total - 2 : 0; k < total; ++k) lds_st(&sh.full[k % kLdsNS], k + 1);
    return;
  }

  // ---------------- consumer waves: 8 groups of 32 lanes ----------------
  const int g = 2 * wv + (lane >> 5), l = lane & 31;
  float4 acc[NCH];
  float4 cmx = make_float4(0.f, 0.f, 0.f, 0.f);
  uint32_t j = 0, pcount = 0;                    // local row of the part, rows in the part
  uint32_t e_beg = 0, e_end = 0, part = 0, part_ord = 0;
  // per-row operands known before the row's edges (kAggPostMask: the row's
  // mask, kAggColmax: its scale), loaded one row ahead: a global load used
  // right away would make the compiler wait for every older store as well
  float4 pm[NCH], pm_n[NCH];
  float rsd = 1.f, rsd_n = 1.f;
  auto zero = [&]() {
#pragma unroll
    for (int c = 0; c < NCH; ++c) acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  };
  zero();
  auto row_ctx = [&](uint32_t d) {  // -> the "next" registers
    if constexpr (MODE == kAggPostMask)
#pragma unroll
      for (int c = 0; c < NCH; ++c)
        pm_n[c] = *reinterpret_cast<const float4*>(ax.mx + (uint64_t)d * ax.ldm + 4 * (l + 32 * c));
    if constexpr (CM) rsd_n = ax.cm_rs ? ax.cm_rs[ax.cm_map ? ax.cm_map[d] : d] : 1.f;
  };
  auto take_ctx = [&]() {
#pragma unroll
    for (int c = 0; c < NCH; ++c) pm[c] = pm_n[c];
    rsd = rsd_n;
  };
  uint32_t total = 1;
  for (uint32_t k = 0; k < total; ++k) {
    const uint32_t slot = k % kLdsNS;
    const int q = (int)(k % kLdsID);
    lds_wait_ge(&sh.full[slot], k + 1);
    const uint4 mt = sh.meta[q];
    total = mt.w >> 8;
    const uint32_t sb = mt.y, se = mt.z, fl = mt.w & 255u;
    if (fl & 1u) {  // first stage of part mt.x: this group's first row
      part = mt.x;
      pcount = min(R, n - part * R);
      j = (uint32_t)g;
      if (j < pcount) {
        e_beg = sh.ids[q][64 + j];
        e_end = j + 1 < pcount ? sh.ids[q][64 + j + 1] : sh.pend[q];
        row_ctx(part * R + j);
        take_ctx();
        if (j + 8 < pcount) row_ctx(part * R + j + 8);
      }
      zero();
      cmx = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float4* srow = &sh.rows[slot][l];
    const float* sw = reinterpret_cast<const float*>(&sh.ids[q][32]);
    // rows whose edges start in this stage (a row without edges at the
    // stage's end included): sum their edges here, store the complete ones
    while (j < pcount && (e_beg < se || (e_beg == e_end && e_beg <= se))) {
      uint32_t e = max(e_beg, sb);
      const uint32_t hi = min(e_end, se);
      constexpr int UL = 8 / NCH;  // rows of x read ahead of their adds
      for (; e + UL <= hi; e += UL) {
        float4 xv[UL][NCH];
        float wv4[UL];
#pragma unroll
        for (int u = 0; u < UL; ++u) {
#pragma unroll
          for (int c = 0; c < NCH; ++c) xv[u][c] = srow[(e + u - sb) * RF4 + 32 * c];
          wv4[u] = w ? sw[e + u - sb] : 1.f;
        }
#pragma unroll
        for (int u = 0; u < UL; ++u)
#pragma unroll
          for (int c = 0; c < NCH; ++c) acc[c] = VT<4>::madd(acc[c], xv[u][c], wv4[u]);
      }
      for (; e < hi; ++e)
#pragma unroll
        for (int c = 0; c < NCH; ++c)
          acc[c] = VT<4>::madd(acc[c], srow[(e - sb) * RF4 + 32 * c], w ? sw[e - sb] : 1.f);
      if (e_end > se) break;  // continues in the next stage
      const uint32_t d = part * R + j;
      if constexpr (MODE == kAggPostMask)
#pragma unroll
        for (int c = 0; c < NCH; ++c)
          acc[c] = make_float4(pm[c].x > 0.f ? acc[c].x * ax.scale : 0.f, pm[c].y > 0.f ? acc[c].y * ax.scale : 0.f,
                               pm[c].z > 0.f ? acc[c].z * ax.scale : 0.f, pm[c].w > 0.f ? acc[c].w * ax.scale : 0.f);
      store_row<4, 32, NCH, MODE == kAggPostMask ? kAggPlain : EM>(acc, d, 0, l, RF4, 4, y, ldy, ax);
      if constexpr (CM) {
        cmx.x = fmaxf(cmx.x, fabsf(acc[0].x * rsd));
        cmx.y = fmaxf(cmx.y, fabsf(acc[0].y * rsd));
        cmx.z = fmaxf(cmx.z, fabsf(acc[0].z * rsd));
        cmx.w = fmaxf(cmx.w, fabsf(acc[0].w * rsd));
      }
      zero();
      j += 8;
      if (j < pcount) {
        e_beg = sh.ids[q][64 + j];
        e_end = j + 1 < pcount ? sh.ids[q][64 + j + 1] : sh.pend[q];
        take_ctx();
        if (j + 8 < pcount) row_ctx(part * R + j + 8);
      }
    }
    if (CM && (fl & 2u)) {
      // part done for this group: fold its maxima into the part's ring slot;
      // the eighth group to arrive writes the part's row and clears the slot
      // (a group can be at most a few parts ahead: every stage of a part is
      // consumed by every wave before the ring moves NS stages on)
      const uint32_t cs = part_ord % kLdsCmSlots;
      atomicMax(&sh.cm[cs][4 * l + 0], __float_as_uint(cmx.x));
      atomicMax(&sh.cm[cs][4 * l + 1], __float_as_uint(cmx.y));
      atomicMax(&sh.cm[cs][4 * l + 2], __float_as_uint(cmx.z));
      atomicMax(&sh.cm[cs][4 * l + 3], __float_as_uint(cmx.w));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      uint32_t arrived = 0;
      if (l == 0) arrived = atomicAdd(&sh.cm_cnt[cs], 1u);
      arrived = __shfl(arrived, lane & 32);
      if (arrived == 7u) {
        const uint4 m4 = *reinterpret_cast<const uint4*>(&sh.cm[cs][4 * l]);
        *reinterpret_cast<uint4*>(ax.cm_out + (uint64_t)part * kLdsF + 4 * l) = m4;
        *reinterpret_cast<uint4*>(&sh.cm[cs][4 * l]) = make_uint4(0u, 0u, 0u, 0u);
        if (l == 0) sh.cm_cnt[cs] = 0u;
      }
    }
    if (fl & 2u) ++part_ord;
    // this wave is done reading the slot
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0)
      __hip_atomic_fetch_add(&sh.freed[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}
#endif  // NTS_WITH_AGG_LDS

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------
static int pick_vec(uint32_t F, uint64_t ld1, uint64_t ld2, const void* p1, const void* p2) {
  auto al = [](const void* p, uintptr_t a) { return ((uintptr_t)p % a) == 0; };
  if (F % 4 == 0 && ld1 % 4 == 0 && ld2 % 4 == 0 && al(p1, 16) && al(p2, 16)) return 4;
  if (F % 2 == 0 && ld1 % 2 == 0 && ld2 % 2 == 0 && al(p1, 8) && al(p2, 8)) return 2;
  return 1;
}

struct Shape {
  int lpd, nch;
};
// (128-float rows on 16-lane groups of two float4 per lane — four rows per
// wave instead of two — measured: hop-0 backward 42.5 vs 44.8 us, the bottom
// CSR backward 125-127 vs 122, C2 0.824 vs 0.807 ms/step; not kept)
static Shape pick_shape(uint32_t nv) {
  if (nv <= 8) return {8, 1};
  if (nv <= 16) return {16, 1};
  if (nv <= 32) return {32, 1};
  if (nv <= 64) return {64, 1};
  uint32_t nch = (nv + 63) / 64;
  return {64, (int)std::min<uint32_t>(nch, 8)};
}

// the vector width launch_gather picks for a local-row gather (no tier, no
// mask operand): rows padded to a 16-byte multiple take float4 loads, the
// partial last vector reading pitch padding and storing only its valid floats
static int plain_vec(uint32_t F, uint64_t ldx, uint64_t ldy, const void* x, const void* y) {
  int vec = pick_vec(F, ldx, ldy, x, y);
  const uint32_t F4 = (F + 3) / 4 * 4;
  if (vec < 4 && F4 <= ldx && F4 <= ldy && ldx % 4 == 0 && ldy % 4 == 0 &&
      (uintptr_t)x % 16 == 0 && (uintptr_t)y % 16 == 0)
    vec = 4;
  return vec;
}

// compile-time A/B (make variant VFLAGS=-DNTS_GATHER_U=4): 4 rows in flight
// for the mid-width rows instead of 5
#ifndef NTS_GATHER_U
#define NTS_GATHER_U 0
#endif
constexpr int gather_u_env() { return NTS_GATHER_U; }
// rows in flight for the post-mask CSR gather (the hop above a transform-first
// bottom layer: ~2 edges per row at C2); 0: gather_u's (compile-time A/B)
#ifndef NTS_AGG_PM_U
#define NTS_AGG_PM_U 0
#endif
constexpr int kAggPmU = NTS_AGG_PM_U;
constexpr int gather_u(int floats_per_lane) {
  return floats_per_lane <= 4 ? 8 : floats_per_lane <= 12 ? 5 : 4;
}

template <int VEC, bool MAP, bool TIER, int MODE, bool COOP>
static int launch_gather_vec(hipStream_t st, uint32_t grid, uint32_t last_valid, Shape s,
                             const uint32_t* off,
                             const uint32_t* idx, const float* w, const uint32_t* n_dev,
                             uint32_t n_cap, const float* x, uint64_t ldx, const uint32_t* map,
                             uint32_t nv, float* y, uint64_t ldy, Tier tier, const AggExtra& ax) {
// rows in flight per lane group: 8 for narrow rows, 5 for mid-width rows
// (F ~ 600: 3 float4 per lane; fanout 10/25 -> full batches), 4 for the
// widest (register budget); -DNTS_GATHER_U=4 forces 4 for the mid-width rows
#define NTS_G(LPD, NCH)                                                                     \
  do {                                                                                      \
    constexpr int u = (MODE == kAggPostMask && kAggPmU > 0) ? kAggPmU : gather_u(VEC * NCH); \
    if (u == 5 && gather_u_env() == 4)                                                      \
      hipLaunchKernelGGL((k_spmm_gather<VEC, LPD, NCH, MAP, 4, TIER, MODE, COOP>), dim3(grid), \
                         dim3(kAggThreads), 0, st, off, idx, w, n_dev, n_cap, x, ldx, map, \
                         nv, y, ldy, last_valid, tier, ax);                                 \
    else                                                                                    \
      hipLaunchKernelGGL((k_spmm_gather<VEC, LPD, NCH, MAP, u, TIER, MODE, COOP>), dim3(grid), \
                         dim3(kAggThreads), 0, st, off, idx, w, n_dev, n_cap, x, ldx, map, \
                         nv, y, ldy, last_valid, tier, ax);                                 \
  } while (0)
  if (s.lpd == 8) NTS_G(8, 1);
  else if (s.lpd == 16) NTS_G(16, 1);
  else if (s.lpd == 32) NTS_G(32, 1);
  else switch (s.nch) {
      case 1: NTS_G(64, 1); break;
      case 2: NTS_G(64, 2); break;
      case 3: NTS_G(64, 3); break;
      case 4: NTS_G(64, 4); break;
      case 5: NTS_G(64, 5); break;
      case 6: NTS_G(64, 6); break;
      case 7: NTS_G(64, 7); break;
      default: NTS_G(64, 8); break;
    }
#undef NTS_G
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

// the LDS-staged gather (k_agg_lds) takes 128-float rows gathered by local id
// (no row map, no host tier, no per-edge mask rows) in 16-byte vectors; it
// exists only in variant builds (make variant V=agglds VFLAGS=-DNTS_WITH_AGG_LDS)
#ifdef NTS_WITH_AGG_LDS
template <bool MAP, bool TIER, int MODE>
static bool agg_lds_applies(int vec, uint32_t F) {
  return !MAP && !TIER && MODE != kAggMask && vec == 4 &&
         (F == (uint32_t)kLdsF || (F == 2u * kLdsF && MODE != kAggColmax));
}
#endif

template <bool MAP, bool TIER = false, int MODE = kAggPlain, bool COOP = false>
static int launch_gather(hipStream_t st, const uint32_t* off, const uint32_t* idx,
                         const float* w, const uint32_t* n_dev, uint32_t n_cap, const float* x,
                         uint64_t ldx, const uint32_t* map, uint32_t F, float* y, uint64_t ldy,
                         Tier tier = Tier{nullptr, nullptr, 0, 0}, AggExtra ax = AggExtra(),
                         uint32_t expect_grid = 0) {
  int vec = pick_vec(F, ldx, ldy, x, y);
  if (TIER) vec = std::min(vec, pick_vec(F, tier.ldh, ldx, tier.host, x));
  if (MODE == kAggMask || (MODE == kAggPostMask && !ax.bits_in))
    vec = std::min(vec, pick_vec(F, ax.ldm, ldx, ax.mx, x));
  // rows padded to a 16-byte multiple (the 128-byte feature / output pitch):
  // float4 loads, the partial last vector reads pitch padding and stores only
  // its valid floats
  const uint32_t F4 = (F + 3) / 4 * 4;
  if ((MODE == kAggPlain || MODE == kAggColmax) && vec < 4 && F4 <= ldx && F4 <= ldy && ldx % 4 == 0 && ldy % 4 == 0 &&
      (uintptr_t)x % 16 == 0 && (uintptr_t)y % 16 == 0 &&
      (!TIER || (F4 <= tier.ldh && tier.ldh % 4 == 0 && (uintptr_t)tier.host % 16 == 0)))
    vec = 4;
  const uint32_t nv = (F + vec - 1) / vec;
  const uint32_t last_valid = F - (nv - 1) * vec;
#ifdef NTS_WITH_AGG_LDS
  if (agg_lds_applies<MAP, TIER, MODE>(vec, F)) {
    // 128-float rows: the LDS-staged gather (k_agg_lds)
    // rows per part: kLdsR for the column maxima (the parts the TN GEMM reads,
    // nts_hip_csr_bwd_colmax_rows_per_part), else smaller parts for small
    // layers (~1,000 parts: enough blocks for the chip)
    uint32_t R = (uint32_t)kLdsR;
    if (MODE != kAggColmax)
      while (R > 8 && (uint64_t)R * 1024 > n_cap) R /= 2;
    const uint32_t parts_cap = ceil_div(n_cap, R);
    const uint32_t grid = std::max(std::min(parts_cap, 1024u), ceil_div(parts_cap, kLdsMaxParts));
    if (grid == 0) return NTS_OK;
    if constexpr (MODE == kAggColmax)
      hipLaunchKernelGGL((k_agg_lds<MODE, 1>), dim3(grid), dim3(kLdsThreads), 0, st, off, idx, w, n_dev,
                         n_cap, x, ldx, y, ldy, R, ax);
    else if (F == (uint32_t)kLdsF)
      hipLaunchKernelGGL((k_agg_lds<MODE, 1>), dim3(grid), dim3(kLdsThreads), 0, st, off, idx, w, n_dev,
                         n_cap, x, ldx, y, ldy, R, ax);
    else
      hipLaunchKernelGGL((k_agg_lds<MODE, 2>), dim3(grid), dim3(kLdsThreads), 0, st, off, idx, w, n_dev,
                         n_cap, x, ldx, y, ldy, R, ax);
    NTS_LAUNCH_CHECK();
    return NTS_OK;
  }
#endif
  const Shape s = pick_shape(nv);
  const uint32_t gpb = kAggThreads / s.lpd;
  // one destination per lane group: every row's dependent loads (offsets ->
  // ids -> rows) are in flight at once; a grid-stride cap (NTS_AGG_GRID)
  // serialises rows per group and measured slower (C2: 1.069 vs 1.097 ms per
  // step at a 4096-block cap; the narrow CSR backward 50 -> ~25 us;
  // compile-time A/B: -DNTS_AGG_GRID=<blocks>)
#ifndef NTS_AGG_GRID
#define NTS_AGG_GRID (1u << 24)
#endif
  constexpr uint32_t cap = NTS_AGG_GRID;
  // the post-mask CSR gather (the hop above a transform-first bottom layer,
  // ~2 edges per row at C2) with a few rows per group instead of one
  // (compile-time A/B, -DNTS_AGG_PM_GRID=<blocks>): 44.7 / 44.6 / 51.7 us at
  // 4096 / 8192 / 2048 blocks against 44.9 at one row per group
  // (scripts/ab/r05_au.sh) — bound by its bytes, not by block lifetimes
#ifndef NTS_AGG_PM_GRID
#define NTS_AGG_PM_GRID (1u << 24)
#endif
  constexpr uint32_t pm_cap = MODE == kAggPostMask ? NTS_AGG_PM_GRID : (1u << 24);
  // COOP: at most kCoopRows rows per lane group (the colmax parts: one)
  const uint32_t grid =
      std::max(1u, COOP ? std::max(ceil_div(n_cap, gpb * kCoopRows), std::min(ceil_div(n_cap, gpb), pm_cap))
                        : std::min(ceil_div(n_cap, gpb), cap));
  // kAggColmax: the per-block buffer was sized for this grid
  NTS_CHECK_ARG(expect_grid == 0 || expect_grid == grid, "aggregation grid != the sized one");
  if (vec == 4)
    return launch_gather_vec<4, MAP, TIER, MODE, COOP>(st, grid, last_valid, s, off, idx, w, n_dev,
                                                 n_cap, x, ldx, map, nv, y, ldy, tier, ax);
  if (vec == 2)
    return launch_gather_vec<2, MAP, TIER, MODE, COOP>(st, grid, last_valid, s, off, idx, w, n_dev,
                                                 n_cap, x, ldx, map, nv, y, ldy, tier, ax);
  return launch_gather_vec<1, MAP, TIER, MODE, COOP>(st, grid, last_valid, s, off, idx, w, n_dev, n_cap,
                                               x, ldx, map, nv, y, ldy, tier, ax);
}


}  // namespace nts_hip

using namespace nts_hip;

extern "C" {

int nts_hip_spmm_csc_fwd(nts_hip_ctx* ctx, const uint32_t* column_offset,
                         const uint32_t* row_indices, const float* weight, const uint32_t* v,
                         uint32_t v_cap, const float* x, uint64_t ldx,
                         const uint32_t* x_row_map, uint32_t feature_size, float* y,
                         uint64_t ldy) {
  NTS_CHECK_ARG(ctx && column_offset && row_indices && x && y, "NULL argument");
  NTS_CHECK_ARG(ldx >= feature_size && ldy >= feature_size, "leading dimension < feature_size");
  if (v_cap == 0 || feature_size == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  if (x_row_map)
    return launch_gather<true>(ctx->stream, column_offset, row_indices, weight, v, v_cap, x, ldx,
                               x_row_map, feature_size, y, ldy);
  return launch_gather<false>(ctx->stream, column_offset, row_indices, weight, v, v_cap, x, ldx,
                              nullptr, feature_size, y, ldy);
}

int nts_hip_spmm_csr_bwd(nts_hip_ctx* ctx, const uint32_t* row_offset,
                         const uint32_t* column_indices, const float* weight_backward,
                         const uint32_t* s, uint32_t s_cap, const float* g_out, uint64_t ld_gout,
                         uint32_t feature_size, float* g_in, uint64_t ld_gin) {
  NTS_CHECK_ARG(ctx && row_offset && column_indices && g_out && g_in, "NULL argument");
  NTS_CHECK_ARG(ld_gout >= feature_size && ld_gin >= feature_size,
                "leading dimension < feature_size");
  if (s_cap == 0 || feature_size == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  return launch_gather<false, false, kAggPlain, true>(ctx->stream, row_offset, column_indices,
                                                      weight_backward, s, s_cap,
                              g_out, ld_gout, nullptr, feature_size, g_in, ld_gin);
}

uint32_t nts_hip_csr_bwd_colmax_rows_per_part(uint32_t feature_size) {
  if (feature_size == 0) return 0;
  // (the colmax gather always runs on float4 rows: vec 4)
#ifdef NTS_WITH_AGG_LDS
  if (agg_lds_applies<false, false, kAggColmax>(4, feature_size)) return (uint32_t)kLdsR;
#endif
  return (uint32_t)(kAggThreads / pick_shape((feature_size + 3) / 4).lpd);
}

int nts_hip_spmm_csr_bwd_colmax(nts_hip_ctx* ctx, const uint32_t* row_offset,
                                const uint32_t* column_indices, const float* weight_backward,
                                const uint32_t* s, uint32_t s_cap, const float* g_out,
                                uint64_t ld_gout, uint32_t feature_size, float* g_in,
                                uint64_t ld_gin, uint32_t* part_max, const float* row_scale,
                                const uint32_t* row_map) {
  NTS_CHECK_ARG(ctx && row_offset && column_indices && g_out && g_in && part_max, "NULL argument");
  NTS_CHECK_ARG(row_scale || !row_map, "row_map without row_scale");
  NTS_CHECK_ARG(ld_gout >= feature_size && ld_gin >= feature_size,
                "leading dimension < feature_size");
  NTS_CHECK_ARG(feature_size <= 512, "column maxima: at most 512 columns");
  if (s_cap == 0 || feature_size == 0) return NTS_OK;
  // the parts follow the COOP grid (one output row per lane group): the
  // float4 row shape nts_hip_csr_bwd_colmax_rows_per_part assumes
  NTS_CHECK_ARG(plain_vec(feature_size, ld_gout, ld_gin, g_out, g_in) == 4,
                "column maxima: 16-byte aligned rows with ld % 4 == 0");
  const uint32_t rpp = nts_hip_csr_bwd_colmax_rows_per_part(feature_size);
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  AggExtra ax;
  ax.cm_out = part_max;
  ax.cm_rs = row_scale;
  ax.cm_map = row_map;
  return launch_gather<false, false, kAggColmax, true>(ctx->stream, row_offset, column_indices,
                                                       weight_backward, s, s_cap, g_out, ld_gout,
                                                       nullptr, feature_size, g_in, ld_gin,
                                                       Tier{nullptr, nullptr, 0, 0}, ax,
                                                       ceil_div(s_cap, rpp));
}

int nts_hip_spmm_csc_fwd_act(nts_hip_ctx* ctx, const uint32_t* column_offset,
                             const uint32_t* row_indices, const float* weight, const uint32_t* v,
                             uint32_t v_cap, const float* x, uint64_t ldx, uint32_t feature_size,
                             float* y, uint64_t ldy, float p, uint64_t seed, uint64_t offset) {
  NTS_CHECK_ARG(ctx && column_offset && row_indices && x && y, "NULL argument");
  NTS_CHECK_ARG(ldx >= feature_size && ldy >= feature_size, "leading dimension < feature_size");
  NTS_CHECK_ARG(p >= 0.f && p <= 1.f, "dropout probability must be in [0, 1]");
  if (v_cap == 0 || feature_size == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  AggExtra ax;
  ax.keep_threshold = dropout_threshold(p);
  ax.scale = p >= 1.f ? 0.f : 1.0f / (1.0f - p);  // as the GEMM epilogue
  ax.seed = seed;
  ax.offset = offset;
  return launch_gather<false, false, kAggAct>(ctx->stream, column_offset, row_indices, weight, v,
                                              v_cap, x, ldx, nullptr, feature_size, y, ldy,
                                              Tier{nullptr, nullptr, 0, 0}, ax);
}

int nts_hip_spmm_csr_bwd_masked(nts_hip_ctx* ctx, const uint32_t* row_offset,
                                const uint32_t* column_indices, const float* weight_backward,
                                const uint32_t* s, uint32_t s_cap, const float* g_out,
                                uint64_t ld_gout, const float* x_act, uint64_t ld_act, float scale,
                                uint32_t feature_size, float* g_in, uint64_t ld_gin) {
  NTS_CHECK_ARG(ctx && row_offset && column_indices && g_out && x_act && g_in, "NULL argument");
  NTS_CHECK_ARG(ld_gout >= feature_size && ld_act >= feature_size && ld_gin >= feature_size,
                "leading dimension < feature_size");
  if (s_cap == 0 || feature_size == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  AggExtra ax;
  ax.mx = x_act;
  ax.ldm = ld_act;
  ax.scale = scale;
  return launch_gather<false, false, kAggMask, true>(ctx->stream, row_offset, column_indices,
                                               weight_backward, s, s_cap, g_out, ld_gout, nullptr,
                                               feature_size, g_in, ld_gin,
                                               Tier{nullptr, nullptr, 0, 0}, ax);
}

int nts_hip_spmm_csr_bwd_postmask(nts_hip_ctx* ctx, const uint32_t* row_offset,
                                  const uint32_t* column_indices, const float* weight_backward,
                                  const uint32_t* s, uint32_t s_cap, const float* g_out,
                                  uint64_t ld_gout, const float* x_act, uint64_t ld_act, float scale,
                                  uint32_t feature_size, float* g_in, uint64_t ld_gin) {
  NTS_CHECK_ARG(ctx && row_offset && column_indices && g_out && x_act && g_in, "NULL argument");
  NTS_CHECK_ARG(ld_gout >= feature_size && ld_act >= feature_size && ld_gin >= feature_size,
                "leading dimension < feature_size");
  if (s_cap == 0 || feature_size == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  AggExtra ax;
  ax.mx = x_act;
  ax.ldm = ld_act;
  ax.scale = scale;
  return launch_gather<false, false, kAggPostMask, true>(ctx->stream, row_offset, column_indices,
                                                         weight_backward, s, s_cap, g_out, ld_gout,
                                                         nullptr, feature_size, g_in, ld_gin,
                                                         Tier{nullptr, nullptr, 0, 0}, ax);
}

uint32_t nts_hip_act_bits_words(uint32_t feature_size) {
  if (feature_size == 0 || feature_size % 4) return 0;
  const uint32_t nv = feature_size / 4;
  const Shape s = pick_shape(nv);
  if (s.lpd < 32 || nv > (uint32_t)(s.lpd * s.nch)) return 0;  // float4 rows of one chunk
  return (uint32_t)(s.lpd / 32) * (uint32_t)s.nch * 4u;  // act_bits_words<LPD, NCH>()
}

int nts_hip_spmm_csc_fwd_act_bits(nts_hip_ctx* ctx, const uint32_t* column_offset,
                                  const uint32_t* row_indices, const float* weight,
                                  const uint32_t* v, uint32_t v_cap, const float* x, uint64_t ldx,
                                  uint32_t feature_size, float* y, uint64_t ldy, float p,
                                  uint64_t seed, uint64_t offset, uint32_t* mask_bits) {
  NTS_CHECK_ARG(ctx && column_offset && row_indices && x && y && mask_bits, "NULL argument");
  NTS_CHECK_ARG(ldx >= feature_size && ldy >= feature_size, "leading dimension < feature_size");
  NTS_CHECK_ARG(p >= 0.f && p <= 1.f, "dropout probability must be in [0, 1]");
  const uint32_t words = nts_hip_act_bits_words(feature_size);
  if (words == 0) return NTS_ERR_UNSUPPORTED;
  NTS_CHECK_ARG(pick_vec(feature_size, ldx, ldy, x, y) == 4 && (uintptr_t)mask_bits % 16 == 0,
                "mask bits: 16-byte aligned rows with ld % 4 == 0");
  if (v_cap == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  AggExtra ax;
  ax.keep_threshold = dropout_threshold(p);
  ax.scale = p >= 1.f ? 0.f : 1.0f / (1.0f - p);
  ax.seed = seed;
  ax.offset = offset;
  ax.bits_out = mask_bits;
  ax.ldb = words;
  return launch_gather<false, false, kAggAct>(ctx->stream, column_offset, row_indices, weight, v,
                                              v_cap, x, ldx, nullptr, feature_size, y, ldy,
                                              Tier{nullptr, nullptr, 0, 0}, ax);
}

int nts_hip_spmm_csr_bwd_postmask_bits(nts_hip_ctx* ctx, const uint32_t* row_offset,
                                       const uint32_t* column_indices,
                                       const float* weight_backward, const uint32_t* s,
                                       uint32_t s_cap, const float* g_out, uint64_t ld_gout,
                                       const uint32_t* mask_bits, float scale,
                                       uint32_t feature_size, float* g_in, uint64_t ld_gin) {
  NTS_CHECK_ARG(ctx && row_offset && column_indices && g_out && mask_bits && g_in, "NULL argument");
  NTS_CHECK_ARG(ld_gout >= feature_size && ld_gin >= feature_size,
                "leading dimension < feature_size");
  const uint32_t words = nts_hip_act_bits_words(feature_size);
  if (words == 0) return NTS_ERR_UNSUPPORTED;
  NTS_CHECK_ARG(pick_vec(feature_size, ld_gout, ld_gin, g_out, g_in) == 4 &&
                    (uintptr_t)mask_bits % 16 == 0,
                "mask bits: 16-byte aligned rows with ld % 4 == 0");
  if (s_cap == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  AggExtra ax;
  ax.bits_in = mask_bits;
  ax.ldb = words;
  ax.scale = scale;
  return launch_gather<false, false, kAggPostMask, true>(ctx->stream, row_offset, column_indices,
                                                         weight_backward, s, s_cap, g_out, ld_gout,
                                                         nullptr, feature_size, g_in, ld_gin,
                                                         Tier{nullptr, nullptr, 0, 0}, ax);
}

int nts_hip_spmm_csc_bwd_atomic(nts_hip_ctx* ctx, const uint32_t* column_offset,
                                const uint32_t* row_indices, const float* weight,
                                const uint32_t* v, uint32_t v_cap, const float* g_out,
                                uint64_t ld_gout, uint32_t feature_size, float* g_in,
                                uint64_t ld_gin) {
  NTS_CHECK_ARG(ctx && column_offset && row_indices && g_out && g_in, "NULL argument");
  NTS_CHECK_ARG(ld_gout >= feature_size && ld_gin >= feature_size,
                "leading dimension < feature_size");
  if (v_cap == 0 || feature_size == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  const int vec = pick_vec(feature_size, ld_gout, ld_gin, g_out, g_in);
  const uint32_t nv = feature_size / vec;
  const int lpd = nv <= 16 ? 16 : (nv <= 32 ? 32 : 64);
  const uint32_t grid = std::max(1u, std::min(ceil_div(v_cap, kAggThreads / lpd), 4096u));
#define NTS_S(VEC, LPD)                                                                    \
  hipLaunchKernelGGL((k_spmm_scatter_atomic<VEC, LPD>), dim3(grid), dim3(kAggThreads), 0,   \
                     ctx->stream, column_offset, row_indices, weight, v, v_cap, g_out, ld_gout, \
                     nv, g_in, ld_gin)
  if (vec == 4) {
    if (lpd == 16) NTS_S(4, 16); else if (lpd == 32) NTS_S(4, 32); else NTS_S(4, 64);
  } else if (vec == 2) {
    if (lpd == 16) NTS_S(2, 16); else if (lpd == 32) NTS_S(2, 32); else NTS_S(2, 64);
  } else {
    if (lpd == 16) NTS_S(1, 16); else if (lpd == 32) NTS_S(1, 32); else NTS_S(1, 64);
  }
#undef NTS_S
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

}  // extern "C"

template <bool TIER, bool STAGE = false>
static int gather_rows(nts_hip_ctx* ctx, const float* table, uint64_t ld_table,
                       const uint32_t* index, const uint32_t* n, uint32_t n_cap,
                       uint32_t feature_size, float* out, uint64_t ld_out, Tier tier) {
  int vec = pick_vec(feature_size, ld_table, ld_out, table, out);
  if (TIER) vec = std::min(vec, pick_vec(feature_size, tier.ldh, ld_out, tier.host, out));
  const uint32_t nv = feature_size / vec;
  const int lpd = nv <= 16 ? 16 : (nv <= 32 ? 32 : 64);
  const uint32_t grid = std::max(1u, std::min(ceil_div(n_cap, kAggThreads / lpd), 4096u));
#define NTS_R(VEC, LPD)                                                                      \
  hipLaunchKernelGGL((k_gather_rows<VEC, LPD, TIER, STAGE>), dim3(grid), dim3(kAggThreads), 0, \
                     ctx->stream, table, ld_table, index, n, n_cap, nv, out, ld_out, tier)
  if (vec == 4) {
    if (lpd == 16) NTS_R(4, 16); else if (lpd == 32) NTS_R(4, 32); else NTS_R(4, 64);
  } else if (vec == 2) {
    if (lpd == 16) NTS_R(2, 16); else if (lpd == 32) NTS_R(2, 32); else NTS_R(2, 64);
  } else {
    if (lpd == 16) NTS_R(1, 16); else if (lpd == 32) NTS_R(1, 32); else NTS_R(1, 64);
  }
#undef NTS_R
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

extern "C" {

int nts_hip_gather_rows(nts_hip_ctx* ctx, const float* table, uint64_t ld_table,
                        const uint32_t* index, const uint32_t* n, uint32_t n_cap,
                        uint32_t feature_size, float* out, uint64_t ld_out) {
  NTS_CHECK_ARG(ctx && table && index && out, "NULL argument");
  NTS_CHECK_ARG(ld_table >= feature_size && ld_out >= feature_size,
                "leading dimension < feature_size");
  if (n_cap == 0 || feature_size == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  return gather_rows<false>(ctx, table, ld_table, index, n, n_cap, feature_size, out, ld_out,
                            Tier{nullptr, nullptr, 0, 0});
}

int nts_hip_gather_rows_cached(nts_hip_ctx* ctx, const float* cache, uint64_t ld_cache,
                               const uint32_t* cache_map, const float* host_table,
                               uint64_t ld_host, const uint32_t* index, const uint32_t* n,
                               uint32_t n_cap, uint32_t feature_size, float* out,
                               uint64_t ld_out) {
  NTS_CHECK_ARG(ctx && cache_map && host_table && index && out, "NULL argument");
  NTS_CHECK_ARG(ld_cache >= feature_size && ld_host >= feature_size && ld_out >= feature_size,
                "leading dimension < feature_size");
  if (n_cap == 0 || feature_size == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  // an empty cache (no HBM rows) still needs a non-NULL, aligned base
  if (!cache) cache = host_table, ld_cache = ld_host;
  return gather_rows<true>(ctx, cache, ld_cache, index, n, n_cap, feature_size, out, ld_out,
                           Tier{cache_map, host_table, ld_host, 0});
}

int nts_hip_stage_uncached_rows(nts_hip_ctx* ctx, const uint32_t* cache_map,
                                const float* host_table, uint64_t ld_host, const uint32_t* index,
                                const uint32_t* n, uint32_t n_cap, uint32_t feature_size,
                                float* stage, uint64_t ld_stage) {
  NTS_CHECK_ARG(ctx && cache_map && host_table && index && stage, "NULL argument");
  NTS_CHECK_ARG(ld_host >= feature_size && ld_stage >= feature_size,
                "leading dimension < feature_size");
  if (n_cap == 0 || feature_size == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  return gather_rows<true, true>(ctx, host_table, ld_host, index, n, n_cap, feature_size, stage,
                                 ld_stage, Tier{cache_map, host_table, ld_host, 0});
}

int nts_hip_spmm_csc_fwd_cached(nts_hip_ctx* ctx, const uint32_t* column_offset,
                                const uint32_t* row_indices, const float* weight,
                                const uint32_t* v, uint32_t v_cap, const float* cache,
                                uint64_t ld_cache, const uint32_t* cache_map,
                                const float* host_table, uint64_t ld_host, int host_local,
                                const uint32_t* x_row_map, uint32_t feature_size, float* y,
                                uint64_t ldy) {
  NTS_CHECK_ARG(ctx && column_offset && row_indices && cache_map && host_table && x_row_map && y,
                "NULL argument");
  NTS_CHECK_ARG(ld_cache >= feature_size && ld_host >= feature_size && ldy >= feature_size,
                "leading dimension < feature_size");
  if (v_cap == 0 || feature_size == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  if (!cache) cache = host_table, ld_cache = ld_host;
  return launch_gather<true, true>(ctx->stream, column_offset, row_indices, weight, v, v_cap,
                                   cache, ld_cache, x_row_map, feature_size, y, ldy,
                                   Tier{cache_map, host_table, ld_host, host_local});
}

int nts_hip_act_backward(nts_hip_ctx* ctx, uint32_t rows, uint32_t feature_size, const float* g,
                         uint64_t ldg, const float* x_act, uint64_t ldx, float scale, float* out,
                         uint64_t ldo) {
  NTS_CHECK_ARG(ctx && g && x_act && out, "NULL argument");
  NTS_CHECK_ARG(ldg >= feature_size && ldx >= feature_size && ldo >= feature_size,
                "leading dimension < feature_size");
  if (rows == 0 || feature_size == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  const uint64_t n = (uint64_t)rows * feature_size;
  const bool flat = ldg == feature_size && ldx == feature_size && ldo == feature_size &&
                    n % 4 == 0 && (uintptr_t)g % 16 == 0 && (uintptr_t)x_act % 16 == 0 &&
                    (uintptr_t)out % 16 == 0;
  if (flat) {
    const uint32_t grid = std::max(1u, std::min(ceil_div(n / 4, 256), kMaxGrid));
    hipLaunchKernelGGL(k_act_backward, dim3(grid), dim3(256), 0, ctx->stream,
                       reinterpret_cast<const float4*>(g), reinterpret_cast<const float4*>(x_act),
                       reinterpret_cast<float4*>(out), n / 4, scale);
  } else {
    const uint32_t grid = std::max(1u, std::min(ceil_div(n, 256), kMaxGrid));
    hipLaunchKernelGGL(k_act_backward_2d, dim3(grid), dim3(256), 0, ctx->stream, g, ldg, x_act,
                       ldx, out, ldo, rows, feature_size, scale);
  }
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

int nts_hip_gather_labels(nts_hip_ctx* ctx, const int64_t* labels, const uint32_t* index,
                          const uint32_t* n, uint32_t n_cap, int64_t* out) {
  NTS_CHECK_ARG(ctx && labels && index && out, "NULL argument");
  if (n_cap == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  const uint32_t grid = std::max(1u, std::min(ceil_div(n_cap, 256), kMaxGrid));
  hipLaunchKernelGGL(k_gather_labels, dim3(grid), dim3(256), 0, ctx->stream, labels, index, n,
                     n_cap, out);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

int nts_hip_adam(nts_hip_ctx* ctx, float* w, const float* grad, float* m, float* v, uint64_t n,
                 float alpha, float beta1, float beta2, float epsilon, float weight_decay,
                 float beta1_t, float beta2_t, int bias_correction) {
  NTS_CHECK_ARG(ctx && w && grad && m && v, "NULL argument");
  if (n == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  const uint32_t grid = std::max(1u, std::min(ceil_div(n, 256), kMaxGrid));
  hipLaunchKernelGGL(k_adam, dim3(grid), dim3(256), 0, ctx->stream, w, grad, m, v, n, alpha,
                     beta1, beta2, epsilon, weight_decay, beta1_t, beta2_t, bias_correction);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

}  // extern "C"
