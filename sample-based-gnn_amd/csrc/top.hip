// Output layer + loss of the GCN/GraphSAGE drivers, fused.
//
// Reference (toolkits/GCN_SAMPLE_ALLGPU.hpp:214-222, 247-252):
//   vertexForward, last layer:  y = (a.matmul(W)).log_softmax(1)
//   Loss:                       loss = nll_loss(y.log_softmax(1), target)   (mean)
// i.e. logits Z = Y W, log_softmax applied twice (the second is numerically
// ~idempotent but kept: same arithmetic as the reference), the mean negative
// log-likelihood of the target class, and libtorch's backward of all of it.
// On the GPU drivers that is ~12 tiny kernels per step (GEMM, 2 softmax, NLL,
// fills, their backwards, dW and dY GEMMs).  Here one kernel template:
//   LOSS: the loss (block partials);
//   GRAD: dY and per-wave dW partials for the upstream gradient (*grad, or
//         exactly 1 for the training call);
// then k_top_finish sums the partials in a fixed order (deterministic, no
// atomics).  dW partials are stored as chunks [k][ct][wave][16]: a wave
// writes 64-byte runs and the finish kernel reads 256-byte runs.
// forward = <LOSS>, backward = <GRAD>, train = <LOSS, GRAD> (bit-identical
// to forward + backward with grad 1: same code, same orders).
//
// One wave owns 16 rows.  Its Y tile is staged into LDS with coalesced
// 16-byte loads (all issued up front), then the three products run on
// v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation):
//   Z  [16 x Cp] = Y [16 x K] W [K x Cp]      (Cp = C rounded up to 16, <= 64)
//   dY [16 x K]  = dZ [16 x Cp] W^T            (dZ staged through LDS)
//   dW_part [K x Cp] = Y^T [K x 16] dZ [16 x Cp]  (one slab per wave)
// W lives in LDS (zero-padded to Cp columns).  In the accumulator layout a lane
// (i, g) holds Z[4g + v][16 ct + i]; row-wise softmax reductions run over the
// 16 lanes of a group g (xor shuffles 1..8).  Y tile pitch K + 4: the logits'
// A reads (row i, k0 + g) hit 64 distinct banks.
// Layout: Y [n x K] (ld ldy), W [K x C] row-major, labels int64 [n].
#include "common.hpp"

namespace nts_hip {

typedef float f32x4 __attribute__((ext_vector_type(4)));
// waves (16-row tiles) per block; a build-time knob for A/B builds
#ifndef NTS_TOP_WAVES
#define NTS_TOP_WAVES 4
#endif
constexpr int kTopWaves = NTS_TOP_WAVES;
constexpr int kTopThreads = kTopWaves * 64;
constexpr int kTopRowsPerWave = 16;
constexpr int kTopRows = kTopWaves * kTopRowsPerWave;  // rows per block

struct TopArgs {
  const float* Y;
  uint64_t ldy;
  const float* W;
  const int64_t* labels;
  const float* grad;  // GRAD: d loss (device scalar); nullptr = exactly 1
  int n, K, C;
  float* lpart;       // LOSS: [blocks] loss partials
  float* part;        // GRAD: dW partials [K][Cp/16][waves][16]
  float* dY;          // GRAD: [n x K]
  uint32_t* cpart;    // LOSS with accuracy: [blocks] rows whose argmax is the label
};

// Reductions over the 16 lanes of a group (a DPP row) by DPP moves: the
// partner of each step is lane ^ 1, lane ^ 2 (quad permutes), then the other
// quad of the 8-lane half (half mirror) and the other half (row mirror) — the
// pairing tree of an xor butterfly 1, 2, 4, 8, so every lane ends with the
// same sum as that butterfly's.  (The butterfly by __shfl_xor is a chain of
// ds_bpermute round trips: 4-8 us of each block's softmax phase,
// NTS_TOP_TIMING.)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
constexpr int kDppX1 = 0xB1, kDppX2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;
__device__ __forceinline__ float grp_max(float v) {
  v = fmaxf(v, dpp_f<kDppX1>(v));
  v = fmaxf(v, dpp_f<kDppX2>(v));
  v = fmaxf(v, dpp_f<kDppHalfMirror>(v));
  return fmaxf(v, dpp_f<kDppMirror>(v));
}
__device__ __forceinline__ float grp_sum(float v) {
  v += dpp_f<kDppX1>(v);
  v += dpp_f<kDppX2>(v);
  v += dpp_f<kDppHalfMirror>(v);
  return v + dpp_f<kDppMirror>(v);
}
// argmax over the group (first index among equal values)
__device__ __forceinline__ void grp_argmax_step(float& best, int& bi, float ob, int oi) {
  if (ob > best || (ob == best && oi < bi)) {
    best = ob;
    bi = oi;
  }
}
__device__ __forceinline__ int grp_argmax(float best, int bi) {
  grp_argmax_step(best, bi, dpp_f<kDppX1>(best), dpp_i<kDppX1>(bi));
  grp_argmax_step(best, bi, dpp_f<kDppX2>(best), dpp_i<kDppX2>(bi));
  grp_argmax_step(best, bi, dpp_f<kDppHalfMirror>(best), dpp_i<kDppHalfMirror>(bi));
  grp_argmax_step(best, bi, dpp_f<kDppMirror>(best), dpp_i<kDppMirror>(bi));
  return bi;
}

// Stage W into LDS as sW[k][Cp] (zero columns >= C): coalesced loads of the
// contiguous [K x C] matrix.  K % 16 == 0 makes K x C a multiple of 4: with a
// 16-byte aligned W the whole matrix goes as float4s, up to 16 per thread in
// flight (one memory round trip for C3's 256 x 47; the scalar form took six
// dependent rounds of 8 loads, most of the kernel at 16 blocks).
template <int CP>
__device__ __forceinline__ void stage_w(const TopArgs& a, float* sW) {
  const int C = a.C, KC = a.K * C;
  if (((uintptr_t)a.W & 15) == 0) {
    const float4* W4 = reinterpret_cast<const float4*>(a.W);
    const int nq = KC / 4;
    constexpr int B = 16;
    for (int q0 = threadIdx.x; q0 < nq; q0 += B * kTopThreads) {
      float4 v[B];
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int q = q0 + u * kTopThreads;
        v[u] = q < nq ? W4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int q = q0 + u * kTopThreads;
        if (q < nq) {
          const float x[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
          int r = 4 * q / C, cc = 4 * q - r * C;  // one division per float4
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            sW[r * CP + cc] = x[c];
            if (++cc == C) {
              cc = 0;
              ++r;
            }
          }
        }
      }
    }
  } else {
    constexpr int B = 8;
    for (int e0 = threadIdx.x; e0 < KC; e0 += B * kTopThreads) {
      float v[B];
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int e = e0 + u * kTopThreads;
        v[u] = e < KC ? a.W[e] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int e = e0 + u * kTopThreads;
        if (e < KC) sW[(e / C) * CP + e % C] = v[u];
      }
    }
  }
  const int pad = CP - C;
  for (int e = threadIdx.x; e < a.K * pad; e += kTopThreads)
    sW[(e / pad) * CP + C + e % pad] = 0.f;
}

// Stage this wave's 16 Y rows into sY[16][K + 4] (rows >= n are zero).
// VEC4: 16-byte loads (ldy % 4 == 0, Y 16-byte aligned).
template <bool VEC4>
__device__ __forceinline__ void stage_y(const TopArgs& a, float* sY, int r0, int lane) {
  const int K = a.K, P = K + 4;
  constexpr int B = VEC4 ? 16 : 8;  // loads in flight per lane (K = 256: one round)
  if (VEC4) {
    const int kq = K / 4, it = K / 16;  // float4 per row; per lane (16 rows x kq / 64)
    for (int j0 = 0; j0 < it; j0 += B) {
      float4 v[B];
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int q = lane + kWave * (j0 + u), rr = q / kq, r = r0 + rr;
        v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (j0 + u < it && r < a.n)
          v[u] = *reinterpret_cast<const float4*>(a.Y + (uint64_t)r * a.ldy + 4 * (q % kq));
      }
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int q = lane + kWave * (j0 + u);
        if (j0 + u < it) *reinterpret_cast<float4*>(sY + (q / kq) * P + 4 * (q % kq)) = v[u];
      }
    }
  } else {
    const int it = K / 4;  // 16 rows x K / 64 per lane
    for (int j0 = 0; j0 < it; j0 += B) {
      float v[B];
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int q = lane + kWave * (j0 + u), r = r0 + q / K;
        v[u] = (j0 + u < it && r < a.n) ? a.Y[(uint64_t)r * a.ldy + q % K] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int q = lane + kWave * (j0 + u);
        if (j0 + u < it) sY[(q / K) * P + q % K] = v[u];
      }
    }
  }
}

// Z tile of this wave's 16 rows: z[ct][v] = Z[r0 + 4g + v][16 ct + i].
template <int NCT>
__device__ __forceinline__ void wave_logits(int K, const float* sW, const float* sY, int i, int g,
                                            f32x4 (&z)[NCT]) {
  constexpr int CP = 16 * NCT;
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) z[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* yr = sY + i * (K + 4);
  for (int k1 = 0; k1 < K; k1 += 16) {  // K % 16 == 0
#pragma unroll
    for (int k0 = k1; k0 < k1 + 16; k0 += 4) {
      const float av = yr[k0 + g];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        z[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sW[(k0 + g) * CP + 16 * ct + i], z[ct],
                                                     0, 0, 0);
    }
  }
}

// log_softmax of rows 4g+v (one value per column tile per lane), twice.
// lp/lp2 in the same layout; columns >= C excluded.
template <int NCT>
__device__ __forceinline__ void log_softmax2(const f32x4 (&z)[NCT], int C, int i,
                                             float (&lp)[NCT][4], float (&lp2)[NCT][4]) {
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    float m = -INFINITY;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
      if (16 * ct + i < C) m = fmaxf(m, z[ct][v]);
    m = grp_max(m);
    float s = 0.f;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
      if (16 * ct + i < C) s += expf(z[ct][v] - m);
    s = grp_sum(s);
    const float lse = m + logf(s);
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) lp[ct][v] = z[ct][v] - lse;
    float m2 = -INFINITY;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
      if (16 * ct + i < C) m2 = fmaxf(m2, lp[ct][v]);
    m2 = grp_max(m2);
    float s2 = 0.f;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
      if (16 * ct + i < C) s2 += expf(lp[ct][v] - m2);
    s2 = grp_sum(s2);
    const float lse2 = m2 + logf(s2);
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) lp2[ct][v] = lp[ct][v] - lse2;
  }
}

static inline size_t top_lds(int K, int Cp) {
  return ((size_t)K * Cp + (size_t)kTopWaves * 16 * (K + 4) + (size_t)kTopRows * Cp) *
         sizeof(float);
}

template <int NCT, bool LOSS, bool GRAD, bool VEC4>
__global__ __launch_bounds__(kTopThreads) void k_top_xent(TopArgs a) {
  constexpr int CP = 16 * NCT;
  extern __shared__ float smem[];
  __shared__ float wl[kTopWaves];
  __shared__ uint32_t wc[kTopWaves];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int K = a.K;
  float* sW = smem;                                      // [K][CP]
  float* sY = smem + K * CP + w * 16 * (K + 4);          // this wave's [16][K + 4]
  float* dz = smem + K * CP + kTopWaves * 16 * (K + 4) + w * 16 * CP;  // [16][CP]
  const int r0 = blockIdx.x * kTopRows + w * kTopRowsPerWave;
  stage_y<VEC4>(a, sY, r0, lane);
  stage_w<CP>(a, sW);
  __syncthreads();
  f32x4 z[NCT];
  wave_logits<NCT>(K, sW, sY, i, g, z);
  float lp[NCT][4], lp2[NCT][4];
  log_softmax2<NCT>(z, a.C, i, lp, lp2);
  int tgt[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int r = r0 + 4 * g + v;
    tgt[v] = r < a.n ? (int)a.labels[r] : -1;
  }
  if (LOSS) {
    // -lp2[target] of each valid row, summed in a fixed order (v, then lanes)
    float l = 0.f;
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        if (16 * ct + i == tgt[v]) l -= lp2[ct][v];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) l += __shfl_down(l, o, kWave);
    if (lane == 0) wl[w] = l;
    if (a.cpart) {
      // getCorrect (toolkits/GCN_SAMPLE_ALLGPU.hpp:166-172): argmax of the
      // log_softmax output (first index among equal values, as torch's
      // argmax) == label
      uint32_t ok = 0;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float best = -INFINITY;
        int bi = 0x7fffffff;
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
          if (16 * ct + i < a.C && lp[ct][v] > best) {
            best = lp[ct][v];
            bi = 16 * ct + i;
          }
        bi = grp_argmax(best, bi);
        ok += (i == 0 && tgt[v] >= 0 && bi == tgt[v]) ? 1u : 0u;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) ok += __shfl_down(ok, o, kWave);
      if (lane == 0) wc[w] = ok;
    }
  }
  if (GRAD) {
    const float gl = (a.grad ? *a.grad : 1.0f) / (float)a.n;
    // nll backward, then y = log_softmax(x): dx = dy - exp(y) * sum(dy), twice
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int r = r0 + 4 * g + v;
      float d2[NCT], s2 = 0.f;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        d2[ct] = (16 * ct + i == tgt[v]) ? -gl : 0.f;
        s2 += d2[ct];
      }
      s2 = grp_sum(s2);
      float d1[NCT], s1 = 0.f;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const bool on = 16 * ct + i < a.C;
        d1[ct] = on ? d2[ct] - expf(lp2[ct][v]) * s2 : 0.f;
        s1 += d1[ct];
      }
      s1 = grp_sum(s1);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const bool on = 16 * ct + i < a.C && r < a.n;
        dz[(4 * g + v) * CP + 16 * ct + i] = on ? d1[ct] - expf(lp[ct][v]) * s1 : 0.f;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's dZ stores landed
    __builtin_amdgcn_wave_barrier();
    // dY [16 x K] = dZ [16 x CP] W^T: A lane (i,g) = dZ[i][c], B = W[k = 16 kt + i][c].
    // Four k tiles at a time: four independent MFMA chains share each dZ read
    // (one chain per tile was a serial LDS-read -> MFMA latency chain, and a
    // block of 4 waves has one wave per SIMD to hide it).  Tiles past K/16
    // repeat the last one and are not stored; each chain's order is unchanged.
    const int nkt = K / 16;
    constexpr int KT = 4;
    for (int kt0 = 0; kt0 < nkt; kt0 += KT) {
      f32x4 acc[KT];
      int ktu[KT];
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        ktu[u] = min(kt0 + u, nkt - 1);
      }
#pragma unroll
      for (int c0 = 0; c0 < CP; c0 += 4) {
        const float av = dz[i * CP + c0 + g];
#pragma unroll
        for (int u = 0; u < KT; ++u)
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sW[(16 * ktu[u] + i) * CP + c0 + g], acc[u],
                                                        0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        if (kt0 + u >= nkt) break;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int r = r0 + 4 * g + v;
          if (r < a.n) a.dY[(uint64_t)r * K + 16 * (kt0 + u) + i] = acc[u][v];
        }
      }
    }
    // dW partial [K x CP] = Y^T [K x 16] dZ [16 x CP]:
    //   A lane (i,g) = Y[r0 + 4s + g][16 kt + i], B = dZ[4s + g][16 ct + i]
    // two k tiles at a time (2 NCT chains sharing the dZ reads)
    const uint64_t nslab = (uint64_t)gridDim.x * kTopWaves;
    const uint64_t slab = (uint64_t)blockIdx.x * kTopWaves + w;
    constexpr int KW = 2;
    for (int kt0 = 0; kt0 < nkt; kt0 += KW) {
      f32x4 acc[KW][NCT];
      int ktu[KW];
#pragma unroll
      for (int u = 0; u < KW; ++u) {
        ktu[u] = min(kt0 + u, nkt - 1);
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) acc[u][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        float bv[NCT];
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) bv[ct] = dz[(4 * s + g) * CP + 16 * ct + i];
#pragma unroll
        for (int u = 0; u < KW; ++u) {
          const float av = sY[(4 * s + g) * (K + 4) + 16 * ktu[u] + i];
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct)
            acc[u][ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[ct], acc[u][ct], 0, 0, 0);
        }
      }
      // acc[u][ct][v] = dW[16 kt + 4 g + v][16 ct + i] -> chunk (k, ct), lane i
#pragma unroll
      for (int u = 0; u < KW; ++u) {
        if (kt0 + u >= nkt) break;
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const uint64_t q = (uint64_t)(16 * (kt0 + u) + 4 * g + v) * NCT + ct;
            a.part[(q * nslab + slab) * 16 + i] = acc[u][ct][v];
          }
      }
    }
  }
  if (LOSS) {
    __syncthreads();
    if (threadIdx.x == 0) {
      float s = 0.f;
      uint32_t c = 0;
      for (int q = 0; q < kTopWaves; ++q) {
        s += wl[q];
        c += wc[q];
      }
      a.lpart[blockIdx.x] = s;
      if (a.cpart) a.cpart[blockIdx.x] = c;
    }
  }
}

// K-split form (the default): one block of kTopWaves waves per 16-row tile,
// wave w taking the k tiles kt = w, w + kTopWaves, ... of every product.
// The per-wave form above runs a whole tile's three products on one wave —
// ~600 dependent v_mfma_f32_16x16x4_f32 at K = 256 with one wave per SIMD,
// 35 us however few rows (C3: 1,024 rows, 64 waves on 256 CUs).  Here the
// logits are four partial chains summed in a fixed order (w = 0..3) through
// LDS; every wave then holds the same Z and log-softmax, wave 0 writes dZ
// and the loss; dY and dW run on each wave's k tiles (two at a time).  One dW
// slab per block.  Deterministic; the logits' summation order differs from
// the per-wave form (NTS_TOP_KSPLIT=0) by rounding only.
static inline size_t top_ks_lds(int K, int Cp) {
  return ((size_t)K * Cp + (size_t)16 * (K + 4) + (size_t)(kTopWaves + 1) * 16 * Cp) * sizeof(float);
}

template <int NCT, bool LOSS, bool GRAD, bool VEC4>
__global__ __launch_bounds__(kTopThreads) void k_top_xent_ks(TopArgs a) {
  constexpr int CP = 16 * NCT, NW = kTopWaves;
  extern __shared__ float smem[];
  __shared__ float wl[NW];
  __shared__ uint32_t wc[NW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int K = a.K, P = K + 4, nkt = K / 16;
  float* sW = smem;                // [K][CP]
  float* sY = sW + K * CP;         // [16][K + 4]
  float* zp = sY + 16 * P;         // [NW][16][CP] partial logits
  float* dz = zp + NW * 16 * CP;   // [16][CP]
  const int r0 = blockIdx.x * 16;
#ifdef NTS_TOP_TIMING  // (probe builds: phase times of two blocks, printf)
  uint64_t tt[8];
  int nt_ = 0;
  auto mark = [&] { tt[nt_++] = wall_clock64(); };
#else
  auto mark = [] {};
#endif
  mark();
  // the rows' labels and the upstream gradient first: their global loads
  // then overlap the staging instead of following the logits (a dependent
  // memory latency of 4-6 us per block there, NTS_TOP_TIMING)
  constexpr int VPW = 4 / NW;  // rows 4 g + v per lane group finished by this wave
  static_assert(4 % NW == 0, "kTopWaves must divide 4");
  int tgt[VPW];
#pragma unroll
  for (int vv = 0; vv < VPW; ++vv) {
    const int r = r0 + 4 * g + w + vv * NW;
    tgt[vv] = r < a.n ? (int)a.labels[r] : -1;
  }
  const float gl = GRAD ? (a.grad ? *a.grad : 1.0f) / (float)a.n : 0.f;
  {  // the tile's 16 rows, all threads (rows >= n are zero)
    constexpr int B = 8;
    if (VEC4) {
      const int kq = K / 4, tot = 16 * kq;
      for (int q0 = threadIdx.x; q0 < tot; q0 += B * kTopThreads) {
        float4 v[B];
#pragma unroll
        for (int u = 0; u < B; ++u) {
          const int q = q0 + u * kTopThreads, rr = q / kq, r = r0 + rr;
          v[u] = (q < tot && r < a.n) ? *reinterpret_cast<const float4*>(a.Y + (uint64_t)r * a.ldy + 4 * (q % kq))
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < B; ++u) {
          const int q = q0 + u * kTopThreads;
          if (q < tot) *reinterpret_cast<float4*>(sY + (q / kq) * P + 4 * (q % kq)) = v[u];
        }
      }
    } else {
      const int tot = 16 * K;
      for (int q0 = threadIdx.x; q0 < tot; q0 += B * kTopThreads) {
        float v[B];
#pragma unroll
        for (int u = 0; u < B; ++u) {
          const int q = q0 + u * kTopThreads, r = r0 + q / K;
          v[u] = (q < tot && r < a.n) ? a.Y[(uint64_t)r * a.ldy + q % K] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < B; ++u) {
          const int q = q0 + u * kTopThreads;
          if (q < tot) sY[(q / K) * P + q % K] = v[u];
        }
      }
    }
  }
  stage_w<CP>(a, sW);
  __syncthreads();
  mark();
  f32x4 z[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) z[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    const float* yr = sY + i * P;
    for (int kt = w; kt < nkt; kt += NW) {
#pragma unroll
      for (int k0 = 16 * kt; k0 < 16 * kt + 16; k0 += 4) {
        const float av = yr[k0 + g];
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
          z[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sW[(k0 + g) * CP + 16 * ct + i], z[ct], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
    for (int v = 0; v < 4; ++v) zp[(w * 16 + 4 * g + v) * CP + 16 * ct + i] = z[ct][v];
  __syncthreads();
  mark();
  // each wave finishes the rows 4 g + v of its own v (v = w, w + NW, ...): the
  // logits' sum over the waves' k-splits, log_softmax twice (log_softmax2's
  // arithmetic per row), the loss and accuracy terms and dZ — a quarter of the
  // tile each (the whole tile on wave 0 was 4-6 us of every block, NTS_TOP_TIMING)
  float lw = 0.f;
  uint32_t okw = 0;
#pragma unroll
  for (int vv = 0; vv < VPW; ++vv) {
    const int v = w + vv * NW;
    float zv[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      float t = zp[(4 * g + v) * CP + 16 * ct + i];
#pragma unroll
      for (int q = 1; q < NW; ++q) t += zp[(q * 16 + 4 * g + v) * CP + 16 * ct + i];
      zv[ct] = t;
    }
    float lp[NCT], lp2[NCT];
    {
      float m = -INFINITY;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        if (16 * ct + i < a.C) m = fmaxf(m, zv[ct]);
      m = grp_max(m);
      float sm = 0.f;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        if (16 * ct + i < a.C) sm += expf(zv[ct] - m);
      sm = grp_sum(sm);
      const float lse = m + logf(sm);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) lp[ct] = zv[ct] - lse;
      float m2 = -INFINITY;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        if (16 * ct + i < a.C) m2 = fmaxf(m2, lp[ct]);
      m2 = grp_max(m2);
      float s2 = 0.f;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        if (16 * ct + i < a.C) s2 += expf(lp[ct] - m2);
      s2 = grp_sum(s2);
      const float lse2 = m2 + logf(s2);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) lp2[ct] = lp[ct] - lse2;
    }
    if (LOSS) {
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        if (16 * ct + i == tgt[vv]) lw -= lp2[ct];
      if (a.cpart) {  // getCorrect (toolkits/GCN_SAMPLE_ALLGPU.hpp:166-172), as k_top_xent
        float best = -INFINITY;
        int bi = 0x7fffffff;
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
          if (16 * ct + i < a.C && lp[ct] > best) {
            best = lp[ct];
            bi = 16 * ct + i;
          }
        bi = grp_argmax(best, bi);
        okw += (i == 0 && tgt[vv] >= 0 && bi == tgt[vv]) ? 1u : 0u;
      }
    }
    if (GRAD) {
      const int r = r0 + 4 * g + v;
      float d2[NCT], s2 = 0.f;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        d2[ct] = (16 * ct + i == tgt[vv]) ? -gl : 0.f;
        s2 += d2[ct];
      }
      s2 = grp_sum(s2);
      float d1[NCT], s1 = 0.f;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const bool on = 16 * ct + i < a.C;
        d1[ct] = on ? d2[ct] - expf(lp2[ct]) * s2 : 0.f;
        s1 += d1[ct];
      }
      s1 = grp_sum(s1);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const bool on = 16 * ct + i < a.C && r < a.n;
        dz[(4 * g + v) * CP + 16 * ct + i] = on ? d1[ct] - expf(lp[ct]) * s1 : 0.f;
      }
    }
  }
  if (LOSS) {  // the wave's terms, then the block's in wave order (below)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) lw += __shfl_down(lw, o, kWave);
    if (lane == 0) wl[w] = lw;
    if (a.cpart) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) okw += __shfl_down(okw, o, kWave);
      if (lane == 0) wc[w] = okw;
    }
  }
  if (GRAD) {
    __syncthreads();
    mark();
    // dY [16 x K] = dZ W^T on this wave's k tiles, two at a time
    constexpr int KT = 2;
    for (int j0 = w; j0 < nkt; j0 += KT * NW) {
      f32x4 acc[KT];
      int ktu[KT];
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        ktu[u] = min(j0 + u * NW, nkt - 1);
      }
#pragma unroll
      for (int c0 = 0; c0 < CP; c0 += 4) {
        const float av = dz[i * CP + c0 + g];
#pragma unroll
        for (int u = 0; u < KT; ++u)
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sW[(16 * ktu[u] + i) * CP + c0 + g], acc[u],
                                                        0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        const int kt = j0 + u * NW;
        if (kt >= nkt) break;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int r = r0 + 4 * g + v;
          if (r < a.n) a.dY[(uint64_t)r * K + 16 * kt + i] = acc[u][v];
        }
      }
    }
    mark();
    // dW slab of this block [K x CP] = Y^T dZ, rows of this wave's k tiles
    const uint64_t nslab = gridDim.x, slab = blockIdx.x;
    for (int j0 = w; j0 < nkt; j0 += KT * NW) {
      f32x4 acc[KT][NCT];
      int ktu[KT];
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        ktu[u] = min(j0 + u * NW, nkt - 1);
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) acc[u][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        float bv[NCT];
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) bv[ct] = dz[(4 * s4 + g) * CP + 16 * ct + i];
#pragma unroll
        for (int u = 0; u < KT; ++u) {
          const float av = sY[(4 * s4 + g) * P + 16 * ktu[u] + i];
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct)
            acc[u][ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[ct], acc[u][ct], 0, 0, 0);
        }
      }
#pragma unroll
      for (int u = 0; u < KT; ++u) {
        const int kt = j0 + u * NW;
        if (kt >= nkt) break;
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const uint64_t q = (uint64_t)(16 * kt + 4 * g + v) * NCT + ct;
            a.part[(q * nslab + slab) * 16 + i] = acc[u][ct][v];
          }
      }
    }
  }
  mark();
  if (LOSS) {
    __syncthreads();
    if (threadIdx.x == 0) {
      float l = 0.f;
      uint32_t c = 0;
      for (int q = 0; q < NW; ++q) {
        l += wl[q];
        c += wc[q];
      }
      a.lpart[blockIdx.x] = l;
      if (a.cpart) a.cpart[blockIdx.x] = c;
    }
  }
#ifdef NTS_TOP_TIMING
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  mark();
  if ((blockIdx.x == 3 || blockIdx.x == gridDim.x - 5) && threadIdx.x == 64 && nt_ == 7)
    printf("top blk %d: stage %d logits %d softmax %d dY %d dW %d tail %d (x10ns)\n", blockIdx.x,
           (int)(tt[1] - tt[0]), (int)(tt[2] - tt[1]), (int)(tt[3] - tt[2]), (int)(tt[4] - tt[3]),
           (int)(tt[5] - tt[4]), (int)(tt[6] - tt[5]));
#endif
}

// Blocks [0, K*NCT): dW chunk (k, ct) = sum over the wave slabs — thread
// (sg, i) sums slabs sg, sg+16, ... in order (40 loads in flight), then a fixed
// pairwise tree over the 16 slab groups.  Block K*NCT (or 0 without GRAD):
// loss = (sum of block partials, fixed tree) / n.
template <int NCT>
__global__ __launch_bounds__(256) void k_top_finish(const float* __restrict__ part, int nslab,
                                                    const float* __restrict__ lpart, int nblk,
                                                    int n, int K, int C, int nchunks,
                                                    float* __restrict__ dW, float* loss,
                                                    const uint32_t* __restrict__ cpart,
                                                    uint32_t* correct) {
  __shared__ float red[256];
  const int t = threadIdx.x;
  float acc = 0.f;
  if ((int)blockIdx.x < nchunks) {
    const int q = blockIdx.x, sg = t >> 4, i = t & 15;
    const float* p = part + (uint64_t)q * nslab * 16 + i;
    // every load of a thread in flight at once up to 640 slabs (C2: 625; the
    // sum order is unchanged: z ascending)
    constexpr int B = 40;
    for (int z = sg; z < nslab; z += 16 * B) {
      float v[B];
#pragma unroll
      for (int u = 0; u < B; ++u) v[u] = z + 16 * u < nslab ? p[(uint64_t)(z + 16 * u) * 16] : 0.f;
#pragma unroll
      for (int u = 0; u < B; ++u)
        if (z + 16 * u < nslab) acc += v[u];
    }
    red[t] = acc;
    __syncthreads();
#pragma unroll
    for (int h = 128; h >= 16; h >>= 1) {
      if (t < h) red[t] += red[t + h];
      __syncthreads();
    }
    const int k = q / NCT, c = 16 * (q % NCT) + t;
    if (t < 16 && c < C) dW[(uint64_t)k * C + c] = red[t];
  } else {
    uint32_t c = 0;
    for (int b = t; b < nblk; b += 256) {
      acc += lpart[b];
      if (cpart) c += cpart[b];
    }
    red[t] = acc;
    __shared__ uint32_t cred[256];
    cred[t] = c;
    __syncthreads();
#pragma unroll
    for (int h = 128; h >= 1; h >>= 1) {
      if (t < h) {
        red[t] += red[t + h];
        cred[t] += cred[t + h];
      }
      __syncthreads();
    }
    if (t == 0) {
      *loss = red[0] / (float)n;
      if (correct) *correct += cred[0];  // accumulates over batches
    }
  }
  (void)K;
}

static bool top_ksplit() {  // compile-time A/B: -DNTS_TOP_KSPLIT=0 runs the per-wave form
#ifdef NTS_TOP_KSPLIT
  return NTS_TOP_KSPLIT != 0;
#else
  return true;
#endif
}

template <int NCT, bool LOSS, bool GRAD>
static int launch_top_ks(hipStream_t st, int nblk, const TopArgs& a) {
  const size_t lds = top_ks_lds(a.K, 16 * NCT);
  const bool v4 = a.ldy % 4 == 0 && (uintptr_t)a.Y % 16 == 0;
  const void* f = v4 ? reinterpret_cast<const void*>(&k_top_xent_ks<NCT, LOSS, GRAD, true>)
                     : reinterpret_cast<const void*>(&k_top_xent_ks<NCT, LOSS, GRAD, false>);
  NTS_HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  if (v4)
    hipLaunchKernelGGL((k_top_xent_ks<NCT, LOSS, GRAD, true>), dim3(nblk), dim3(kTopThreads), lds,
                       st, a);
  else
    hipLaunchKernelGGL((k_top_xent_ks<NCT, LOSS, GRAD, false>), dim3(nblk), dim3(kTopThreads), lds,
                       st, a);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

template <int NCT, bool LOSS, bool GRAD>
static int launch_top(hipStream_t st, int nblk, const TopArgs& a) {
  if (top_ksplit()) return launch_top_ks<NCT, LOSS, GRAD>(st, nblk, a);
  const size_t lds = top_lds(a.K, 16 * NCT);
  const bool v4 = a.ldy % 4 == 0 && (uintptr_t)a.Y % 16 == 0;
  const void* f = v4 ? reinterpret_cast<const void*>(&k_top_xent<NCT, LOSS, GRAD, true>)
                     : reinterpret_cast<const void*>(&k_top_xent<NCT, LOSS, GRAD, false>);
  NTS_HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  if (v4)
    hipLaunchKernelGGL((k_top_xent<NCT, LOSS, GRAD, true>), dim3(nblk), dim3(kTopThreads), lds,
                       st, a);
  else
    hipLaunchKernelGGL((k_top_xent<NCT, LOSS, GRAD, false>), dim3(nblk), dim3(kTopThreads), lds,
                       st, a);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

template <bool LOSS, bool GRAD>
static int launch_top_any(hipStream_t st, int nblk, int Cp, const TopArgs& a) {
  switch (Cp / 16) {
    case 1: return launch_top<1, LOSS, GRAD>(st, nblk, a);
    case 2: return launch_top<2, LOSS, GRAD>(st, nblk, a);
    case 3: return launch_top<3, LOSS, GRAD>(st, nblk, a);
    default: return launch_top<4, LOSS, GRAD>(st, nblk, a);
  }
}

static int launch_finish(hipStream_t st, int Cp, const float* part, int nslab, const float* lpart,
                         int nblk, int n, int K, int C, bool grad, bool loss_on, float* dW,
                         float* loss, const uint32_t* cpart, uint32_t* correct) {
  const int nchunks = grad ? K * (Cp / 16) : 0;
  const dim3 grid(nchunks + (loss_on ? 1 : 0));
#define NTS_F(NCT)                                                                             \
  hipLaunchKernelGGL(k_top_finish<NCT>, grid, dim3(256), 0, st, part, nslab, lpart, nblk, n, K, \
                     C, nchunks, dW, loss, cpart, correct)
  switch (Cp / 16) {
    case 1: NTS_F(1); break;
    case 2: NTS_F(2); break;
    case 3: NTS_F(3); break;
    default: NTS_F(4); break;
  }
#undef NTS_F
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

}  // namespace nts_hip

using namespace nts_hip;

extern "C" {

static int top_check(nts_hip_ctx* ctx, int n, int K, int C, uint64_t ldy) {
  NTS_CHECK_ARG(n > 0 && K > 0 && C > 0 && ldy >= (uint64_t)K, "shape");
  NTS_CHECK_ARG(C <= kWave, "class count above 64 is not supported by the fused loss");
  NTS_CHECK_ARG(K % 16 == 0, "the fused loss needs K % 16 == 0");
  NTS_CHECK_ARG(top_lds(K, (C + 15) / 16 * 16) <= 160 * 1024, "K x C too large for the fused loss");
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  return NTS_OK;
}

// scratch: [loss partials, 64-float aligned][correct partials][dW partial chunks]
static int top_run(nts_hip_ctx* ctx, bool loss_on, bool grad_on, const float* Y, uint64_t ldy,
                   int n, int K, const float* W, int C, const int64_t* labels,
                   const float* grad_loss, float* loss, float* dY, float* dW, uint32_t* correct) {
  NTS_RET(top_check(ctx, n, K, C, ldy));
  const int Cp = (C + 15) / 16 * 16;
  const bool ks = top_ksplit();
  const int nblk = ks ? (n + 15) / 16 : (n + kTopRows - 1) / kTopRows;
  const int nslab = ks ? nblk : nblk * kTopWaves;
  const size_t lp = ((size_t)nblk + 63) / 64 * 64;
  NTS_RET(ensure_scratch(
      ctx, (2 * lp + (grad_on ? (size_t)nslab * K * Cp : 0)) * sizeof(float)));
  float* base = (float*)ctx->scratch;
  uint32_t* cpart = (loss_on && correct) ? reinterpret_cast<uint32_t*>(base + lp) : nullptr;
  TopArgs a{Y, ldy, W, labels, grad_loss, n, K, C, base, base + 2 * lp, dY, cpart};
  hipStream_t st = ctx->stream;
  if (loss_on && grad_on) NTS_RET((launch_top_any<true, true>(st, nblk, Cp, a)));
  else if (loss_on) NTS_RET((launch_top_any<true, false>(st, nblk, Cp, a)));
  else NTS_RET((launch_top_any<false, true>(st, nblk, Cp, a)));
  return launch_finish(st, Cp, a.part, nslab, a.lpart, nblk, n, K, C, grad_on, loss_on, dW, loss,
                       cpart, cpart ? correct : nullptr);
}

int nts_hip_linear_xent_fwd(nts_hip_ctx* ctx, const float* Y, uint64_t ldy, int n, int K,
                            const float* W, int C, const int64_t* labels, float* loss,
                            uint32_t* correct) {
  NTS_CHECK_ARG(ctx && Y && W && labels && loss, "NULL argument");
  return top_run(ctx, true, false, Y, ldy, n, K, W, C, labels, nullptr, loss, nullptr, nullptr,
                 correct);
}

int nts_hip_linear_xent_bwd(nts_hip_ctx* ctx, const float* Y, uint64_t ldy, int n, int K,
                            const float* W, int C, const int64_t* labels, const float* grad_loss,
                            float* dY, float* dW) {
  NTS_CHECK_ARG(ctx && Y && W && labels && grad_loss && dY && dW, "NULL argument");
  return top_run(ctx, false, true, Y, ldy, n, K, W, C, labels, grad_loss, nullptr, dY, dW,
                 nullptr);
}

int nts_hip_linear_xent_train(nts_hip_ctx* ctx, const float* Y, uint64_t ldy, int n, int K,
                              const float* W, int C, const int64_t* labels, float* loss,
                              float* dY, float* dW, uint32_t* correct) {
  NTS_CHECK_ARG(ctx && Y && W && labels && loss && dY && dW, "NULL argument");
  return top_run(ctx, true, true, Y, ldy, n, K, W, C, labels, nullptr, loss, dY, dW, correct);
}

}  // extern "C"
