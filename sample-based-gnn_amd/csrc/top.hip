// Output layer + loss of the GCN/GraphSAGE drivers, fused.
//
// Reference (toolkits/GCN_SAMPLE_ALLGPU.hpp:214-222, 247-252):
//   vertexForward, last layer:  y = (a.matmul(W)).log_softmax(1)
//   Loss:                       loss = nll_loss(y.log_softmax(1), target)   (mean)
// i.e. logits Z = Y W, log_softmax applied twice (the second is numerically
// ~idempotent but kept: same arithmetic as the reference), the mean negative
// log-likelihood of the target class, and libtorch's backward of all of it.
// On the GPU drivers that is ~12 tiny kernels per step (GEMM, 2 softmax, NLL,
// fills, their backwards, dW and dY GEMMs).  Here: one forward kernel and one
// backward kernel plus fixed-order reductions of their partials
// (deterministic, no atomics).
//
// One wave owns 16 rows.  The three products run on v_mfma_f32_16x16x4_f32
// (exact fp32 products, fp32 accumulation):
//   Z  [16 x Cp] = Y [16 x K] W [K x Cp]      (Cp = C rounded up to 16, <= 64)
//   dY [16 x K]  = dZ [16 x Cp] W^T            (dZ staged through LDS)
//   dW_part [K x Cp] = Y^T [K x 16] dZ [16 x Cp]  (one slab per wave)
// W lives in LDS (zero-padded to Cp columns).  In the accumulator layout a lane
// (i, g) holds Z[4g + v][16 ct + i]; row-wise softmax reductions run over the
// 16 lanes of a group g (xor shuffles 1..8).
// Layout: Y [n x K] (ld ldy), W [K x C] row-major, labels int64 [n].
#include "common.hpp"

namespace nts_hip {

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kTopWaves = 4;
constexpr int kTopThreads = kTopWaves * 64;
constexpr int kTopRowsPerWave = 16;
constexpr int kTopRows = kTopWaves * kTopRowsPerWave;  // rows per block

struct TopArgs {
  const float* Y;
  uint64_t ldy;
  const float* W;
  const int64_t* labels;
  const float* grad;  // backward: d loss (device scalar)
  int n, K, C, Cp;
  float* part;        // forward: [blocks] loss partials; backward: [waves][K*C] dW partials
  float* dY;          // backward: [n x K]
};

__device__ __forceinline__ float grp_max(float v) {  // over the 16 lanes of a group
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ float grp_sum(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Stage W into LDS as sW[k][Cp] (zero columns >= C).
__device__ __forceinline__ void stage_w(const TopArgs& a, float* sW) {
  for (int e = threadIdx.x; e < a.K * a.Cp; e += kTopThreads) {
    const int k = e / a.Cp, c = e % a.Cp;
    sW[e] = c < a.C ? a.W[(uint64_t)k * a.C + c] : 0.f;
  }
  __syncthreads();
}

// Z tile of this wave's 16 rows: z[ct][v] = Z[r0 + 4g + v][16 ct + i].
template <int NCT>
__device__ __forceinline__ void wave_logits(const TopArgs& a, const float* sW, int r0, int i,
                                            int g, f32x4 (&z)[NCT]) {
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) z[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int row = min(r0 + i, a.n - 1);  // rows past n compute garbage, never stored
  const float* yr = a.Y + (uint64_t)row * a.ldy;
  for (int k0 = 0; k0 < a.K; k0 += 4) {
    const int k = k0 + g;
    const float av = k < a.K ? yr[k] : 0.f;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const float bv = k < a.K ? sW[k * a.Cp + 16 * ct + i] : 0.f;
      z[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, z[ct], 0, 0, 0);
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

template <int NCT>
__global__ __launch_bounds__(kTopThreads) void k_top_xent_fwd(TopArgs a) {
  extern __shared__ float smem[];
  float* sW = smem;
  __shared__ float wl[kTopWaves];
  stage_w(a, sW);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int r0 = blockIdx.x * kTopRows + w * kTopRowsPerWave;
  f32x4 z[NCT];
  wave_logits<NCT>(a, sW, r0, i, g, z);
  float lp[NCT][4], lp2[NCT][4];
  log_softmax2<NCT>(z, a.C, i, lp, lp2);
  // -lp2[target] of each valid row, summed in a fixed order (v, then groups)
  float l = 0.f;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int r = r0 + 4 * g + v;
    const int t = r < a.n ? (int)a.labels[r] : -1;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
      if (16 * ct + i == t) l -= lp2[ct][v];
  }
  // lane-order reduction over the wave (deterministic)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) l += __shfl_down(l, o, kWave);
  if (lane == 0) wl[w] = l;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int q = 0; q < kTopWaves; ++q) s += wl[q];
    a.part[blockIdx.x] = s;
  }
}

// loss = (sum of block partials) / n, fixed tree
__global__ void k_top_loss_reduce(const float* part, int nblk, int n, float* loss) {
  __shared__ float red[256];
  float s = 0.f;
  for (int b = threadIdx.x; b < nblk; b += 256) s += part[b];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = red[0] / (float)n;
}

template <int NCT>
__global__ __launch_bounds__(kTopThreads) void k_top_xent_bwd(TopArgs a) {
  extern __shared__ float smem[];
  float* sW = smem;                               // [K][Cp]
  float* sD = smem + a.K * a.Cp;                  // [waves][16][Cp]: dZ rows of each wave
  stage_w(a, sW);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int r0 = blockIdx.x * kTopRows + w * kTopRowsPerWave;
  float* dz = sD + w * kTopRowsPerWave * a.Cp;
  f32x4 z[NCT];
  wave_logits<NCT>(a, sW, r0, i, g, z);
  float lp[NCT][4], lp2[NCT][4];
  log_softmax2<NCT>(z, a.C, i, lp, lp2);
  const float gl = *a.grad / (float)a.n;
  // nll backward, then y = log_softmax(x): dx = dy - exp(y) * sum(dy), twice
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int r = r0 + 4 * g + v;
    const int t = r < a.n ? (int)a.labels[r] : -1;
    float d2[NCT], s2 = 0.f;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      d2[ct] = (16 * ct + i == t) ? -gl : 0.f;
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
      dz[(4 * g + v) * a.Cp + 16 * ct + i] = on ? d1[ct] - expf(lp[ct][v]) * s1 : 0.f;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's dZ stores landed
  __builtin_amdgcn_wave_barrier();
  // dY [16 x K] = dZ [16 x Cp] W^T: A lane (i,g) = dZ[i][c], B = W[k = 16 kt + i][c]
  for (int kt = 0; kt < a.K / 16; ++kt) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c0 = 0; c0 < 16 * NCT; c0 += 4) {
      const float av = dz[i * a.Cp + c0 + g];
      const float bv = sW[(16 * kt + i) * a.Cp + c0 + g];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int r = r0 + 4 * g + v;
      if (r < a.n) a.dY[(uint64_t)r * a.K + 16 * kt + i] = acc[v];
    }
  }
  // dW partial [K x Cp] = Y^T [K x 16] dZ [16 x Cp]:
  //   A lane (i,g) = Y[r0 + 4s + g][16 kt + i], B = dZ[4s + g][16 ct + i]
  float* pw = a.part + ((uint64_t)blockIdx.x * kTopWaves + w) * a.K * a.C;
  for (int kt = 0; kt < a.K / 16; ++kt) {
    f32x4 acc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int r = r0 + 4 * s + g;
      const float av = r < a.n ? a.Y[(uint64_t)r * a.ldy + 16 * kt + i] : 0.f;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, dz[(4 * s + g) * a.Cp + 16 * ct + i],
                                                       acc[ct], 0, 0, 0);
    }
    // acc[ct][v] = dW[16 kt + 4 g + v][16 ct + i]
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int c = 16 * ct + i;
        if (c < a.C) pw[(uint64_t)(16 * kt + 4 * g + v) * a.C + c] = acc[ct][v];
      }
  }
}

static size_t top_lds(int K, int Cp, bool bwd) {
  return ((size_t)K * Cp + (bwd ? (size_t)kTopRows * Cp : 0)) * sizeof(float);
}

template <int NCT>
static int launch_top(hipStream_t st, bool bwd, int nblk, size_t lds, const TopArgs& a) {
  if (bwd) {
    NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_top_xent_bwd<NCT>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_top_xent_bwd<NCT>, dim3(nblk), dim3(kTopThreads), lds, st, a);
  } else {
    NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_top_xent_fwd<NCT>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_top_xent_fwd<NCT>, dim3(nblk), dim3(kTopThreads), lds, st, a);
  }
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

static int launch_top_any(hipStream_t st, bool bwd, int nblk, size_t lds, const TopArgs& a) {
  switch (a.Cp / 16) {
    case 1: return launch_top<1>(st, bwd, nblk, lds, a);
    case 2: return launch_top<2>(st, bwd, nblk, lds, a);
    case 3: return launch_top<3>(st, bwd, nblk, lds, a);
    default: return launch_top<4>(st, bwd, nblk, lds, a);
  }
}

}  // namespace nts_hip

using namespace nts_hip;

extern "C" {

int nts_hip_linear_xent_fwd(nts_hip_ctx* ctx, const float* Y, uint64_t ldy, int n, int K,
                            const float* W, int C, const int64_t* labels, float* loss) {
  NTS_CHECK_ARG(ctx && Y && W && labels && loss, "NULL argument");
  NTS_CHECK_ARG(n > 0 && K > 0 && C > 0 && ldy >= (uint64_t)K, "shape");
  NTS_CHECK_ARG(C <= kWave, "class count above 64 is not supported by the fused loss");
  NTS_CHECK_ARG(K % 16 == 0, "the fused loss needs K % 16 == 0");
  const int Cp = (C + 15) / 16 * 16;
  const size_t lds = top_lds(K, Cp, true);
  NTS_CHECK_ARG(lds <= 160 * 1024, "K x C too large for the fused loss");
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  const int nblk = (n + kTopRows - 1) / kTopRows;
  NTS_RET(ensure_scratch(ctx, (size_t)nblk * sizeof(float) + 256));
  TopArgs a{Y, ldy, W, labels, nullptr, n, K, C, Cp, (float*)ctx->scratch, nullptr};
  NTS_RET(launch_top_any(ctx->stream, false, nblk, top_lds(K, Cp, false), a));
  hipLaunchKernelGGL(k_top_loss_reduce, dim3(1), dim3(256), 0, ctx->stream, a.part, nblk, n, loss);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

int nts_hip_linear_xent_bwd(nts_hip_ctx* ctx, const float* Y, uint64_t ldy, int n, int K,
                            const float* W, int C, const int64_t* labels, const float* grad_loss,
                            float* dY, float* dW) {
  NTS_CHECK_ARG(ctx && Y && W && labels && grad_loss && dY && dW, "NULL argument");
  NTS_CHECK_ARG(n > 0 && K > 0 && C > 0 && ldy >= (uint64_t)K, "shape");
  NTS_CHECK_ARG(C <= kWave, "class count above 64 is not supported by the fused loss");
  NTS_CHECK_ARG(K % 16 == 0, "the fused loss needs K % 16 == 0");
  const int Cp = (C + 15) / 16 * 16;
  const size_t lds = top_lds(K, Cp, true);
  NTS_CHECK_ARG(lds <= 160 * 1024, "K x C too large for the fused loss");
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  const int nblk = (n + kTopRows - 1) / kTopRows;
  const uint64_t slab = (uint64_t)K * C;
  const int nslab = nblk * kTopWaves;
  NTS_RET(ensure_scratch(ctx, (size_t)nslab * slab * sizeof(float) + 256));
  TopArgs a{Y, ldy, W, labels, grad_loss, n, K, C, Cp, (float*)ctx->scratch, dY};
  NTS_RET(launch_top_any(ctx->stream, true, nblk, lds, a));
  return sum_splits(ctx->stream, a.part, nslab, slab, K, C, dW, (uint64_t)C);
}

}  // extern "C"
