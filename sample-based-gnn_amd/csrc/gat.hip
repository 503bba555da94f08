// Sampled GAT layer (the reference's GAT_SAMPLE_ALL_GPU chain,
// toolkits/GAT_SAMPLE_ALL_GPU.hpp:308-391) fused into three kernels.
//
// Reference forward of one layer on a merged src/dst sampled block
// (core/ntsPushdownGraphOp.hpp:490-748, kernels cuda/ntsCUDADistKernel.cuh):
//   H     = X W                                   (Parameter::forward)
//   msg_e = [H[src_e], H[dst_local(d_e)]]         (BatchGPUSrcDstScatterOp)
//   m_e   = leaky_relu(msg_e . W_att, 0.2)        (edge NN, W_att [2F, 1])
//   a_e   = exp(m_e - max_d) / sum_d exp(...)     (BatchGPUEdgeSoftMax, :319-370)
//   Z_d   = sum_e a_e H[src_e]                    (e_msg * a, BatchGPUAggregateDst)
//   X'_d  = relu(Z_d)
// Here msg_e is never materialised: msg_e . W_att = H[src].a1 + H[dst].a2 with
// a1 = W_att[0:F], a2 = W_att[F:2F]; one wave per destination reads each
// neighbour row once and keeps an online softmax (running max / sum, the
// accumulator rescaled when the max grows).  Backward (all deterministic,
// no atomics):
//   k_gat_bwd_dst  per dst: g = G (.) [X' > 0] (stored: GM); ga_e = g . H[src_e];
//                  du_e = a_e (ga_e - sum a ga) * leaky'(m_e); ds2[dst_local(d)] = sum du_e
//   k_gat_bwd_src  per src v over the CSR: dH[v] = sum a_e g_{d_e} + ds1[v] a1 + ds2[v] a2,
//                  ds1[v] = sum du_e;  dS[v] = (ds1[v], ds2[v])
// and W_att.grad = H^T dS, W.grad = X^T dH, dX = dH W^T (layer GEMMs).
#include "common.hpp"

namespace nts_hip {

constexpr int kGatThreads = 256;  // 4 waves, one destination / source each
constexpr int kGatU = 4;          // neighbour rows in flight per wave

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

template <int VEC>
struct GV;
template <>
struct GV<1> {
  using T = float;
  __device__ static T zero() { return 0.f; }
  __device__ static float dot(T a, T b) { return a * b; }
  __device__ static T axpy(T acc, float w, T x) { return acc + w * x; }
  __device__ static T scale(T x, float s) { return x * s; }
  __device__ static T relu(T x) { return x > 0.f ? x : 0.f; }
  __device__ static T mask(T g, T y) { return y > 0.f ? g : 0.f; }
};
template <>
struct GV<4> {
  using T = float4;
  __device__ static T zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ static float dot(T a, T b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
  __device__ static T axpy(T acc, float w, T x) {
    return make_float4(acc.x + w * x.x, acc.y + w * x.y, acc.z + w * x.z, acc.w + w * x.w);
  }
  __device__ static T scale(T x, float s) { return make_float4(x.x * s, x.y * s, x.z * s, x.w * s); }
  __device__ static T relu(T x) {
    return make_float4(x.x > 0.f ? x.x : 0.f, x.y > 0.f ? x.y : 0.f, x.z > 0.f ? x.z : 0.f,
                       x.w > 0.f ? x.w : 0.f);
  }
  __device__ static T mask(T g, T y) {
    return make_float4(y.x > 0.f ? g.x : 0.f, y.y > 0.f ? g.y : 0.f, y.z > 0.f ? g.z : 0.f,
                       y.w > 0.f ? g.w : 0.f);
  }
};

__device__ __forceinline__ float leaky(float u) { return u > 0.f ? u : 0.2f * u; }

// ---- forward -----------------------------------------------------------------
template <int VEC, int NCH>
__global__ __launch_bounds__(kGatThreads) void k_gat_fwd(
    const uint32_t* __restrict__ co, const uint32_t* __restrict__ ri,
    const uint32_t* __restrict__ dl, uint32_t nv_dst, const float* __restrict__ H, uint64_t ldh,
    uint32_t nvec, const float* __restrict__ att, float* __restrict__ m_out,
    float* __restrict__ a_out, float* __restrict__ Y, uint64_t ldy) {
  using G = GV<VEC>;
  using T = typename G::T;
  const int lane = threadIdx.x & 63;
  const uint32_t d = blockIdx.x * (kGatThreads / 64) + (threadIdx.x >> 6);
  if (d >= nv_dst) return;
  const T* a1 = reinterpret_cast<const T*>(att);
  const T* a2 = reinterpret_cast<const T*>(att + (uint64_t)nvec * VEC);
  T w1[NCH], w2[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const uint32_t col = lane + 64 * c;
    w1[c] = col < nvec ? a1[col] : G::zero();
    w2[c] = col < nvec ? a2[col] : G::zero();
  }
  // score of the destination's own row
  const T* hd = reinterpret_cast<const T*>(H + (uint64_t)dl[d] * ldh);
  float p2 = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const uint32_t col = lane + 64 * c;
    if (col < nvec) p2 += G::dot(hd[col], w2[c]);
  }
  const float s2 = wave_sum(p2);
  const uint32_t beg = co[d], end = co[d + 1];
  T acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c] = G::zero();
  float M = -INFINITY, S = 0.f;
  for (uint32_t cb = beg; cb < end; cb += 64) {
    const uint32_t ne = min(end - cb, 64u);
    const uint32_t my_r = lane < (int)ne ? ri[cb + lane] : 0u;
    float my_m = 0.f;
    for (uint32_t j0 = 0; j0 < ne; j0 += kGatU) {  // kGatU neighbour rows in flight
      T x[kGatU][NCH];
      float p1[kGatU];
#pragma unroll
      for (int u = 0; u < kGatU; ++u) {
        const bool ok = j0 + u < ne;
        const uint32_t r = (uint32_t)__shfl((int)my_r, (int)min(j0 + u, ne - 1), 64);
        const T* hr = reinterpret_cast<const T*>(H + (uint64_t)r * ldh);
        p1[u] = 0.f;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const uint32_t col = lane + 64 * c;
          x[u][c] = (ok && col < nvec) ? hr[col] : G::zero();
          p1[u] += G::dot(x[u][c], w1[c]);
        }
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
        for (int u = 0; u < kGatU; ++u) p1[u] += __shfl_xor(p1[u], o, 64);
#pragma unroll
      for (int u = 0; u < kGatU; ++u) {
        if (j0 + u >= ne) break;
        const float m = leaky(p1[u] + s2);
        if (lane == (int)(j0 + u)) my_m = m;
        const float Mn = fmaxf(M, m);
        const float sc = expf(M - Mn);  // 0 for the first edge (M = -inf)
        const float p = expf(m - Mn);
        S = S * sc + p;
#pragma unroll
        for (int c = 0; c < NCH; ++c) acc[c] = G::axpy(G::scale(acc[c], sc), p, x[u][c]);
        M = Mn;
      }
    }
    if (lane < (int)ne) m_out[cb + lane] = my_m;
  }
  const float inv = S > 0.f ? 1.f / S : 0.f;
  T* y = reinterpret_cast<T*>(Y + (uint64_t)d * ldy);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const uint32_t col = lane + 64 * c;
    if (col < nvec) y[col] = G::relu(G::scale(acc[c], inv));
  }
  // attention coefficients (needed by the backward)
  for (uint32_t e = beg + lane; e < end; e += 64) a_out[e] = expf(m_out[e] - M) * inv;
}

// ---- backward, per destination ------------------------------------------------
template <int VEC, int NCH>
__global__ __launch_bounds__(kGatThreads) void k_gat_bwd_dst(
    const uint32_t* __restrict__ co, const uint32_t* __restrict__ ri,
    const uint32_t* __restrict__ dl, uint32_t nv_dst, const float* __restrict__ H, uint64_t ldh,
    uint32_t nvec, const float* __restrict__ a, const float* __restrict__ m,
    const float* __restrict__ Y, uint64_t ldy, const float* __restrict__ GY, uint64_t ldg,
    float* __restrict__ du, float* __restrict__ ds2, float* __restrict__ GM, uint64_t ldm) {
  using G = GV<VEC>;
  using T = typename G::T;
  const int lane = threadIdx.x & 63;
  const uint32_t d = blockIdx.x * (kGatThreads / 64) + (threadIdx.x >> 6);
  if (d >= nv_dst) return;
  const T* gy = reinterpret_cast<const T*>(GY + (uint64_t)d * ldg);
  const T* yy = reinterpret_cast<const T*>(Y + (uint64_t)d * ldy);
  T* gm = reinterpret_cast<T*>(GM + (uint64_t)d * ldm);
  T g[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const uint32_t col = lane + 64 * c;
    g[c] = col < nvec ? G::mask(gy[col], yy[col]) : G::zero();
    if (col < nvec) gm[col] = g[c];  // relu-masked gradient, read per edge by k_gat_bwd_src
  }
  const uint32_t beg = co[d], end = co[d + 1];
  // pass 1: ga_e = g . H[src_e] (kept by the lane owning e, chunk by chunk:
  // du needs sum_e a_e ga_e first, so ga is parked in du and rescaled below)
  float sag = 0.f;
  for (uint32_t cb = beg; cb < end; cb += 64) {
    const uint32_t ne = min(end - cb, 64u);
    const uint32_t my_r = lane < (int)ne ? ri[cb + lane] : 0u;
    float my_ga = 0.f;
    for (uint32_t j0 = 0; j0 < ne; j0 += kGatU) {
      float p[kGatU];
#pragma unroll
      for (int u = 0; u < kGatU; ++u) {
        const bool ok = j0 + u < ne;
        const uint32_t r = (uint32_t)__shfl((int)my_r, (int)min(j0 + u, ne - 1), 64);
        const T* hr = reinterpret_cast<const T*>(H + (uint64_t)r * ldh);
        p[u] = 0.f;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const uint32_t col = lane + 64 * c;
          if (ok && col < nvec) p[u] += G::dot(g[c], hr[col]);
        }
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
        for (int u = 0; u < kGatU; ++u) p[u] += __shfl_xor(p[u], o, 64);
#pragma unroll
      for (int u = 0; u < kGatU; ++u)
        if (lane == (int)(j0 + u)) my_ga = p[u];
    }
    if (lane < (int)ne) {
      du[cb + lane] = my_ga;
      sag += a[cb + lane] * my_ga;
    }
  }
  sag = wave_sum(sag);
  // pass 2: softmax and leaky_relu backward
  float s = 0.f;
  for (uint32_t e = beg + lane; e < end; e += 64) {
    const float dm = a[e] * (du[e] - sag);
    const float u = m[e] > 0.f ? dm : 0.2f * dm;
    du[e] = u;
    s += u;
  }
  s = wave_sum(s);
  if (lane == 0) ds2[dl[d]] = s;
}

// ---- backward, per source (CSR) ------------------------------------------------
template <int VEC, int NCH>
__global__ __launch_bounds__(kGatThreads) void k_gat_bwd_src(
    const uint32_t* __restrict__ ro, const uint32_t* __restrict__ ci,
    const uint32_t* __restrict__ ceid, uint32_t nv_src, uint32_t nvec,
    const float* __restrict__ a, const float* __restrict__ du, const float* __restrict__ ds2,
    const float* __restrict__ att, const float* __restrict__ GM, uint64_t ldm,
    float* __restrict__ dH, uint64_t lddh, float* __restrict__ dS) {
  using G = GV<VEC>;
  using T = typename G::T;
  const int lane = threadIdx.x & 63;
  const uint32_t v = blockIdx.x * (kGatThreads / 64) + (threadIdx.x >> 6);
  if (v >= nv_src) return;
  const uint32_t beg = ro[v], end = ro[v + 1];
  T acc[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c] = G::zero();
  float s1 = 0.f;
  for (uint32_t cb = beg; cb < end; cb += 64) {
    const uint32_t ne = min(end - cb, 64u);
    uint32_t my_d = 0;
    float my_a = 0.f, my_u = 0.f;
    if (lane < (int)ne) {
      const uint32_t eid = ceid[cb + lane];
      my_d = ci[cb + lane];
      my_a = a[eid];
      my_u = du[eid];
    }
    s1 += my_u;
    for (uint32_t j0 = 0; j0 < ne; j0 += kGatU) {
      T x[kGatU][NCH];
      float w[kGatU];
#pragma unroll
      for (int u = 0; u < kGatU; ++u) {
        const bool ok = j0 + u < ne;
        const int jj = (int)min(j0 + u, ne - 1);
        const uint32_t dd = (uint32_t)__shfl((int)my_d, jj, 64);
        w[u] = ok ? __shfl(my_a, jj, 64) : 0.f;
        const T* gm = reinterpret_cast<const T*>(GM + (uint64_t)dd * ldm);
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const uint32_t col = lane + 64 * c;
          x[u][c] = (ok && col < nvec) ? gm[col] : G::zero();
        }
      }
#pragma unroll
      for (int u = 0; u < kGatU; ++u)
        if (j0 + u < ne) {  // edge order kept
#pragma unroll
          for (int c = 0; c < NCH; ++c) acc[c] = G::axpy(acc[c], w[u], x[u][c]);
        }
    }
  }
  s1 = wave_sum(s1);
  const float s2 = ds2[v];
  const T* a1 = reinterpret_cast<const T*>(att);
  const T* a2 = reinterpret_cast<const T*>(att + (uint64_t)nvec * VEC);
  T* out = reinterpret_cast<T*>(dH + (uint64_t)v * lddh);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const uint32_t col = lane + 64 * c;
    if (col < nvec) out[col] = G::axpy(G::axpy(acc[c], s1, a1[col]), s2, a2[col]);
  }
  if (lane == 0) {
    dS[2 * (uint64_t)v] = s1;
    dS[2 * (uint64_t)v + 1] = s2;
  }
}

static bool gat_vec4(uint32_t F, uint64_t l1, uint64_t l2, const void* p1, const void* p2,
                     const void* att) {
  return F % 4 == 0 && l1 % 4 == 0 && l2 % 4 == 0 && ((uintptr_t)p1 % 16) == 0 &&
         ((uintptr_t)p2 % 16) == 0 && ((uintptr_t)att % 16) == 0;
}

}  // namespace nts_hip

using namespace nts_hip;

#define NTS_GAT_DISPATCH(KERNEL, ARGS)                                                   \
  do {                                                                                   \
    const uint32_t nvec = v4 ? F / 4 : F;                                                \
    const int nch = (int)((nvec + 63) / 64);                                             \
    NTS_CHECK_ARG(nch <= 4, "feature width too large (<= 1024 with float4, 256 else)"); \
    const dim3 grid(std::max(1u, ceil_div(n, kGatThreads / 64)));                        \
    if (v4) {                                                                            \
      switch (nch) {                                                                     \
        case 1: hipLaunchKernelGGL((KERNEL<4, 1>), grid, dim3(kGatThreads), 0, st, ARGS); break; \
        case 2: hipLaunchKernelGGL((KERNEL<4, 2>), grid, dim3(kGatThreads), 0, st, ARGS); break; \
        case 3: hipLaunchKernelGGL((KERNEL<4, 3>), grid, dim3(kGatThreads), 0, st, ARGS); break; \
        default: hipLaunchKernelGGL((KERNEL<4, 4>), grid, dim3(kGatThreads), 0, st, ARGS); break; \
      }                                                                                  \
    } else {                                                                             \
      switch (nch) {                                                                     \
        case 1: hipLaunchKernelGGL((KERNEL<1, 1>), grid, dim3(kGatThreads), 0, st, ARGS); break; \
        case 2: hipLaunchKernelGGL((KERNEL<1, 2>), grid, dim3(kGatThreads), 0, st, ARGS); break; \
        case 3: hipLaunchKernelGGL((KERNEL<1, 3>), grid, dim3(kGatThreads), 0, st, ARGS); break; \
        default: hipLaunchKernelGGL((KERNEL<1, 4>), grid, dim3(kGatThreads), 0, st, ARGS); break; \
      }                                                                                  \
    }                                                                                    \
    NTS_LAUNCH_CHECK();                                                                  \
  } while (0)

extern "C" {

int nts_hip_gat_forward(nts_hip_ctx* ctx, const uint32_t* column_offset,
                        const uint32_t* row_indices, const uint32_t* dst_local_id,
                        uint32_t v_size, const float* H, uint64_t ldh, uint32_t F,
                        const float* att, float* m_out, float* a_out, float* Y, uint64_t ldy) {
  NTS_CHECK_ARG(ctx && column_offset && row_indices && dst_local_id && H && att && m_out &&
                    a_out && Y,
                "NULL argument");
  NTS_CHECK_ARG(ldh >= F && ldy >= F, "leading dimension");
  if (v_size == 0 || F == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  const hipStream_t st = ctx->stream;
  const bool v4 = gat_vec4(F, ldh, ldy, H, Y, att);
  const uint32_t n = v_size;
#define ARGS column_offset, row_indices, dst_local_id, v_size, H, ldh, nvec, att, m_out, a_out, Y, ldy
  NTS_GAT_DISPATCH(k_gat_fwd, ARGS);
#undef ARGS
  return NTS_OK;
}

int nts_hip_gat_backward(nts_hip_ctx* ctx, const uint32_t* column_offset,
                         const uint32_t* row_indices, const uint32_t* dst_local_id,
                         uint32_t v_size, const uint32_t* row_offset,
                         const uint32_t* column_indices, const uint32_t* csr_edge_id,
                         uint32_t src_size, const float* H, uint64_t ldh, uint32_t F,
                         const float* att, const float* a, const float* m, const float* Y,
                         uint64_t ldy, const float* GY, uint64_t ldg, float* du, float* ds2,
                         float* GM, uint64_t ldm, float* dH, uint64_t lddh, float* dS) {
  NTS_CHECK_ARG(ctx && column_offset && row_indices && dst_local_id && row_offset &&
                    column_indices && csr_edge_id && H && att && a && m && Y && GY && du &&
                    ds2 && GM && dH && dS,
                "NULL argument");
  NTS_CHECK_ARG(ldm >= F, "leading dimension of GM");
  NTS_CHECK_ARG(ldh >= F && ldy >= F && ldg >= F && lddh >= F, "leading dimension");
  if (F == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  const hipStream_t st = ctx->stream;
  if (src_size) NTS_HIP_TRY(hipMemsetAsync(ds2, 0, (size_t)src_size * sizeof(float), st));
  const bool v4 = gat_vec4(F, ldh, ldy, H, Y, att) && ldg % 4 == 0 && lddh % 4 == 0 &&
                  ldm % 4 == 0 && ((uintptr_t)GY % 16) == 0 && ((uintptr_t)dH % 16) == 0 &&
                  ((uintptr_t)GM % 16) == 0;
  if (v_size) {
    const uint32_t n = v_size;
#define ARGS column_offset, row_indices, dst_local_id, v_size, H, ldh, nvec, a, m, Y, ldy, GY, ldg, du, ds2, GM, ldm
    NTS_GAT_DISPATCH(k_gat_bwd_dst, ARGS);
#undef ARGS
  }
  if (src_size) {
    const uint32_t n = src_size;
#define ARGS row_offset, column_indices, csr_edge_id, src_size, nvec, a, du, ds2, att, GM, ldm, dH, lddh, dS
    NTS_GAT_DISPATCH(k_gat_bwd_src, ARGS);
#undef ARGS
  }
  return NTS_OK;
}

}  // extern "C"
