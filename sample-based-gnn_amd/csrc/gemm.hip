// fp32 GEMMs of the GCN layer update on the matrix cores (v_mfma_f32_32x32x2_f32,
// exact fp32 products, fp32 accumulate).
//
// The layer GEMMs are tall-skinny: Z = Y W with Y [~150K x 602], W [602 x 128]
// (Parameter::forward, core/NtsScheduler.hpp:859-862) and the weight gradient
// dW = Y^T dZ (reduction over the ~150K sampled rows).  Library kernels run
// these at ~40 TF/s; here the tiles are shaped for them:
//   NN: block 128 rows x 128 cols, 4 waves of 32 rows x 4 MFMA tiles; A rows
//       are read straight into registers (16 consecutive k per lane — the k
//       order inside an MFMA step is a free permutation shared by A and B),
//       the B k-slice [32 x 128] is staged in LDS (double buffered) and shared
//       by the 4 waves.
//   TN: C = A^T B with the long reduction split over blocks; per-split
//       partial tiles are summed in split order by a second kernel
//       (deterministic, no atomics).
#include "common.hpp"

namespace nts_hip {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kGT = 256;   // threads per block
constexpr int kBM = 128;   // block rows (4 waves x 32)
constexpr int kBN = 128;   // block cols (4 MFMA tiles of 32)
constexpr int kBK = 32;    // k per step (16 MFMA 32x32x2 steps)

// Stage B[k0 .. k0+32) x [n0 .. n0+128) (row-major, ldb) into LDS.
// Each thread moves 16 consecutive floats of one k-row.
template <bool BVEC>
__device__ __forceinline__ void load_b_slice(const float* __restrict__ B, uint64_t ldb, int K,
                                             int N, int k0, int n0, float (&v)[16]) {
  const int kk = threadIdx.x >> 3;
  const int c = (threadIdx.x & 7) * 16;
  const int k = k0 + kk;
  const float* row = B + (uint64_t)k * ldb;
  if (BVEC) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int col = n0 + c + 4 * q;
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < K && col < N) x = *reinterpret_cast<const float4*>(row + col);
      v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int col = n0 + c + q;
      v[q] = (k < K && col < N) ? row[col] : 0.f;
    }
  }
}

__device__ __forceinline__ void store_b_slice(float (*Bs)[kBN], const float (&v)[16]) {
  const int kk = threadIdx.x >> 3;
  const int c = (threadIdx.x & 7) * 16;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    *reinterpret_cast<float4*>(&Bs[kk][c + 4 * q]) =
        make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}

// 16 A values of this lane for the k-step at k0:
//   NN (TRANS_A=false): A[row][k0 + 16h + s]       (row-major M x K)
//   TN (TRANS_A=true):  A[k0 + 16h + s][row]       (row-major K x M)
template <bool TRANS_A, int AVEC>
__device__ __forceinline__ void load_a(const float* __restrict__ A, uint64_t lda, int M, int K,
                                       int64_t row, int k0, int h, float (&a)[16]) {
  const int kb = k0 + 16 * h;
  if (!TRANS_A) {
    const bool ok = row < M;
    const float* p = A + (uint64_t)row * lda + kb;
    if (AVEC == 2) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float2 x = make_float2(0.f, 0.f);
        if (ok && kb + 2 * q < K) x = *reinterpret_cast<const float2*>(p + 2 * q);
        a[2 * q] = x.x;
        a[2 * q + 1] = x.y;
      }
    } else if (AVEC == 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok && kb + 4 * q < K) x = *reinterpret_cast<const float4*>(p + 4 * q);
        a[4 * q] = x.x; a[4 * q + 1] = x.y; a[4 * q + 2] = x.z; a[4 * q + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int s = 0; s < 16; ++s) a[s] = (ok && kb + s < K) ? p[s] : 0.f;
    }
  } else {
    const bool ok = row < M;
#pragma unroll
    for (int s = 0; s < 16; ++s)
      a[s] = (ok && kb + s < K) ? A[(uint64_t)(kb + s) * lda + row] : 0.f;
  }
}

// C_tile = op(A) B over k in [kbeg, kend); result written to C (ldc) or to a
// partial slab.  grid: x = M tiles, y = N tiles, z = k splits.
template <bool TRANS_A, int AVEC, bool BVEC>
__global__ __launch_bounds__(kGT) void k_gemm(int M, int N, int K, const float* __restrict__ A,
                                              uint64_t lda, const float* __restrict__ B,
                                              uint64_t ldb, float* __restrict__ C, uint64_t ldc,
                                              int kchunk, uint64_t split_stride) {
  __shared__ float Bs[2][kBK][kBN];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t row = (int64_t)blockIdx.x * kBM + w * 32 + r;
  const int n0 = blockIdx.y * kBN;
  const int kbeg = blockIdx.z * kchunk;
  const int kend = min(K, kbeg + kchunk);
  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  float a[16], bv[16];
  if (kbeg < kend) {
    load_a<TRANS_A, AVEC>(A, lda, M, kend, row, kbeg, h, a);
    load_b_slice<BVEC>(B, ldb, kend, N, kbeg, n0, bv);
    store_b_slice(Bs[0], bv);
  }
  __syncthreads();
  int buf = 0;
  for (int k0 = kbeg; k0 < kend; k0 += kBK) {
    const bool more = k0 + kBK < kend;
    float an[16];
    if (more) {
      load_a<TRANS_A, AVEC>(A, lda, M, kend, row, k0 + kBK, h, an);
      load_b_slice<BVEC>(B, ldb, kend, N, k0 + kBK, n0, bv);
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float b = Bs[buf][16 * h + s][32 * t + r];
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b, acc[t], 0, 0, 0);
      }
    }
    if (more) {
      store_b_slice(Bs[buf ^ 1], bv);
#pragma unroll
      for (int s = 0; s < 16; ++s) a[s] = an[s];
    }
    __syncthreads();
    buf ^= 1;
  }
  // epilogue: acc[t][i] -> (row = 8*(i>>2) + 4*h + (i&3), col = 32t + r) of the wave tile
  float* Cb = C + (uint64_t)blockIdx.z * split_stride;
  const int64_t wrow0 = (int64_t)blockIdx.x * kBM + w * 32;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int col = n0 + 32 * t + r;
    if (col >= N) continue;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int64_t rr = wrow0 + 8 * (i >> 2) + 4 * h + (i & 3);
      if (rr < M) Cb[(uint64_t)rr * ldc + col] = acc[t][i];
    }
  }
}

// C = sum over splits of the partial slabs (in split order)
__global__ void k_sum_splits(const float* __restrict__ part, int splits, uint64_t stride, int M,
                             int N, float* __restrict__ C, uint64_t ldc) {
  const uint64_t total = (uint64_t)M * N;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (uint64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += part[(uint64_t)z * stride + i];
    C[(i / N) * ldc + (i % N)] = s;
  }
}

template <bool TRANS_A>
static int launch(hipStream_t st, int M, int N, int K, const float* A, uint64_t lda,
                  const float* B, uint64_t ldb, float* C, uint64_t ldc, int splits, int kchunk,
                  uint64_t split_stride) {
  dim3 grid(ceil_div(M, kBM), ceil_div(N, kBN), splits);
  const bool bvec = (N % 4 == 0) && (ldb % 4 == 0) && ((uintptr_t)B % 16 == 0);
  int avec = 1;
  if (!TRANS_A) {
    if (K % 4 == 0 && lda % 4 == 0 && (uintptr_t)A % 16 == 0) avec = 4;
    else if (K % 2 == 0 && lda % 2 == 0 && (uintptr_t)A % 8 == 0) avec = 2;
  }
#define NTS_GEMM(AV, BV)                                                                        \
  hipLaunchKernelGGL((k_gemm<TRANS_A, AV, BV>), grid, dim3(kGT), 0, st, M, N, K, A, lda, B, ldb, \
                     C, ldc, kchunk, split_stride)
  if (avec == 4) { if (bvec) NTS_GEMM(4, true); else NTS_GEMM(4, false); }
  else if (avec == 2) { if (bvec) NTS_GEMM(2, true); else NTS_GEMM(2, false); }
  else { if (bvec) NTS_GEMM(1, true); else NTS_GEMM(1, false); }
#undef NTS_GEMM
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

}  // namespace nts_hip

using namespace nts_hip;

extern "C" int nts_hip_gemm_f32(nts_hip_ctx* ctx, int trans_a, int M, int N, int K,
                                const float* A, uint64_t lda, const float* B, uint64_t ldb,
                                float* C, uint64_t ldc) {
  NTS_CHECK_ARG(ctx && C, "NULL argument");
  NTS_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "negative size");
  if (M == 0 || N == 0) return NTS_OK;
  NTS_CHECK_ARG((A && B) || K == 0, "NULL operand");
  NTS_CHECK_ARG(ldb >= (uint64_t)N && ldc >= (uint64_t)N, "leading dimension");
  NTS_CHECK_ARG(trans_a ? lda >= (uint64_t)M : lda >= (uint64_t)K, "lda");
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  if (K == 0) {
    for (int i = 0; i < M; ++i) NTS_HIP_TRY(hipMemsetAsync(C + (uint64_t)i * ldc, 0, N * 4, st));
    return NTS_OK;
  }
  // split the reduction when the output grid alone cannot fill 256 CUs
  const int tiles = (int)(ceil_div(M, kBM) * ceil_div(N, kBN));
  int splits = 1;
  const int ksteps = (K + kBK - 1) / kBK;
  if (tiles < 512) splits = std::max(1, std::min(1024 / tiles, ksteps / 4));
  const int kchunk = ((ksteps + splits - 1) / splits) * kBK;
  splits = (K + kchunk - 1) / kchunk;
  if (splits == 1)
    return trans_a ? launch<true>(st, M, N, K, A, lda, B, ldb, C, ldc, 1, kchunk, 0)
                   : launch<false>(st, M, N, K, A, lda, B, ldb, C, ldc, 1, kchunk, 0);
  const uint64_t stride = (uint64_t)M * N;
  NTS_RET(ensure_scratch(ctx, stride * splits * sizeof(float) + 256));
  float* part = (float*)ctx->scratch;
  NTS_RET(trans_a ? launch<true>(st, M, N, K, A, lda, B, ldb, part, N, splits, kchunk, stride)
                  : launch<false>(st, M, N, K, A, lda, B, ldb, part, N, splits, kchunk, stride));
  const uint32_t g = std::max(1u, std::min(ceil_div(stride, 256), kMaxGrid));
  hipLaunchKernelGGL(k_sum_splits, dim3(g), dim3(256), 0, st, part, splits, stride, M, N, C, ldc);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}
