// fp32 layer GEMMs on the f16 matrix cores with two-piece operands
// (NTS_GEMM_H2): the transform-first bottom layer's row-gathered GEMMs.
//
// Every fp32 operand row (or column) is brought to a power-of-two scale s so
// that its largest |x| / s lies in [2^14, 2^15), and y = x / s (exact) is
// split into two fp16 pieces
//     y0 = f16(y),  y1 = f16(y - y0)            (round to nearest even)
// y - y0 is exact in fp32 and |y - y0| <= 2^-11 |y|, so y0 + y1 carries 22
// significant bits: |y - y0 - y1| <= 2^-23 |y| while y1 is a normal fp16
// (|y| >= 2^-2), and <= 2^-25 absolute below that, i.e. <= 2^-39 of the
// row's largest element.  A product a·b becomes the three f16 products
//     a0 b0 + a0 b1 + a1 b0           (dropped: a1 b1 <= 2^-22 |a b|)
// each exact in the fp32 accumulator of v_mfma_f32_16x16x32_f16, and the
// scales are applied to the fp32 result (exact: powers of two).  Three f16
// MFMAs per k-slice against six bf16 ones in gemm3.hip (NTS_GEMM_SPLIT3):
// the same fp32-level error bound up to a small constant (measured against
// fp64 in tests/test_gemm_h2.py), half the matrix-core work.
//
// The feature table is static, so its rows are pre-split once (at driver
// construction) into a "pair table": one 32-bit word per element, f16 y0 in
// the low half and y1 in the high half, rows zero-padded to a multiple of 32
// words, plus a row scale rs[r] (float, a power of two).  The word layout
// keeps the fp32 path's byte addresses: the NN kernel's A slabs are the same
// 16-byte global_load_lds pieces as k_gemm3_nn's, the TN kernel's A^T
// fragments the same dword loads as k_s3_tn's — and no split work is left in
// either loop.
//
// Kernels:
//   k_h2_split_rows  fp32 rows -> pair table + row scales (one wave per row)
//   k_colmax         per-column max |rs[row] * B[row, c]| (as float bits,
//                    atomicMax) — the column scales of W (NN) and of dH (TN)
//   k_h2_split_b     W [K x N] -> the NN kernel's two-piece fragment image
//   k_h2_nn          C = diag(rs[amap]) P[amap] W (+ relu/dropout epilogue)
//   k_h2_tn          C = P[amap]^T diag(rs[amap]) op(B) (weight gradient),
//                    op = B or the relu/dropout backward B * bscale where X > 0
#include "common.hpp"
#include <type_traits>

namespace nts_hip {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4h __attribute__((ext_vector_type(4)));
typedef short s16x4h __attribute__((ext_vector_type(4)));
typedef short s16x8h __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4h lds_s16x4h;
typedef __attribute__((address_space(3))) void* lds_ptr_h;

constexpr int kH2Frag = 64 * 16;  // one fragment image: 64 lanes x 8 f16

// scale exponent for a block whose largest magnitude is m: y = x * 2^e puts
// m * 2^e in [2^14, 2^15); the scale returned to the caller is 2^-e
__device__ __forceinline__ int h2_exp(float m) {
  if (!(m > 0.f) || !(m < INFINITY)) return 0;
  int e;
  (void)frexpf(m, &e);  // m = f * 2^e, f in [0.5, 1)
  return 15 - e;
}

__device__ __forceinline__ uint32_t h2_pair(float y) {
  const _Float16 h0 = (_Float16)y;
  const _Float16 h1 = (_Float16)(y - (float)h0);
  return (uint32_t)__builtin_bit_cast(uint16_t, h0) |
         ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
}

// 8 pair words -> the y0 and y1 fragment vectors (v_perm_b32 pairs)
__device__ __forceinline__ void h2_unpack(const uint32_t (&w)[8], f16x8& p0, f16x8& p1) {
  uint32_t lo[4], hi[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    lo[j] = __builtin_amdgcn_perm(w[2 * j + 1], w[2 * j], 0x05040100u);
    hi[j] = __builtin_amdgcn_perm(w[2 * j + 1], w[2 * j], 0x07060302u);
  }
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 a = {lo[0], lo[1], lo[2], lo[3]}, b = {hi[0], hi[1], hi[2], hi[3]};
  p0 = __builtin_bit_cast(f16x8, a);
  p1 = __builtin_bit_cast(f16x8, b);
}

// acc += a * b over one 32-deep k-slice (small products first)
__device__ __forceinline__ f32x4h mfma3(const f16x8 (&a)[2], const f16x8 (&b)[2], f32x4h acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}

// ---------------------------------------------------------------------------
// pair table: one wave per row
__global__ __launch_bounds__(256) void k_h2_split_rows(uint64_t R, uint32_t K, const float* __restrict__ X,
                                                      uint64_t ldx, uint32_t Kp, uint32_t* __restrict__ P,
                                                      uint64_t ldp, float* __restrict__ rs) {
  const uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= R) return;
  const float* x = X + r * ldx;
  float m = 0.f;
  for (uint32_t k = lane; k < K; k += 64) m = fmaxf(m, fabsf(x[k]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  const int e = h2_exp(m);
  uint32_t* p = P + r * ldp;
  for (uint32_t k = lane; k < Kp; k += 64) p[k] = k < K ? h2_pair(ldexpf(x[k], e)) : 0u;
  if (lane == 0) rs[r] = ldexpf(1.f, -e);
}

// planar pair table: per row the y0 plane (Kp f16), then the y1 plane
__global__ __launch_bounds__(256) void k_h2_split_rows_planar(uint64_t R, uint32_t K, const float* __restrict__ X,
                                                             uint64_t ldx, uint32_t Kp, uint16_t* __restrict__ Q,
                                                             uint64_t ldq, float* __restrict__ rs) {
  const uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= R) return;
  const float* x = X + r * ldx;
  float m = 0.f;
  for (uint32_t k = lane; k < K; k += 64) m = fmaxf(m, fabsf(x[k]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  const int e = h2_exp(m);
  uint16_t* q = Q + r * ldq;
  for (uint32_t k = lane; k < Kp; k += 64) {
    const uint32_t w = k < K ? h2_pair(ldexpf(x[k], e)) : 0u;
    q[k] = (uint16_t)(w & 0xFFFFu);
    q[Kp + k] = (uint16_t)(w >> 16);
  }
  if (lane == 0) {
    const float sc = ldexpf(1.f, -e);
    rs[r] = sc;
    if (ldq >= 2 * (uint64_t)Kp + 8) {  // a row tail: the scale rides along with the row
      const uint32_t b = __float_as_uint(sc);
      q[2 * Kp] = (uint16_t)(b & 0xFFFFu);
      q[2 * Kp + 1] = (uint16_t)(b >> 16);
    }
  }
}

// out[c] = max(out[c], max over rows k of |B[k, c]| * (rs ? rs[amap ? amap[k] : k] : 1)) as
// float bits (non-negative floats order like their bit patterns); out zeroed
// by the caller; rsg != NULL: rsg[k] = that row scale.  Thread t: column quad
// q = t % Q, row lane t / Q.
__global__ __launch_bounds__(256) void k_colmax(const float* __restrict__ B, uint64_t ldb, uint64_t K,
                                               int N, const float* __restrict__ rs,
                                               const uint32_t* __restrict__ amap, uint64_t rows_per_block,
                                               uint32_t* __restrict__ out, float* __restrict__ rsg) {
  __shared__ float red[256 * 4];
  const int Q = N / 4, RL = 256 / Q;
  const int t = threadIdx.x, q = t % Q, rl = t / Q;
  float m[4] = {0.f, 0.f, 0.f, 0.f};
  const uint64_t k0 = (uint64_t)blockIdx.x * rows_per_block;
  const uint64_t k1 = k0 + rows_per_block < K ? k0 + rows_per_block : K;
  if (rl < RL) {
    // four rows in flight per thread (the id -> scale gathers are dependent loads)
    for (uint64_t k = k0 + rl; k < k1; k += 4 * (uint64_t)RL) {
      float4 v[4];
      float sv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint64_t kk = k + (uint64_t)u * RL < k1 ? k + (uint64_t)u * RL : k1 - 1;
        v[u] = *reinterpret_cast<const float4*>(B + kk * ldb + 4 * q);
        sv[u] = rs ? fabsf(rs[amap ? amap[kk] : kk]) : 1.f;
        if (rsg && q == 0) rsg[kk] = sv[u];  // the row's scale, gathered once for the TN kernel
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        m[0] = fmaxf(m[0], fabsf(v[u].x) * sv[u]);
        m[1] = fmaxf(m[1], fabsf(v[u].y) * sv[u]);
        m[2] = fmaxf(m[2], fabsf(v[u].z) * sv[u]);
        m[3] = fmaxf(m[3], fabsf(v[u].w) * sv[u]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[4 * t + j] = m[j];
  __syncthreads();
  if (rl == 0) {
    for (int l = 1; l < RL; ++l)
#pragma unroll
      for (int j = 0; j < 4; ++j) m[j] = fmaxf(m[j], red[4 * (l * Q + q) + j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) atomicMax(out + 4 * q + j, __float_as_uint(m[j]));
  }
}

// ---------------------------------------------------------------------------
// B (W, [K x N]) -> img[s][cb][ct][piece][lane] (16 B) =
//   piece of W[32 s + 8 (lane >> 4) + j][128 cb + 16 ct + (lane & 15)] * 2^e(col)
// zero past K and N; cmax[col] = the column max bits (k_colmax).
constexpr int kH2Img = 8 * 2 * kH2Frag;  // one (step, column block) image: 16 KB

__global__ __launch_bounds__(256) void k_h2_split_b(const float* __restrict__ B, uint64_t ldb, int K,
                                                   int N, int total, int ncb,
                                                   const uint32_t* __restrict__ cmax,
                                                   char* __restrict__ out) {
  const int id = blockIdx.x * 256 + threadIdx.x;
  if (id >= total) return;
  const int lane = id & 63, ct = (id >> 6) & 7, rest = id >> 9;
  const int cb = rest % ncb, s = rest / ncb;
  const int col = cb * 128 + ct * 16 + (lane & 15);
  const int k0 = 32 * s + 8 * (lane >> 4);
  const int e = col < N ? h2_exp(__uint_as_float(cmax[col])) : 0;
  uint32_t w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    w[j] = (col < N && k0 + j < K) ? h2_pair(ldexpf(B[(uint64_t)(k0 + j) * ldb + col], e)) : 0u;
  f16x8 p0, p1;
  h2_unpack(w, p0, p1);
  char* dst = out + (size_t)rest * kH2Img + ct * 2 * kH2Frag + 16 * lane;
  *reinterpret_cast<f16x8*>(dst) = p0;
  *reinterpret_cast<f16x8*>(dst + kH2Frag) = p1;
}

// W's column maxima and its two-piece fragment image in one launch (the
// NN kernels' per-step weight preparation: one k-step x 128 columns per
// block; every block takes its columns' maxima over all K rows itself, block
// (0, cb) also stores them for the epilogue's column scales).  The fragment's
// own 8 values are loaded first (they do not depend on the maxima) and the
// maxima scan keeps 16 row loads in flight per thread: one memory round trip
// at K <= 256, three at K = 602 (was one per 64 rows plus one for the
// fragment: 19 us a call at C2, 15 us at C3's K = 100)
__global__ __launch_bounds__(512) void k_h2_prep_w(const float* __restrict__ B, uint64_t ldb, int K,
                                                  int N, uint32_t* __restrict__ cmax,
                                                  char* __restrict__ out) {
  __shared__ float red[16][128];
  __shared__ int sexp[128];
  const int s = blockIdx.x, cb = blockIdx.y, ncb = gridDim.y, tid = threadIdx.x;
  const int lane = tid & 63, ct = tid >> 6;
  const int cl = ct * 16 + (lane & 15), fcol = cb * 128 + cl;
  const int k0 = 32 * s + 8 * (lane >> 4);
  float raw[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    raw[j] = (fcol < N && k0 + j < K) ? B[(uint64_t)(k0 + j) * ldb + fcol] : 0.f;
  {  // thread: 4 columns (one float4), rows rl + 16 j, sixteen rows in flight
    constexpr int RF = 16;
    const int q = tid & 31, rl = tid >> 5, col = cb * 128 + 4 * q;
    float m[4] = {0.f, 0.f, 0.f, 0.f};
    if (col < N) {  // N % 16 == 0: the float4 is whole
      for (int k = rl; k < K; k += 16 * RF) {
        float4 v[RF];
#pragma unroll
        for (int u = 0; u < RF; ++u) {
          const int kk = min(k + 16 * u, K - 1);  // a clamped duplicate does not change a max
          v[u] = *reinterpret_cast<const float4*>(B + (uint64_t)kk * ldb + col);
        }
#pragma unroll
        for (int u = 0; u < RF; ++u) {
          m[0] = fmaxf(m[0], fabsf(v[u].x));
          m[1] = fmaxf(m[1], fabsf(v[u].y));
          m[2] = fmaxf(m[2], fabsf(v[u].z));
          m[3] = fmaxf(m[3], fabsf(v[u].w));
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) red[rl][4 * q + u] = m[u];
  }
  __syncthreads();
  if (tid < 128) {
    float m = 0.f;
#pragma unroll
    for (int l = 0; l < 16; ++l) m = fmaxf(m, red[l][tid]);
    sexp[tid] = h2_exp(m);
    if (s == 0 && cb * 128 + tid < N) cmax[cb * 128 + tid] = __float_as_uint(m);
  }
  __syncthreads();
  const int e = sexp[cl];
  uint32_t w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = (fcol < N && k0 + j < K) ? h2_pair(ldexpf(raw[j], e)) : 0u;
  f16x8 p0, p1;
  h2_unpack(w, p0, p1);
  char* dst = out + ((size_t)s * ncb + cb) * kH2Img + ct * 2 * kH2Frag + 16 * lane;
  *reinterpret_cast<f16x8*>(dst) = p0;
  *reinterpret_cast<f16x8*>(dst + kH2Frag) = p1;
}

// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lds_addr_h(const void* p) {
  return (uint32_t)(uintptr_t)(lds_ptr_h)p;
}
// 16 bytes per lane from `src` to LDS (wave-uniform base `lds`) + 16 * lane
// (inline asm: see gemm3.hip — a compiler-visible LDS DMA drains the pipeline)
__device__ __forceinline__ void glds16h(const void* src, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}
__device__ __forceinline__ void raw_barrier_h() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// CUs the one-block-per-CU pair-table GEMMs spread over (k_h2_nn3/4 row
// tiles, k_h2_tn4 k-chunks, k_h2_nnd tiles): 256, or NTS_GEMM_CUS (A/B: a grid
// below the CU count leaves CUs to the pipelined sampler's blocks instead of
// waiting for them)
static int gemm_cus() {  // compile-time A/B: -DNTS_GEMM_CUS=n
#ifdef NTS_GEMM_CUS
  return NTS_GEMM_CUS > 0 && NTS_GEMM_CUS <= 256 ? NTS_GEMM_CUS : 256;
#else
  return 256;
#endif
}

struct H2Extra {
  uint32_t keep_threshold = 0;  // EPI: relu + inverted dropout (common.hpp dropout_*)
  float scale = 1.f;
  uint64_t seed = 0, offset = 0;
  const uint32_t* amap = nullptr;  // gathered A rows (NN: M rows, TN: K rows)
  const float* rs = nullptr;       // row scales of the pair table
  const uint32_t* cmax = nullptr;  // column max bits (W for NN, rs * op(B) for TN)
  const float* rsg = nullptr;      // TN v2: the B rows' scales rs[amap[k]], gathered
  // TN v4: per-part column maxima of |B| (part p = B rows [p rpp, (p+1) rpp),
  // N words per part; nts_hip_spmm_csr_bwd_colmax) instead of the pre-pass
  const uint32_t* cparts = nullptr;
  uint32_t rpp = 0;
  uint64_t nparts_ld = 0;  // words per part (>= N)
  const float* bx = nullptr;       // TN BMASK: op(B) = B * bscale where X > 0
  uint64_t ldbx = 0;
  float bscale = 1.f;
};

// NN.  The structure of k_gemm3_nn (gemm3.hip): 8 waves, one column block of
// 128 per grid.y, 16-row tiles two at a time per wave, B's image (2 pieces,
// 16 KB per step, 2 stages) and A's pair slabs (3 stages) by global_load_lds,
// counted vmcnt waits and raw barriers.  K is the pair table's padded width
// (a multiple of 32: no partial step).  Per step and row tile: 8 column tiles
// x 3 MFMAs.  Epilogue: rs[row] * 2^-e(col) * acc, then relu/dropout.
constexpr int kH2NnThreads = 512;
constexpr int kH2NnAWave = 2 * 2048;
constexpr int kH2NnA = 8 * kH2NnAWave;
constexpr int kH2NnLds = 2 * kH2Img + 3 * kH2NnA;  // 32 + 96 KB

template <bool EPI, bool AMAP>
__global__ __launch_bounds__(kH2NnThreads, 1) void k_h2_nn(int M, int N, int K,
                                                          const uint32_t* __restrict__ A, uint64_t lda,
                                                          const char* __restrict__ bimg,
                                                          float* __restrict__ C, uint64_t ldc, int rounds,
                                                          H2Extra ex) {
  extern __shared__ __attribute__((aligned(16))) char h2nn[];
  char* const sb = h2nn;
  char* const sa = h2nn + 2 * kH2Img;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.y * 128;
  const int T = (M + 15) / 16;
  const int64_t W = (int64_t)gridDim.x * 8;
  const int64_t gw = (int64_t)blockIdx.x * 8 + wv;
  const int t_lo = (int)(gw * T / W), t_hi = (int)((gw + 1) * T / W);
  const int nsteps = K / 32;
  const size_t bstride = (size_t)gridDim.y * kH2Img;
  const uint32_t lsb = lds_addr_h(sb), lsa = lds_addr_h(sa);
  const char* bsrc = bimg + (size_t)blockIdx.y * kH2Img + wv * 1024 + 16 * lane;
  const int gr = (lane >> 1) & 15, gpo = 8 * (lane >> 5) + 4 * (lane & 1);
  const uint32_t* arow[2];
  auto set_rows = [&](int rd) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int t = min(t_lo + 2 * rd + rt, T - 1);
      const int64_t row = (int64_t)t * 16 + gr;
      const uint64_t rr = (uint64_t)(row < M ? row : M - 1);
      arow[rt] = A + (AMAP ? (uint64_t)ex.amap[rr] : rr) * lda + gpo;
    }
  };
  auto issue_b = [&](int s) {
    const uint32_t dst = lsb + (s & 1) * kH2Img + wv * 1024;
    const char* src = bsrc + (size_t)s * bstride;
#pragma unroll
    for (int p = 0; p < 2; ++p) glds16h(src + 8192 * p, dst + 8192 * p);
  };
  auto issue_a = [&](int s) {
    const uint32_t dst = lsa + (s % 3) * kH2NnA + wv * kH2NnAWave;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int q = 0; q < 2; ++q) glds16h(arow[rt] + 32 * s + 16 * q, dst + rt * 2048 + q * 1024);
  };
  f32x4h acc[2][8];
  for (int rd = 0; rd < rounds; ++rd) {
    const int nt = min(2, max(0, t_hi - (t_lo + 2 * rd)));
    set_rows(rd);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) acc[rt][ct] = f32x4h{0.f, 0.f, 0.f, 0.f};
    issue_b(0);
    if (nsteps > 0) issue_a(0);
    if (nsteps > 1) issue_a(1);
    for (int s = 0; s < nsteps; ++s) {
      // B(s) and A(s) landed (A(s+1), issued after B(s), may stay in flight):
      // per step a wave issues 2 (B) + 4 (A) pieces
      if (s + 1 < nsteps) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      raw_barrier_h();
      if (s + 1 < nsteps) issue_b(s + 1);
      if (s + 2 < nsteps) issue_a(s + 2);
      if (nt == 0) continue;
      const char* as = sa + (s % 3) * kH2NnA + wv * kH2NnAWave + 32 * (i + 16 * g);
      f16x8 a[2][2];
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const uint4 u = *reinterpret_cast<const uint4*>(as + rt * 2048);
        const uint4 v = *reinterpret_cast<const uint4*>(as + rt * 2048 + 16);
        const uint32_t w[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
        h2_unpack(w, a[rt][0], a[rt][1]);
      }
      const char* img = sb + (s & 1) * kH2Img;
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
        f16x8 b[2];
        b[0] = *reinterpret_cast<const f16x8*>(img + ct * 2 * kH2Frag + 16 * lane);
        b[1] = *reinterpret_cast<const f16x8*>(img + ct * 2 * kH2Frag + kH2Frag + 16 * lane);
        acc[0][ct] = mfma3(a[0], b, acc[0][ct]);
        if (nt == 2) acc[1][ct] = mfma3(a[1], b, acc[1][ct]);
      }
    }
    raw_barrier_h();
    // acc[rt][ct][v] = C[16 t + 4 g + v][n0 + 16 ct + i]
    float cs[8];
#pragma unroll
    for (int ct = 0; ct < 8; ++ct) {
      const int col = n0 + 16 * ct + i;
      cs[ct] = col < N ? ldexpf(1.f, -h2_exp(__uint_as_float(ex.cmax[col]))) : 0.f;
    }
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      if (rt >= nt) continue;
      const int64_t r4 = (int64_t)(t_lo + 2 * rd + rt) * 16 + 4 * g;
      float rsv[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const uint64_t rr = (uint64_t)(r4 + v < M ? r4 + v : M - 1);
        rsv[v] = ex.rs[AMAP ? (uint64_t)ex.amap[rr] : rr];
      }
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
        const uint32_t col = (uint32_t)(n0 + 16 * ct + i);
        if ((int)col >= N) continue;
        float o[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) o[v] = acc[rt][ct][v] * cs[ct] * rsv[v];
        if constexpr (EPI) {
          const uint4 rnd = dropout_words((uint64_t)r4, col, ex.seed, ex.offset);
          const uint32_t wd[4] = {rnd.x, rnd.y, rnd.z, rnd.w};
#pragma unroll
          for (int v = 0; v < 4; ++v)
            o[v] = (dropout_bits(wd[v], col) >= ex.keep_threshold && o[v] > 0.f) ? o[v] * ex.scale : 0.f;
        }
#pragma unroll
        for (int v = 0; v < 4; ++v)
          if (r4 + v < M) C[(uint64_t)(r4 + v) * ldc + col] = o[v];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// TN: C[M x N] = A[K x M]^T diag(rs) op(B)[K x N], A the pair table (K rows
// through the map, M <= its width), the structure of k_s3_tn (gemm3.hip): an
// 8-wave block takes one k-chunk, up to 8 x TPW column tiles of A and 128
// columns of B; A^T fragments are pair words loaded straight to registers (two
// steps ahead) and unpacked there; B rows are loaded 8 floats per thread,
// multiplied by their row's scale rs[amap[k]] and by 2^e(col) from the
// column max, split into two f16 pieces and written to LDS (XOR-swizzled
// 256-byte rows), read back transposed by ds_read_b64_tr_b16.  Partials are
// scaled by 2^-e(col) and summed in a fixed order (sum_splits).
constexpr int kH2TnThreads = 512;
constexpr int kH2TnImg = 32 * 256;            // one piece of one step: 32 rows x 128 f16
constexpr int kH2TnLds = 2 * 2 * kH2TnImg;    // 2 stages x 2 pieces = 32 KB

__device__ __forceinline__ int h2_tr_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

template <int TPW, bool BMASK, bool AMAP>
__global__ __launch_bounds__(kH2TnThreads, 1) void k_h2_tn(int M, int N, int K,
                                                          const uint32_t* __restrict__ A, uint64_t lda,
                                                          const float* __restrict__ B, uint64_t ldb,
                                                          float* __restrict__ C, uint64_t ldc, int kchunk,
                                                          uint64_t split_stride, int nmb, int nnb,
                                                          H2Extra ex) {
  extern __shared__ __attribute__((aligned(16))) char h2tn[];  // [2][2][kH2TnImg]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, g = lane >> 4;
  const int mb = blockIdx.x % nmb;
  const int nb = (blockIdx.x / nmb) % nnb;
  const int split = blockIdx.x / (nmb * nnb);
  const int n0 = nb * 128;
  const int T = (M + 15) / 16;
  const int b_lo = mb * T / nmb, b_cnt = (mb + 1) * T / nmb - b_lo;
  const int w_lo = b_lo + wv * b_cnt / 8, w_hi = b_lo + (wv + 1) * b_cnt / 8;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int nsteps = kbeg < kend ? (kend - kbeg + 31) / 32 : 0;

  int acol[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) acol[t] = min(16 * min(w_lo + t, max(w_hi - 1, w_lo)) + i, M - 1);
  // B staging role: row br = tid >> 4 of the step, columns bc .. bc + 7
  const int br = tid >> 4, bc = 8 * (tid & 15);
  const bool bok = n0 + bc < N;  // N % 16 == 0
  const float* bcol = B + (bok ? n0 + bc : 0);
  const float* xcol = BMASK ? ex.bx + (bok ? n0 + bc : 0) : nullptr;
  // column exponent: from the max of |rs * B| (times bscale for the masked
  // operand, an upper bound of |rs * op(B)|)
  auto col_exp = [&](int col) {
    float m = __uint_as_float(ex.cmax[col]);
    if constexpr (BMASK) m *= ex.bscale;
    return h2_exp(m);
  };
  int bexp[8];  // 2^e(col) of this thread's 8 B columns
#pragma unroll
  for (int u = 0; u < 8; ++u) bexp[u] = bok ? col_exp(n0 + bc + u) : 0;

  f32x4h acc[TPW][8];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int ct = 0; ct < 8; ++ct) acc[t][ct] = f32x4h{0.f, 0.f, 0.f, 0.f};
  uint32_t rid[2][8];
  uint32_t xa[TPW][8];
  f16x8 pa[TPW][2];
  float4 braw[2], xraw[BMASK ? 2 : 1];
  float brs = 0.f;

  auto load_ids = [&](int s, uint32_t (&r)[8]) {
    const int k0 = kbeg + 32 * s + 8 * g;
    if constexpr (AMAP) {
      if (k0 + 8 <= kend) {
        const uint4 u0 = *reinterpret_cast<const uint4*>(ex.amap + k0);
        const uint4 u1 = *reinterpret_cast<const uint4*>(ex.amap + k0 + 4);
        r[0] = u0.x; r[1] = u0.y; r[2] = u0.z; r[3] = u0.w;
        r[4] = u1.x; r[5] = u1.y; r[6] = u1.z; r[7] = u1.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = ex.amap[min(k0 + j, kend - 1)];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = (uint32_t)min(k0 + j, kend - 1);
    }
  };
  auto load_x = [&](int s, const uint32_t (&r)[8], int t) {
    const int k0 = kbeg + 32 * s + 8 * g;
#pragma unroll
    for (int j = 0; j < 8; ++j) xa[t][j] = A[(uint64_t)r[j] * lda + acol[t]];
    if (k0 + 8 > kend) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (k0 + j >= kend) xa[t][j] = 0u;
    }
  };
  auto load_b = [&](int s) {
    const int k = min(kbeg + 32 * s + br, kend - 1);
    const float4* p = reinterpret_cast<const float4*>(bcol + (uint64_t)k * ldb);
    braw[0] = p[0];
    braw[1] = p[1];
    if constexpr (BMASK) {
      const float4* px = reinterpret_cast<const float4*>(xcol + (uint64_t)k * ex.ldbx);
      xraw[0] = px[0];
      xraw[1] = px[1];
    }
    brs = ex.rs[AMAP ? (uint64_t)ex.amap[k] : (uint64_t)k];
  };
  auto store_b = [&](int s, int buf) {
    const bool ok = bok && kbeg + 32 * s + br < kend;
    float v[8] = {braw[0].x, braw[0].y, braw[0].z, braw[0].w,
                  braw[1].x, braw[1].y, braw[1].z, braw[1].w};
    if constexpr (BMASK) {
      const float xs[8] = {xraw[0].x, xraw[0].y, xraw[0].z, xraw[0].w,
                           xraw[1].x, xraw[1].y, xraw[1].z, xraw[1].w};
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = xs[u] > 0.f ? v[u] * ex.bscale : 0.f;
    }
    uint32_t w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) w[u] = ok ? h2_pair(ldexpf(v[u] * brs, bexp[u])) : 0u;
    f16x8 q0, q1;
    h2_unpack(w, q0, q1);
    char* dst = h2tn + buf * 2 * kH2TnImg + h2_tr_off(br, bc / 8);
    *reinterpret_cast<f16x8*>(dst) = q0;
    *reinterpret_cast<f16x8*>(dst + kH2TnImg) = q1;
  };
  const int tq = (lane & 15) >> 2, tp = lane & 3;
  const int off_lo = h2_tr_off(8 * g + tq, tp >> 1) + 8 * (tp & 1);
  const int off_hi = h2_tr_off(8 * g + 4 + tq, tp >> 1) + 8 * (tp & 1);
  auto read_b = [&](int buf, int ct, f16x8 (&b)[2]) {
#pragma unroll
    for (int pc = 0; pc < 2; ++pc) {
      const char* img = h2tn + (buf * 2 + pc) * kH2TnImg;
      const s16x4h lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4h*)(img + (off_lo ^ (32 * ct))));
      const s16x4h hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4h*)(img + (off_hi ^ (32 * ct))));
      const s16x8h c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      b[pc] = __builtin_bit_cast(f16x8, c);
    }
  };

  if (nsteps > 0) {
    load_ids(0, rid[0]);
    if (nsteps > 1) load_ids(1, rid[1]);
#pragma unroll
    for (int t = 0; t < TPW; ++t) load_x(0, rid[0], t);
#pragma unroll
    for (int t = 0; t < TPW; ++t) h2_unpack(xa[t], pa[t][0], pa[t][1]);
    if (nsteps > 1)
#pragma unroll
      for (int t = 0; t < TPW; ++t) load_x(1, rid[1], t);
    if (nsteps > 2) load_ids(2, rid[0]);
    load_b(0);
    store_b(0, 0);
    if (nsteps > 1) load_b(1);
  }
  auto step = [&](int s, auto par) {
    constexpr int P = decltype(par)::value;
    __syncthreads();
    if (s + 1 < nsteps) store_b(s + 1, 1 - P);
    if (s + 2 < nsteps) load_b(s + 2);
    if (s + 3 < nsteps) load_ids(s + 3, rid[1 - P]);
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
        f16x8 b[2];
        read_b(P, ct, b);
        acc[t][ct] = mfma3(pa[t], b, acc[t][ct]);
      }
      if (s + 1 < nsteps) h2_unpack(xa[t], pa[t][0], pa[t][1]);
      if (s + 2 < nsteps) load_x(s + 2, rid[P], t);
    }
  };
  for (int s = 0; s < nsteps; s += 2) {
    step(s, std::integral_constant<int, 0>());
    if (s + 1 < nsteps) step(s + 1, std::integral_constant<int, 1>());
  }
  float* Cb = C + (uint64_t)split * split_stride;
  float cs[8];
#pragma unroll
  for (int ct = 0; ct < 8; ++ct) {
    const int col = n0 + 16 * ct + i;
    cs[ct] = col < N ? ldexpf(1.f, -col_exp(col)) : 0.f;
  }
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    if (w_lo + t >= w_hi) continue;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int row = 16 * (w_lo + t) + 4 * g + v;
      if (row >= M) continue;
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
        const int col = n0 + 16 * ct + i;
        if (col < N) Cb[(uint64_t)row * ldc + col] = acc[t][ct][v] * cs[ct];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// TN v2 (interleaved table): every global load is compiler-visible and runs
// several k-steps ahead of its use (the v1 kernel waits on row reads whose
// latency under load exceeds its two-step prefetch).
// TN v2: k_h2_tn with three-deep register rings: a tile's A^T words are
// loaded three steps before its MFMAs (and unpacked just before them), the
// row ids of a step two steps before its loads, B rows two steps before they
// are split into LDS; B's row scales come pre-gathered (ex.rsg, written by
// the column-max pass).  TPW = 2 tiles per wave keeps the rings in registers.
template <int TPW, bool BMASK, bool AMAP>
__global__ __launch_bounds__(kH2TnThreads, 1) void k_h2_tn2(int M, int N, int K,
                                                           const uint32_t* __restrict__ A, uint64_t lda,
                                                           const float* __restrict__ B, uint64_t ldb,
                                                           float* __restrict__ C, uint64_t ldc, int kchunk,
                                                           uint64_t split_stride, int nmb, int nnb,
                                                           H2Extra ex) {
  // [2][2][kH2TnImg] B pieces, then the chunk's row ids and B row scales
  extern __shared__ __attribute__((aligned(16))) char h2tn2[];
  uint32_t* const sid = reinterpret_cast<uint32_t*>(h2tn2 + kH2TnLds);
  float* const ssc = reinterpret_cast<float*>(sid + kchunk);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, g = lane >> 4;
  const int mb = blockIdx.x % nmb;
  const int nb = (blockIdx.x / nmb) % nnb;
  const int split = blockIdx.x / (nmb * nnb);
  const int n0 = nb * 128;
  const int T = (M + 15) / 16;
  const int b_lo = mb * T / nmb, b_cnt = (mb + 1) * T / nmb - b_lo;
  const int w_lo = b_lo + wv * b_cnt / 8, w_hi = b_lo + (wv + 1) * b_cnt / 8;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int nsteps = kbeg < kend ? (kend - kbeg + 31) / 32 : 0;
  const int ntile = w_hi - w_lo;

  int acol[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) acol[t] = min(16 * min(w_lo + t, max(w_hi - 1, w_lo)) + i, M - 1);
  const int br = tid >> 4, bc = 8 * (tid & 15);
  const bool bok = n0 + bc < N;
  const float* bcol = B + (bok ? n0 + bc : 0);
  const float* xcol = BMASK ? ex.bx + (bok ? n0 + bc : 0) : nullptr;
  auto col_exp = [&](int col) {
    float m = __uint_as_float(ex.cmax[col]);
    if constexpr (BMASK) m *= ex.bscale;
    return h2_exp(m);
  };
  int bexp[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) bexp[u] = bok ? col_exp(n0 + bc + u) : 0;

  f32x4h acc[TPW][8];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int ct = 0; ct < 8; ++ct) acc[t][ct] = f32x4h{0.f, 0.f, 0.f, 0.f};
  uint32_t xa[3][TPW][8];
  float4 braw[3][2], xraw[3][BMASK ? 2 : 1];
  float bsc[3];
  // the chunk's row ids and B row scales to LDS once: the per-step reads then
  // count in lgkmcnt, and the only vmcnt streams (A words, B rows) run the
  // same three steps ahead
  for (int k = tid; k < kend - kbeg; k += kH2TnThreads) {
    sid[k] = AMAP ? ex.amap[kbeg + k] : (uint32_t)(kbeg + k);
    ssc[k] = ex.rsg[kbeg + k];
  }
  __syncthreads();

  // every load is unconditional with a clamped address (rows past the chunk
  // are zeroed where the words are consumed): the compiler then counts the
  // loads in flight exactly and waits only for the ones it uses
  const int klast = kend - kbeg - 1;
  auto load_x = [&](int s, uint32_t (&x)[TPW][8]) {
    const int k0 = 32 * s + 8 * g;
    uint32_t r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = sid[min(k0 + j, klast)];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int j = 0; j < 8; ++j) x[t][j] = A[(uint64_t)r[j] * lda + acol[t]];
  };
  auto load_b = [&](int s, float4 (&b)[2], float4 (&x)[BMASK ? 2 : 1], float& sc) {
    const int kl = min(32 * s + br, klast);
    const int k = kbeg + kl;
    const float4* p = reinterpret_cast<const float4*>(bcol + (uint64_t)k * ldb);
    b[0] = p[0];
    b[1] = p[1];
    if constexpr (BMASK) {
      const float4* px = reinterpret_cast<const float4*>(xcol + (uint64_t)k * ex.ldbx);
      x[0] = px[0];
      x[1] = px[1];
    }
    sc = ssc[kl];
  };
  auto store_b = [&](int s, int buf, const float4 (&b)[2], const float4 (&x)[BMASK ? 2 : 1], float sc) {
    const bool ok = bok && kbeg + 32 * s + br < kend;
    float v[8] = {b[0].x, b[0].y, b[0].z, b[0].w, b[1].x, b[1].y, b[1].z, b[1].w};
    if constexpr (BMASK) {
      const float xs[8] = {x[0].x, x[0].y, x[0].z, x[0].w, x[1].x, x[1].y, x[1].z, x[1].w};
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = xs[u] > 0.f ? v[u] * ex.bscale : 0.f;
    }
    uint32_t w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) w[u] = ok ? h2_pair(ldexpf(v[u] * sc, bexp[u])) : 0u;
    f16x8 q0, q1;
    h2_unpack(w, q0, q1);
    char* dst = h2tn2 + buf * 2 * kH2TnImg + h2_tr_off(br, bc / 8);
    *reinterpret_cast<f16x8*>(dst) = q0;
    *reinterpret_cast<f16x8*>(dst + kH2TnImg) = q1;
  };
  const int tq = (lane & 15) >> 2, tp = lane & 3;
  const int off_lo = h2_tr_off(8 * g + tq, tp >> 1) + 8 * (tp & 1);
  const int off_hi = h2_tr_off(8 * g + 4 + tq, tp >> 1) + 8 * (tp & 1);
  auto read_b = [&](int buf, int ct, f16x8 (&b)[2]) {
#pragma unroll
    for (int pc = 0; pc < 2; ++pc) {
      const char* img = h2tn2 + (buf * 2 + pc) * kH2TnImg;
      const s16x4h lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4h*)(img + (off_lo ^ (32 * ct))));
      const s16x4h hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4h*)(img + (off_hi ^ (32 * ct))));
      const s16x8h c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      b[pc] = __builtin_bit_cast(f16x8, c);
    }
  };

  if (nsteps == 0) return;  // (never launched: every split has >= 1 step)
  // prologue: B and A of steps 0..2 (B(0) to LDS)
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    load_b(d, braw[d], xraw[d], bsc[d]);
    load_x(d, xa[d]);
  }
  store_b(0, 0, braw[0], xraw[0], bsc[0]);
  // step s (j = s % 3): B(s) in LDS buffer s & 1, B(s+1) and B(s+2) raw in
  // braw[j+1], braw[j+2]; A(s) raw in xa[j].  Issued: B(s+3) into braw[j]
  // (B(s) went to LDS last step), then A(s+3) into xa[j] once A(s) is read.
  auto step = [&](int s, auto jc) {
    constexpr int j = decltype(jc)::value;
    constexpr int j1 = (j + 1) % 3;
    __syncthreads();
    store_b(s + 1, (s + 1) & 1, braw[j1], xraw[j1], bsc[j1]);
    load_b(s + 3, braw[j], xraw[j], bsc[j]);
    // rows of step s past the chunk: zero words (the pad may hold anything)
    const int kl = kend - (kbeg + 32 * s + 8 * g);
    uint32_t w[TPW][8];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int q = 0; q < 8; ++q) w[t][q] = q < kl ? xa[j][t][q] : 0u;
    load_x(s + 3, xa[j]);
    if (s < nsteps) {
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        if (t >= ntile) continue;
        f16x8 pa[2];
        h2_unpack(w[t], pa[0], pa[1]);
#pragma unroll
        for (int ct = 0; ct < 8; ++ct) {
          f16x8 b[2];
          read_b(s & 1, ct, b);
          acc[t][ct] = mfma3(pa, b, acc[t][ct]);
        }
      }
    }
  };
  // steps past nsteps (the loop runs a multiple of 3) only keep the load
  // stream uniform; their B rows are masked off by store_b's bounds check
  for (int s = 0; s < nsteps; s += 3) {
    step(s, std::integral_constant<int, 0>());
    step(s + 1, std::integral_constant<int, 1>());
    step(s + 2, std::integral_constant<int, 2>());
  }
  float* Cb = C + (uint64_t)split * split_stride;
  float cs[8];
#pragma unroll
  for (int ct = 0; ct < 8; ++ct) {
    const int col = n0 + 16 * ct + i;
    cs[ct] = col < N ? ldexpf(1.f, -col_exp(col)) : 0.f;
  }
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    if (t >= ntile) continue;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int row = 16 * (w_lo + t) + 4 * g + v;
      if (row >= M) continue;
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
        const int col = n0 + 16 * ct + i;
        if (col < N) Cb[(uint64_t)row * ldc + col] = acc[t][ct][v] * cs[ct];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// TN v4 (the default where it applies): the weight gradient of
// the transform-first bottom layer, dW = X[src]^T dH, with whole rows of the
// "planar" pair table (per row: the y0 plane of Kp f16, then the y1 plane)
// streamed by LDS DMA.  One block per k-chunk covers EVERY output row (up to
// 8 waves x TPW 16-row tiles) and 128 columns, so X rows and dH rows are each
// read once (v1/v2 split the output rows over 2-3 blocks and re-read dH).
//   per 16-row step: X rows -> an LDS stage (rows padded to a 512-byte
//   multiple, 16-byte chunks XOR-swizzled by row: conflict-free transposed
//   reads), raw fp32 dH rows -> an LDS stage; both two steps ahead (three
//   stages, counted vmcnt, raw barriers); then the block splits the 16 dH
//   rows (times their row scale and 2^e(col)) into two f16 planes, and each
//   wave reads its A^T fragments (ds_read_b64_tr_b16, 16 x 4 per plane) and
//   the 8 x 2 B fragments and runs TPW x 8 x 3 v_mfma_f32_16x16x16_f16.
constexpr int kH2Tn3Threads = 512;
constexpr int kH2Tn3BRaw = 16 * 512;  // one step of fp32 dH rows (N = 128)
constexpr int kH2Tn3BPl = 16 * 256;   // one plane of the split step

// The X stage's 16-byte chunk swizzle.  Rows sit 2,560 B apart (0 mod the 64
// banks), and a 32-lane group of the A^T reads (ds_read_b64_tr_b16) takes
// four rows (8h + tq, tq < 4) x four consecutive chunks from a 4-aligned
// chunk c: XOR by 4 (row & 3) puts the four rows on disjoint 4-chunk groups,
// 64 distinct banks.  (2 (row & 7), the earlier form, left rows tq = 0, 1
// and tq = 2, 3 on the same four chunks: every A^T read 2-way conflicted.)
__device__ __forceinline__ uint32_t h2_swz(int row) { return (uint32_t)(4 * (row & 3)); }

// TN v4: the structure above on v_mfma_f32_32x32x16_f16 (full-rate f16 MFMA
// at K = 16; the 16x16x16 form issues at the 16x16x32 form's cycles for half
// the work: 232 vs 183 us at C2, measured and dropped).
// DIAG (timing probes only, NTS_TN4_DIAG; results are garbage): bit 0 skips
// the MFMAs, bit 1 stops streaming after the first two steps, bit 2 skips the
// partial-slab stores
// RP (pitch 2560 only): row-aligned LDS-DMA pieces, as k_h2_nn3
template <int TPW, int DIAG = 0, bool RP = false>
__global__ __launch_bounds__(kH2Tn3Threads, 1) void k_h2_tn4(int M, int K, const char* __restrict__ Q,
                                                            uint64_t ldq, int pitch, int plane_bytes,
                                                            const float* __restrict__ B, uint64_t ldb,
                                                            float* __restrict__ C, uint64_t ldc, int kchunk,
                                                            uint64_t split_stride, int nnb, H2Extra ex) {
  extern __shared__ __attribute__((aligned(16))) char h2tn4[];
  const int xstage = 16 * pitch;
  char* const sx = h2tn4;                          // [3][16][pitch]
  char* const sbr = sx + 3 * xstage;               // [3][kH2Tn3BRaw]
  char* const sbp = sbr + 3 * kH2Tn3BRaw;          // [2 planes][kH2Tn3BPl]
  int* const sce = reinterpret_cast<int*>(sbp + 2 * kH2Tn3BPl);  // [128] column exponents
  uint32_t* const sid = reinterpret_cast<uint32_t*>(sce + 128);
  float* const ssc = reinterpret_cast<float*>(sid + kchunk);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nb = blockIdx.x % nnb, split = blockIdx.x / nnb;
  const int n0 = nb * 128;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk), klast = kend - kbeg - 1;
  const int nsteps = (kend - kbeg + 15) / 16;
  for (int k = tid; k <= klast; k += kH2Tn3Threads) {
    const uint32_t id = ex.amap ? ex.amap[kbeg + k] : (uint32_t)(kbeg + k);
    sid[k] = id;
    ssc[k] = ex.rs[id];
  }
  __syncthreads();
  // the chunk's column scales: max |rs[row] B[row, c]| over the chunk's rows
  // (the partial of this chunk is scaled back by its own 2^-e(col))
  // thread t: columns 4 (t & 31) .. +3 (the B split role below), rows t >> 5 + 16 j
  const int sr = tid >> 5, sc = 4 * (tid & 31);
  int bexp[4];
  if (ex.cparts) {
    // the chunk's column scales from dH's producer (nts_hip_spmm_csr_bwd_colmax
    // with the row scales): max |rs[row] B[row, c]| over the parts covering
    // the chunk's rows (a superset at the chunk edges: a scale at most that
    // much smaller), so every |rs B| 2^e(col) < 2^15; dH is read once, by the
    // main loop
    float* red = reinterpret_cast<float*>(sbp);  // [4][128] column maxima
    {
      const int cl = tid & 127, j = tid >> 7;
      const uint32_t p0 = (uint32_t)kbeg / ex.rpp, p1 = (uint32_t)(kbeg + klast) / ex.rpp;
      uint32_t m = 0;
      for (uint32_t p = p0 + j; p <= p1; p += 4) m = max(m, ex.cparts[(uint64_t)p * ex.nparts_ld + n0 + cl]);
      red[128 * j + cl] = __uint_as_float(m);
    }
    __syncthreads();
    if (tid < 128) {
      const float m = fmaxf(fmaxf(red[tid], red[128 + tid]), fmaxf(red[256 + tid], red[384 + tid]));
      sce[tid] = h2_exp(m);  // 2^e m in [2^14, 2^15)
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) bexp[u] = sce[sc + u];
  } else {
    float m[4] = {0.f, 0.f, 0.f, 0.f};
    const float* bp = B + (uint64_t)kbeg * ldb + n0 + sc;
    for (int k = sr; k <= klast; k += 64) {
      float4 v[4];
      float sv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kk = min(k + 16 * u, klast);
        v[u] = *reinterpret_cast<const float4*>(bp + (uint64_t)kk * ldb);
        sv[u] = k + 16 * u <= klast ? fabsf(ssc[kk]) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        m[0] = fmaxf(m[0], fabsf(v[u].x) * sv[u]);
        m[1] = fmaxf(m[1], fabsf(v[u].y) * sv[u]);
        m[2] = fmaxf(m[2], fabsf(v[u].z) * sv[u]);
        m[3] = fmaxf(m[3], fabsf(v[u].w) * sv[u]);
      }
    }
    float* red = reinterpret_cast<float*>(sbp);  // 16 row lanes x 128 columns (8 KB)
    *reinterpret_cast<float4*>(red + 128 * sr + sc) = make_float4(m[0], m[1], m[2], m[3]);
    __syncthreads();
    if (tid < 128) {
      float mm = 0.f;
      for (int l = 0; l < 16; ++l) mm = fmaxf(mm, red[128 * l + tid]);
      sce[tid] = h2_exp(mm);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) bexp[u] = sce[sc + u];
  }
  const uint32_t lsx = (uint32_t)(uintptr_t)(lds_ptr_h)sx, lsbr = (uint32_t)(uintptr_t)(lds_ptr_h)sbr;
  const int row_chunks = 2 * plane_bytes / 16;
  // X(s): 5 x 1 KB pieces per wave per 16-row step (16 * pitch = 40 KB for Kp 608)
  const int xpieces = xstage / 1024 / 8;
  auto issue = [&](int s) {
    s = min(s, nsteps - 1);
    const int st = s % 3;
    if constexpr (RP) {
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        const int p = wv * 6 + q, row = p / 3, part = p - 3 * row;
        const int c = 64 * part + lane;  // LDS slot (16-byte chunk) of the row
        const int gc = c ^ (int)h2_swz(row);
        const uint32_t id = sid[min(16 * s + row, klast)];
        const char* src = Q + (uint64_t)id * ldq + 16 * (gc < row_chunks ? gc : 0);
        const uint32_t dst = __builtin_amdgcn_readfirstlane(lsx + st * xstage + row * 2560 + 1024 * part);
        if (c < 160) glds16h(src, dst);
      }
    } else {
      for (int q = 0; q < xpieces; ++q) {
        const int p = wv * xpieces + q;
        const int o = 1024 * p + 16 * lane;
        const int row = o / pitch, c = (o - row * pitch) / 16;
        const int gc = c ^ (int)h2_swz(row);  // the global chunk this LDS slot holds
        const uint32_t id = sid[min(16 * s + row, klast)];
        const char* src = Q + (uint64_t)id * ldq + 16 * (gc < row_chunks ? gc : 0);
        glds16h(src, lsx + st * xstage + 1024 * p);
      }
    }
    {  // B raw: 1 KB per wave (rows 2 wv, 2 wv + 1)
      const int row = 2 * wv + (lane >> 5);
      const int k = kbeg + min(16 * s + row, klast);
      glds16h(reinterpret_cast<const char*>(B + (uint64_t)k * ldb + n0) + 16 * (lane & 31),
              lsbr + st * kH2Tn3BRaw + 1024 * wv);
    }
  };
  // waves: wn = wv & 1 takes output columns 64 wn .. +63 (two 32-column
  // tiles), wm = wv >> 1 a quarter of the 32-row output tiles (at most TPW)
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  const int wn = wv & 1, wm = wv >> 1;
  const int T32 = (M + 31) / 32;
  const int m_lo = wm * T32 / 4, m_hi = (wm + 1) * T32 / 4, nmt = m_hi - m_lo;
  f32x16 acc[TPW][2];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[t][nt][v] = 0.f;
  // 32x32x16 fragments: lane l = (c = l & 31, h = l >> 5) holds k rows 8h .. 8h+7
  // of column c; read as two transposed 4-row halves by its 16-lane group
  // (lane 4 tq + tp of the group addresses row 8h + tq (+4), columns 4 tp ..)
  const int h = lane >> 5, half = (lane >> 4) & 1;
  const int tq = (lane & 15) >> 2, tp = lane & 3;
  const int r0 = 8 * h + tq, r1 = r0 + 4;
  const uint32_t sw0 = h2_swz(r0), sw1 = h2_swz(r1);
  int boff[2][2];  // [n tile][row half]
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int ch = (2 * (64 * wn + 32 * nt + 16 * half + 4 * tp)) / 16;  // 16-byte chunk of the 256-byte row
    boff[nt][0] = h2_tr_off(r0, ch) + 8 * (tp & 1);
    boff[nt][1] = h2_tr_off(r1, ch) + 8 * (tp & 1);
  }
  issue(0);
  issue(1);
  for (int s = 0; s < nsteps; ++s) {
    // X(s), B(s) landed (X(s+1), B(s+1) may stay in flight: xpieces + 1 per step)
    if (RP) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else if (xpieces == 5) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier_h();
    if (!(DIAG & 2)) issue(s + 2);
    const int st = s % 3;
    {  // split B(s): row sr, 4 columns
      const float4 v = *reinterpret_cast<const float4*>(sbr + st * kH2Tn3BRaw + 512 * sr + 4 * sc);
      const bool ok = 16 * s + sr <= klast;
      const float scl = ssc[min(16 * s + sr, klast)];
      const float x[4] = {v.x, v.y, v.z, v.w};
      uint32_t w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) w[u] = ok ? h2_pair(ldexpf(x[u] * scl, bexp[u])) : 0u;
      const uint32_t lo0 = __builtin_amdgcn_perm(w[1], w[0], 0x05040100u);
      const uint32_t lo1 = __builtin_amdgcn_perm(w[3], w[2], 0x05040100u);
      const uint32_t hi0 = __builtin_amdgcn_perm(w[1], w[0], 0x07060302u);
      const uint32_t hi1 = __builtin_amdgcn_perm(w[3], w[2], 0x07060302u);
      const int off = h2_tr_off(sr, sc / 8) + 8 * ((sc / 4) & 1);
      *reinterpret_cast<uint2*>(sbp + off) = make_uint2(lo0, lo1);
      *reinterpret_cast<uint2*>(sbp + kH2Tn3BPl + off) = make_uint2(hi0, hi1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the planes are written before the barrier
    raw_barrier_h();
    auto tr = [&](const char* p) {
      return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4h*)p);
    };
    f16x8 bf[2][2];  // [n tile][plane]
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int pc = 0; pc < 2; ++pc) {
        const s16x4h lo = tr(sbp + pc * kH2Tn3BPl + boff[nt][0]);
        const s16x4h hi = tr(sbp + pc * kH2Tn3BPl + boff[nt][1]);
        const s16x8h c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bf[nt][pc] = __builtin_bit_cast(f16x8, c);
      }
    const char* xs0 = sx + st * xstage + r0 * pitch;
    const char* xs1 = sx + st * xstage + r1 * pitch;
    // A^T fragments of tile t + 1 read while tile t's MFMAs run (the
    // sched_barriers keep that order; without them each tile's reads were
    // waited on right before its MFMAs)
    auto load_af = [&](int t, f16x8 (&af)[2]) {
#pragma unroll
      for (int pc = 0; pc < 2; ++pc) {
        const int c = (pc * plane_bytes + 2 * (32 * (m_lo + t) + 16 * half + 4 * tp)) / 16;
        const s16x4h lo = tr(xs0 + 16 * (c ^ (int)sw0) + 8 * (tp & 1));
        const s16x4h hi = tr(xs1 + 16 * (c ^ (int)sw1) + 8 * (tp & 1));
        const s16x8h cc = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[pc] = __builtin_bit_cast(f16x8, cc);
      }
    };
    // (the reads are unconditional, past the wave's last tile its last tile
    // again: a conditional read leaves the waitcnt pass only lgkmcnt(0))
    f16x8 afr[2][2];  // ring: [t % 2][plane]
    if (nmt > 0) {
    load_af(0, afr[0]);
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      if (t + 1 < TPW) load_af(min(t + 1, nmt - 1), afr[(t + 1) % 2]);
      __builtin_amdgcn_sched_barrier(0);
      if (t >= nmt) continue;
      const f16x8(&af)[2] = afr[t % 2];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        if constexpr (DIAG & 1) {
          acc[t][nt][0] += (float)af[1][0] + (float)af[0][0] + (float)bf[nt][0][0] + (float)bf[nt][1][0];
        } else {
          acc[t][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1], bf[nt][0], acc[t][nt], 0, 0, 0);
          acc[t][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], bf[nt][1], acc[t][nt], 0, 0, 0);
          acc[t][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0], bf[nt][0], acc[t][nt], 0, 0, 0);
        }
      }
    }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS DMA outlives the block
  raw_barrier_h();
  // acc[t][nt][v] = C[32 (m_lo + t) + 8 (v / 4) + 4 h + v % 4][n0 + 64 wn + 32 nt + (lane & 31)]
  float* Cb = C + (uint64_t)split * split_stride;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int cl = 64 * wn + 32 * nt + (lane & 31);
    const float cs = ldexpf(1.f, -sce[cl]);
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      if (t >= nmt) continue;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = 32 * (m_lo + t) + 8 * (v / 4) + 4 * h + (v % 4);
        if (row < M && (!(DIAG & 4) || acc[t][nt][v] == 1234.5f)) Cb[(uint64_t)row * ldc + n0 + cl] = acc[t][nt][v] * cs;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// NN v3 (planar table, NTS_H2_NN default where it applies): H = diag(rs) X[amap] W
// with W stationary: wave wv holds the f16 fragments of W's 16-column slice
// n0 + 16 wv .. +15 for EVERY k-step in registers (<= 20 steps x 2 pieces),
// loaded once; the block streams 16-row tiles of whole planar rows by LDS DMA
// (the TN v4 stage: rows padded to a 512-byte multiple, 16-byte chunks
// XOR-swizzled by row), two tiles ahead, and per tile each wave runs
// nks x 3 v_mfma_f32_16x16x32_f16 on A fragments read from the stage.
constexpr int kH2Nn3KS = 20;  // k-steps held in registers (Kp <= 640)

// NKS > 0: the k-step count fixed at compile time (Kp = 32 NKS): the step loop
// fully unrolled with the A fragments read from LDS two steps ahead of their
// MFMAs (with a runtime count each step's reads were waited on right before
// its MFMAs: one exposed LDS latency per step).
// DIAG (timing probes only, NTS_NN3_DIAG; results are garbage): bit 0 skips
// the MFMAs, bit 1 stops streaming tiles after the first two
// RP (pitch 2560 only): LDS-DMA pieces cut at row boundaries — three per row
// (1 KiB, 1 KiB, 512 B with 32 lanes), six per wave and tile — instead of
// 1 KiB pieces that straddle rows (MI355X_MICROARCH.md, indexed rows into LDS)
// TR (no epilogue activation, NKS > 0): the MFMA operands swapped so that
// each lane holds four consecutive columns of one row — one 16-byte store per
// lane and tile instead of four 4-byte stores
template <bool EPI, bool AMAP, int NKS = 0, int DIAG = 0, bool RP = false, bool TR = false>
__global__ __launch_bounds__(512, 1) void k_h2_nn3(int M, int N, int Kp, const char* __restrict__ Q,
                                                  uint64_t ldq, int pitch, int plane_bytes,
                                                  const char* __restrict__ bimg, float* __restrict__ C,
                                                  uint64_t ldc, H2Extra ex) {
  extern __shared__ __attribute__((aligned(16))) char h2nn3[];
  const int xstage = 16 * pitch;
  char* const sx = h2nn3;  // [3][16][pitch]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, g = lane >> 4;
  const int nb = blockIdx.y, n0 = nb * 128;
  const int nks = Kp / 32;
  const int T = (M + 15) / 16;
  const int t0 = (int)((int64_t)blockIdx.x * T / gridDim.x);
  const int t1 = (int)((int64_t)(blockIdx.x + 1) * T / gridDim.x);
  const int nt = t1 - t0;
  if (nt <= 0) return;
  uint32_t* const sid = reinterpret_cast<uint32_t*>(sx + 3 * xstage);  // [16 nt] row ids
  float* const srs = reinterpret_cast<float*>(sid + 16 * nt);           // [16 nt] row scales
  for (int r = tid; r < 16 * nt; r += 512) {
    const int64_t row = min((int64_t)t0 * 16 + r, (int64_t)M - 1);
    const uint32_t id = AMAP ? ex.amap[row] : (uint32_t)row;
    sid[r] = id;
    srs[r] = ex.rs[id];
  }
  // W: img[s][cb][ct][piece][lane] (k_h2_split_b) — this wave's ct = wv
  f16x8 wf[kH2Nn3KS][2];
#pragma unroll
  for (int s = 0; s < kH2Nn3KS; ++s)
#pragma unroll
    for (int p = 0; p < 2; ++p)
      wf[s][p] = s < nks ? *reinterpret_cast<const f16x8*>(
                               bimg + ((size_t)s * gridDim.y + nb) * kH2Img + wv * 2 * kH2Frag +
                               p * kH2Frag + 16 * lane)
                         : f16x8{};
  const float cs = ldexpf(1.f, -h2_exp(__uint_as_float(ex.cmax[n0 + 16 * wv + i])));
  float cs4[4];  // TR: the scales of this lane's columns n0 + 16 wv + 4 g + v
#pragma unroll
  for (int v = 0; v < 4; ++v)
    cs4[v] = TR ? ldexpf(1.f, -h2_exp(__uint_as_float(ex.cmax[n0 + 16 * wv + 4 * g + v]))) : 0.f;
  __syncthreads();  // (waits for every load above: the LDS DMA counts below start from zero)
  const uint32_t lsx = (uint32_t)(uintptr_t)(lds_ptr_h)sx;
  const int xpieces = xstage / 1024 / 8;
  const int row_chunks = 2 * plane_bytes / 16;
#define NTS_NN3_ISSUE(R_)                                                                        \
  do {                                                                                           \
    const int r_ = min((R_), nt - 1);                                                            \
    if constexpr (RP) {                                                                          \
      _Pragma("unroll") for (int q = 0; q < 6; ++q) {                                            \
        const int p = wv * 6 + q, row = p / 3, part = p - 3 * row;                               \
        const int c = 64 * part + lane; /* LDS slot (16-byte chunk) of the row */               \
        const int gc = c ^ (row & 15);                                                           \
        const char* src = Q + (uint64_t)sid[16 * r_ + row] * ldq + 16 * (gc < row_chunks ? gc : 0); \
        const uint32_t dst_ = __builtin_amdgcn_readfirstlane(lsx + (r_ % 3) * xstage + row * 2560 + 1024 * part); \
        if (c < 160) glds16h(src, dst_);                                                         \
      }                                                                                          \
    } else {                                                                                     \
      for (int q = 0; q < xpieces; ++q) {                                                        \
        const int p = wv * xpieces + q;                                                          \
        const int o = 1024 * p + 16 * lane;                                                      \
        const int row = o / pitch, c = (o - row * pitch) / 16;                                   \
        const int gc = c ^ (row & 15); /* the global chunk this LDS slot holds */                \
        const char* src = Q + (uint64_t)sid[16 * r_ + row] * ldq + 16 * (gc < row_chunks ? gc : 0); \
        glds16h(src, lsx + (r_ % 3) * xstage + 1024 * p);                                        \
      }                                                                                          \
    }                                                                                            \
  } while (0)
  const int pch = plane_bytes / 16;  // chunks per plane
  const int iswz = i;                 // row i's swizzle (i < 16)
  NTS_NN3_ISSUE(0);
  NTS_NN3_ISSUE(1);
  for (int r = 0; r < nt; ++r) {
    // tile r landed.  Younger VMEM ops: r = 0: tile 1's 5 pieces; r = 1:
    // tile 2's pieces and round 0's 4 stores; r >= 2: round r-2's 4 stores,
    // tile r+1's pieces, round r-1's 4 stores
    constexpr int NST = TR ? 1 : 4;  // stores per wave and tile
    if (RP) {  // six pieces per wave and tile
      if (r == 0) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if (r == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(6 + NST) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(6 + 2 * NST) : "memory");
    } else if (TR && xpieces == 5) {
      if (r == 0) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else if (r == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(5 + NST) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(5 + 2 * NST) : "memory");
    } else if (xpieces == 5) {
      if (r == 0) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else if (r == 1) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    raw_barrier_h();
    if (!(DIAG & 2)) NTS_NN3_ISSUE(r + 2);
    const char* xs = sx + (r % 3) * xstage + i * pitch;
    f32x4h acc = f32x4h{0.f, 0.f, 0.f, 0.f};
    auto step = [&](int s, const f16x8& a1, const f16x8& a0) {
      if constexpr (DIAG & 1) {
        acc[0] += (float)a1[0] + (float)a0[0] + (float)wf[s][0][0] + (float)wf[s][1][0];
      } else if constexpr (TR) {  // D^T: rows of W^T (columns) x columns of X^T (rows)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[s][0], a1, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[s][1], a0, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[s][0], a0, acc, 0, 0, 0);
      } else {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, wf[s][0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, wf[s][1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, wf[s][0], acc, 0, 0, 0);
      }
    };
    auto ld1 = [&](int s) { return *reinterpret_cast<const f16x8*>(xs + 16 * ((pch + 4 * s + g) ^ iswz)); };
    auto ld0 = [&](int s) { return *reinterpret_cast<const f16x8*>(xs + 16 * ((4 * s + g) ^ iswz)); };
    if constexpr (NKS > 0) {
      f16x8 b1[3], b0[3];  // fragments of steps s, s+1, s+2 (ring of three)
      b1[0] = ld1(0);
      b0[0] = ld0(0);
      if (NKS > 1) {
        b1[1] = ld1(1);
        b0[1] = ld0(1);
      }
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        if (s + 2 < NKS) {
          b1[(s + 2) % 3] = ld1(s + 2);
          b0[(s + 2) % 3] = ld0(s + 2);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the reads two steps ahead
        step(s, b1[s % 3], b0[s % 3]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < kH2Nn3KS; ++s)
        if (s < nks) step(s, ld1(s), ld0(s));
    }
    if constexpr (TR) {  // acc[v] = H[16 (t0 + r) + i][n0 + 16 wv + 4 g + v]
      const int64_t row = (int64_t)(t0 + r) * 16 + i;
      const float rsr = srs[16 * r + i];
      const float4 o4 = make_float4(acc[0] * cs4[0] * rsr, acc[1] * cs4[1] * rsr,
                                    acc[2] * cs4[2] * rsr, acc[3] * cs4[3] * rsr);
      if (row < M) *reinterpret_cast<float4*>(C + (uint64_t)row * ldc + n0 + 16 * wv + 4 * g) = o4;
      continue;
    }
    // acc[v] = H[16 (t0 + r) + 4 g + v][n0 + 16 wv + i]
    const int64_t r4 = (int64_t)(t0 + r) * 16 + 4 * g;
    const uint32_t col = (uint32_t)(n0 + 16 * wv + i);
    float o[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) o[v] = acc[v] * cs * srs[16 * r + 4 * g + v];
    if constexpr (EPI) {
      const uint4 rnd = dropout_words((uint64_t)r4, col, ex.seed, ex.offset);
      const uint32_t wd[4] = {rnd.x, rnd.y, rnd.z, rnd.w};
#pragma unroll
      for (int v = 0; v < 4; ++v)
        o[v] = (dropout_bits(wd[v], col) >= ex.keep_threshold && o[v] > 0.f) ? o[v] * ex.scale : 0.f;
    }
#pragma unroll
    for (int v = 0; v < 4; ++v)
      if (r4 + v < M) C[(uint64_t)(r4 + v) * ldc + col] = o[v];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS DMA outlives the block
  raw_barrier_h();
#undef NTS_NN3_ISSUE
}


#ifdef NTS_WITH_H2_NN4
// NN v4 (k_h2_nn4): k_h2_nn3 with FOUR LDS stages, three 16-row tiles in
// flight per block instead of two (the 160 KB of LDS hold exactly four
// 16 x 2560-byte stages; Kp = 608, 19 k-steps): the row ids move to registers (lane t of each wave
// holds its two rows of tile t, read with readlane) and the row scales ride in
// the planar table's row tails (ldq = 1280 halves: the scale at half 2 Kp,
// nts_hip_h2_split_rows_planar), so the stages take the whole LDS.  RP pieces
// (three per row, six per wave and tile), planar rows swizzled by row as in
// k_h2_nn3; the tail chunk (global chunk 2 Kp / 8) lands in LDS slot
// 2Kp/8 ^ (row & 15).  No epilogue activation (the transform-first forward).
template <int NKS>
__global__ __launch_bounds__(512, 1) void k_h2_nn4(int M, int N, const char* __restrict__ Q,
                                                  uint64_t ldq, int plane_bytes,
                                                  const char* __restrict__ bimg, float* __restrict__ C,
                                                  uint64_t ldc, H2Extra ex) {
  extern __shared__ __attribute__((aligned(16))) char h2nn4[];
  constexpr int kPitch = 2560, kStage = 16 * kPitch;
  char* const sx = h2nn4;  // [4][16][2560]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, g = lane >> 4;
  const int nb = blockIdx.y, n0 = nb * 128;
  const int T = (M + 15) / 16;
  const int t0 = (int)((int64_t)blockIdx.x * T / gridDim.x);
  const int t1 = (int)((int64_t)(blockIdx.x + 1) * T / gridDim.x);
  const int nt = t1 - t0;  // <= 64 (host)
  if (nt <= 0) return;
  // lane t: the ids of rows 2 wv and 2 wv + 1 of tile t (this wave's DMA rows)
  uint32_t id0 = 0, id1 = 0;
  if (lane < nt) {
    const int64_t r0 = min((int64_t)(t0 + lane) * 16 + 2 * wv, (int64_t)M - 1);
    const int64_t r1 = min((int64_t)(t0 + lane) * 16 + 2 * wv + 1, (int64_t)M - 1);
    id0 = ex.amap[r0];
    id1 = ex.amap[r1];
  }
  f16x8 wf[kH2Nn3KS][2];
#pragma unroll
  for (int s = 0; s < kH2Nn3KS; ++s)
#pragma unroll
    for (int p = 0; p < 2; ++p)
      wf[s][p] = s < NKS ? *reinterpret_cast<const f16x8*>(
                               bimg + ((size_t)s * gridDim.y + nb) * kH2Img + wv * 2 * kH2Frag +
                               p * kH2Frag + 16 * lane)
                         : f16x8{};
  const float cs = ldexpf(1.f, -h2_exp(__uint_as_float(ex.cmax[n0 + 16 * wv + i])));
  __syncthreads();  // (waits for every load above: the LDS DMA counts below start from zero)
  const uint32_t lsx = (uint32_t)(uintptr_t)(lds_ptr_h)sx;
  auto issue = [&](int r) {
    const int rr = min(r, nt - 1);
    const uint32_t ida = __builtin_amdgcn_readlane(id0, rr), idb = __builtin_amdgcn_readlane(id1, rr);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int row = q / 3, part = q - 3 * row;  // this wave's rows 2 wv + row
      const int grow = 2 * wv + row;
      const int c = 64 * part + lane;              // LDS slot (16-byte chunk) of the row
      const int gc = c ^ (grow & 15);               // the global chunk it holds (tail included)
      const char* src = Q + (uint64_t)(row ? idb : ida) * ldq + 16 * gc;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(lsx + (rr & 3) * kStage + grow * kPitch + 1024 * part);
      if (c < 160) glds16h(src, dst);
    }
  };
  const int pch = plane_bytes / 16;  // chunks per plane
  const int tail = 2 * pch;          // the row-scale chunk
  issue(0);
  issue(1);
  issue(2);
  for (int r = 0; r < nt; ++r) {
    // tile r landed.  Younger VMEM ops (6 DMA pieces per tile, 4 stores per
    // round): r = 0: tiles 1, 2; r = 1: tile 2, tile 3 + round 0's stores;
    // r = 2: + tile 4 + round 1's stores; r >= 3: round r-3's stores, then
    // (tile, stores) of rounds r-2 and r-1
    if (r == 0) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (r == 1) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (r == 2) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    raw_barrier_h();  // also: every wave is past tile r-1 (its stage takes tile r+3)
    issue(r + 3);
    const char* st = sx + (r & 3) * kStage;
    const char* xs = st + i * kPitch;
    // the row scales of this lane's output rows 4 g + v (row tails)
    float rsr[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int row = 4 * g + v;
      rsr[v] = *reinterpret_cast<const float*>(st + row * kPitch + 16 * (tail ^ row));
    }
    f32x4h acc = f32x4h{0.f, 0.f, 0.f, 0.f};
    auto ld1 = [&](int s) { return *reinterpret_cast<const f16x8*>(xs + 16 * ((pch + 4 * s + g) ^ i)); };
    auto ld0 = [&](int s) { return *reinterpret_cast<const f16x8*>(xs + 16 * ((4 * s + g) ^ i)); };
    f16x8 b1[3], b0[3];  // fragments of steps s, s+1, s+2 (ring of three)
    b1[0] = ld1(0);
    b0[0] = ld0(0);
    b1[1] = ld1(1);
    b0[1] = ld0(1);
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      if (s + 2 < NKS) {
        b1[(s + 2) % 3] = ld1(s + 2);
        b0[(s + 2) % 3] = ld0(s + 2);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the reads two steps ahead
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(b1[s % 3], wf[s][0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0[s % 3], wf[s][1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0[s % 3], wf[s][0], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // acc[v] = H[16 (t0 + r) + 4 g + v][n0 + 16 wv + i]
    const int64_t r4 = (int64_t)(t0 + r) * 16 + 4 * g;
    const uint32_t col = (uint32_t)(n0 + 16 * wv + i);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float o = acc[v] * cs * rsr[v];
      // (four stores per round, as the counted waits assume: only the last
      // tile of the last block can lose lanes, and no counted wait follows it)
      if (r4 + v < M) C[(uint64_t)(r4 + v) * ldc + col] = o;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS DMA outlives the block
  raw_barrier_h();
}

#endif  // NTS_WITH_H2_NN4

// ---------------------------------------------------------------------------
// NN with a DYNAMIC fp32 A of at most 128 columns (the aggregate-first layer
// of the products / papers-shaped configs: ~140K aggregated rows x 100 ->
// 256, where the fp32 and split-bf16 MFMA kernels run at ~1.8 TB/s on a
// memory-bound shape): C = act(A W) with A split into f16 pairs INSIDE the
// kernel.  Per 32-row tile: the raw fp32 rows by LDS DMA (three stages, two
// tiles ahead), one thread per row and 8 columns splits them (row max over 16
// lanes -> power-of-two row scale, y0 = f16(y), y1 = f16(y - y0)) into two
// swizzled f16 planes, then each wave runs its W-stationary column tiles
// (NTW x 16 columns, W's fragments in registers as k_h2_nn3) over the two
// 16-row halves: 3 v_mfma_f32_16x16x32_f16 per 32-deep step.  Epilogue:
// rs(row) 2^-e(col) acc, relu/dropout with the Philox keys of
// nts_hip_gemm_relu_dropout_f32.  QOUT: the planes and row scales are also
// written out as A's planar pair table (the weight gradient's operand).
constexpr int kH2dTM = 32;

template <int NKS, int NTW, bool EPI, bool QOUT>
__global__ __launch_bounds__(512) void k_h2_nnd(int M, int K, const float* __restrict__ A, uint64_t lda,
                                                const char* __restrict__ bimg, int ncb,
                                                const uint32_t* __restrict__ cmax, float* __restrict__ C,
                                                uint64_t ldc, uint16_t* __restrict__ Qo, uint64_t ldq,
                                                float* __restrict__ rso, H2Extra ex) {
  constexpr int TM = kH2dTM, KP = 32 * NKS;
  constexpr int CPR = KP / 4;                 // 16-byte fp32 chunks per raw row
  constexpr int PCH = KP / 8;                 // 16-byte f16 chunks of a row's k range
  constexpr int PRB = 256;                    // plane row pitch: 16 chunks (XOR-swizzled by row)
  constexpr int PL = TM * PRB;                // one plane
  constexpr int NPC = (TM * CPR + 511) / 512; // LDS-DMA pieces per thread and tile
  constexpr int RAW = NPC * 512 * 16;         // one raw stage (row-major [TM][KP] fp32 + padding)
  constexpr int NS = 2 * NTW * 4;             // epilogue stores per wave and tile
  constexpr int NQ = QOUT ? 3 : 0;            // pair-table stores per wave and tile
  static_assert(NKS >= 1 && NKS <= 4, "shape");
  __shared__ __attribute__((aligned(16))) char smem[3 * RAW + 2 * PL + TM * 4];
  char* const raw = smem;
  char* const pl = smem + 3 * RAW;
  float* const srs = reinterpret_cast<float*>(pl + 2 * PL);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, g = lane >> 4;
  const int T = (M + TM - 1) / TM;
  const int t0 = (int)((int64_t)blockIdx.x * T / gridDim.x);
  const int t1 = (int)((int64_t)(blockIdx.x + 1) * T / gridDim.x);
  const int nt = t1 - t0;
  if (nt <= 0) return;
  f16x8 wf[NKS][NTW][2];
  float cs[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int gct = wv * NTW + j, cb = gct >> 3, ct = gct & 7;
#pragma unroll
    for (int s = 0; s < NKS; ++s)
#pragma unroll
      for (int p = 0; p < 2; ++p)
        wf[s][j][p] = *reinterpret_cast<const f16x8*>(bimg + ((size_t)s * ncb + cb) * kH2Img +
                                                      ct * 2 * kH2Frag + p * kH2Frag + 16 * lane);
    cs[j] = ldexpf(1.f, -h2_exp(__uint_as_float(cmax[16 * gct + i])));
  }
  __syncthreads();  // every load above done: the counted waits below start from zero
  const uint32_t lraw = (uint32_t)(uintptr_t)(lds_ptr_h)raw;
  // tile r's rows -> raw stage r % 3 (row-major [TM][KP] fp32); chunks past
  // the row's K load the row's first chunk (zeroed by the split), rows past M
  // the last row
  auto issue = [&](int r) {
    r = min(r, nt - 1);
#pragma unroll
    for (int q = 0; q < NPC; ++q) {
      const int pc = q * 512 + wv * 64 + lane;
      const int row = pc / CPR, c = pc - row * CPR;
      const int64_t grow = min((int64_t)(t0 + r) * TM + row, (int64_t)M - 1);
      // (pieces past the tile land in the stage's padding: any valid address)
      const float* src = pc < TM * CPR ? A + (uint64_t)grow * lda + (4 * c < K ? 4 * c : 0) : A;
      glds16h(src, lraw + (r % 3) * RAW + 16 * (q * 512 + wv * 64));
    }
  };
  issue(0);
  issue(1);
  const int sr = tid >> 4, sc = tid & 15;  // split role: row, 8-column group
  for (int r = 0; r < nt; ++r) {
    // raw tile r landed.  Younger VMEM ops: r = 0: tile 1's pieces; r = 1:
    // tile 2's pieces + round 0's stores; r >= 2: round r-2's stores, tile
    // r+1's pieces, round r-1's stores
    if (r == 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NPC) : "memory");
    else if (r == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NPC + NQ + NS) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NPC + 2 * (NQ + NS)) : "memory");
    raw_barrier_h();  // also: every wave is past tile r-1's plane reads
    issue(r + 2);
    const int64_t row0 = (int64_t)(t0 + r) * TM;
    {  // split: row sr, columns 8 sc .. 8 sc + 7 (16 lanes per row; sc >= PCH: zeros)
      float x[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (sc < PCH) {
        const float* xr = reinterpret_cast<const float*>(raw + (r % 3) * RAW + sr * KP * 4) + 8 * sc;
        const float4 u0 = *reinterpret_cast<const float4*>(xr);
        const float4 u1 = *reinterpret_cast<const float4*>(xr + 4);
        x[0] = u0.x; x[1] = u0.y; x[2] = u0.z; x[3] = u0.w;
        x[4] = u1.x; x[5] = u1.y; x[6] = u1.z; x[7] = u1.w;
      }
      float m = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (8 * sc + k >= K) x[k] = 0.f;
        m = fmaxf(m, fabsf(x[k]));
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o));
      const int e = h2_exp(m);
      uint32_t w[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) w[k] = h2_pair(ldexpf(x[k], e));
      f16x8 p0, p1;
      h2_unpack(w, p0, p1);
      const float rsv = ldexpf(1.f, -e);
      if (sc == 0) srs[sr] = rsv;
      if (sc < PCH) {
        const int cw = sc ^ (sr & 15);
        *reinterpret_cast<f16x8*>(pl + sr * PRB + 16 * cw) = p0;
        *reinterpret_cast<f16x8*>(pl + PL + sr * PRB + 16 * cw) = p1;
      }
      if constexpr (QOUT) {  // the planar pair row (clamped duplicates rewrite row M-1 alike)
        const int64_t grow = min(row0 + sr, (int64_t)M - 1);
        uint16_t* q = Qo + (uint64_t)grow * ldq;
        if (sc < PCH) {
          *reinterpret_cast<f16x8*>(q + 8 * sc) = p0;
          *reinterpret_cast<f16x8*>(q + KP + 8 * sc) = p1;
        }
        if (sc == 0) rso[grow] = rsv;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier_h();
    f32x4h acc[2][NTW];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ar = 16 * h + i;
      const char* a0p = pl + ar * PRB;
      const int swz = ar & 15;
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[h][j] = f32x4h{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        const int c = (4 * s + g) ^ swz;
        const f16x8 a[2] = {*reinterpret_cast<const f16x8*>(a0p + 16 * c),
                            *reinterpret_cast<const f16x8*>(a0p + PL + 16 * c)};
#pragma unroll
        for (int j = 0; j < NTW; ++j) acc[h][j] = mfma3(a, wf[s][j], acc[h][j]);
      }
    }
    // epilogue over the (half, column tile) blocks q = 2 h + j.  The keep
    // bits of lanes i and i ^ 1 come from one Philox call (one call per 4 x 2
    // elements): per pair of blocks (q0, q1) the even lane draws q0's words,
    // the odd lane q1's, and they swap.  Instantiated per (dropout on, whole
    // tile) so each form is straight-line selects and unguarded stores (a
    // runtime `drop` and per-row guards inside one body compiled to a scalar
    // branch per element: 81 vs 55 us without activation)
    constexpr int NB = 2 * NTW;
    auto epilogue = [&](auto DROP, auto FULL) {
      constexpr bool D = EPI && decltype(DROP)::value;
      constexpr bool FT = decltype(FULL)::value;
#pragma unroll
      for (int q0 = 0; q0 < NB; q0 += 2) {
        uint32_t wd[2][4] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
        if constexpr (D) {
          const int qm = q0 + (i & 1);  // this lane's draw
          const int64_t r4m = row0 + 16 * (qm / NTW) + 4 * g;
          const uint32_t colm = (uint32_t)(16 * (wv * NTW + qm % NTW) + i);
          const uint4 rnd = dropout_words((uint64_t)r4m, colm, ex.seed, ex.offset);
          const uint32_t mine[4] = {rnd.x, rnd.y, rnd.z, rnd.w};
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const uint32_t other = (uint32_t)__shfl_xor((int)mine[v], 1);
            wd[0][v] = (i & 1) ? other : mine[v];
            wd[1][v] = (i & 1) ? mine[v] : other;
          }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int q = q0 + u, h = q / NTW, j = q % NTW;
          const int64_t r4 = row0 + 16 * h + 4 * g;
          const uint32_t col = (uint32_t)(16 * (wv * NTW + j) + i);
          float o[4];
#pragma unroll
          for (int v = 0; v < 4; ++v) o[v] = acc[h][j][v] * cs[j] * srs[16 * h + 4 * g + v];
          if constexpr (EPI) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              bool keep = o[v] > 0.f;
              if constexpr (D) keep = keep && dropout_bits(wd[u][v], col) >= ex.keep_threshold;
              o[v] = keep ? o[v] * ex.scale : 0.f;
            }
          }
          float* cp = C + (uint64_t)r4 * ldc + col;
#pragma unroll
          for (int v = 0; v < 4; ++v)
            if (FT || r4 + v < M) cp[(uint64_t)v * ldc] = o[v];
        }
      }
    };
    const bool drop = EPI && ex.keep_threshold != 0u;
    const bool full = row0 + TM <= (int64_t)M;
    if (full) {
      if (drop) epilogue(std::true_type{}, std::true_type{});
      else epilogue(std::false_type{}, std::true_type{});
    } else {
      if (drop) epilogue(std::true_type{}, std::false_type{});
      else epilogue(std::false_type{}, std::false_type{});
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS DMA outlives the block
  raw_barrier_h();
}

static int colmax(nts_hip_ctx* ctx, const float* B, uint64_t ldb, uint64_t K, int N, const float* rs,
                  const uint32_t* amap, uint32_t* out, float* rsg = nullptr) {
  NTS_HIP_TRY(hipMemsetAsync(out, 0, (size_t)N * sizeof(uint32_t), ctx->stream));
  if (K == 0) return NTS_OK;
  const uint64_t blocks = std::min<uint64_t>(256, (K + 63) / 64);  // 256 x N atomics at most
  const uint64_t per = (K + blocks - 1) / blocks;
  hipLaunchKernelGGL(k_colmax, dim3((uint32_t)((K + per - 1) / per)), dim3(256), 0, ctx->stream, B, ldb,
                     K, N, rs, amap, per, out, rsg);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

}  // namespace nts_hip

using namespace nts_hip;

extern "C" int nts_hip_h2_split_rows(nts_hip_ctx* ctx, uint64_t R, uint32_t K, const float* X,
                                     uint64_t ldx, uint32_t Kp, uint32_t* P, uint64_t ldp, float* rs) {
  NTS_CHECK_ARG(ctx, "NULL context");
  NTS_CHECK_ARG(Kp >= K && Kp % 32 == 0 && ldp >= Kp && ldp % 4 == 0, "Kp / ldp");
  NTS_CHECK_ARG(ldx >= K, "ldx < K");
  NTS_CHECK_ARG(R == 0 || (X && P && rs), "NULL buffer");
  NTS_CHECK_ARG((uintptr_t)P % 16 == 0, "P must be 16-byte aligned");
  if (R == 0) return NTS_OK;
  hipLaunchKernelGGL(k_h2_split_rows, dim3((uint32_t)((R + 3) / 4)), dim3(256), 0, ctx->stream, R, K, X,
                     ldx, Kp, P, ldp, rs);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

// scratch: [column max bits (N words, padded)][...]
extern "C" int nts_hip_gemm_h2_gather(nts_hip_ctx* ctx, int relu_dropout, int M, int N, int Kp,
                                      const uint32_t* P, uint64_t ldp, const float* rs,
                                      const uint32_t* a_rows, const float* W, uint64_t ldw, int K,
                                      float* C, uint64_t ldc, float p, uint64_t seed, uint64_t offset) {
  NTS_CHECK_ARG(ctx, "NULL context");
  NTS_CHECK_ARG(M >= 0 && N > 0 && N % 16 == 0 && K > 0 && Kp >= K && Kp % 32 == 0, "shape");
  NTS_CHECK_ARG(ldp >= (uint64_t)Kp && ldp % 4 == 0 && (uintptr_t)P % 16 == 0, "pair table layout");
  NTS_CHECK_ARG(ldw >= (uint64_t)N && ldc >= (uint64_t)N, "ld");
  NTS_CHECK_ARG(ldw % 4 == 0 && (uintptr_t)W % 16 == 0, "W rows must be float4-aligned");
  NTS_CHECK_ARG(M == 0 || (P && rs && W && C), "NULL buffer");
  NTS_CHECK_ARG(p >= 0.f && p < 1.f, "p must be in [0, 1)");
  if (M == 0) return NTS_OK;
  const int ncb = (N + 127) / 128, nsteps = Kp / 32;
  const size_t cm_bytes = ((size_t)N * 4 + 255) / 256 * 256;
  const size_t img = (size_t)nsteps * ncb * kH2Img;
  NTS_RET(ensure_scratch(ctx, cm_bytes + img + 256));
  uint32_t* cmax = (uint32_t*)ctx->scratch;
  char* bimg = (char*)ctx->scratch + cm_bytes;
  hipLaunchKernelGGL(k_h2_prep_w, dim3(nsteps, ncb), dim3(512), 0, ctx->stream, W, ldw, K, N, cmax, bimg);
  NTS_LAUNCH_CHECK();
  H2Extra ex;
  ex.keep_threshold = dropout_threshold(p);
  ex.scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  ex.seed = seed;
  ex.offset = offset;
  ex.amap = a_rows;
  ex.rs = rs;
  ex.cmax = cmax;
  const int T = (M + 15) / 16;
  int gx = std::max(8, (256 / ncb) / 8 * 8);
  gx = std::min(gx, std::max(8, ((T + 15) / 16 + 7) / 8 * 8));
  const int64_t Wv = (int64_t)gx * 8;
  const int max_tiles = (int)((T + Wv - 1) / Wv);
  const int rounds = (max_tiles + 1) / 2;
  const dim3 grid(gx, ncb);
#define NTS_H2NN(E, MP)                                                                          \
  do {                                                                                           \
    NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_h2_nn<E, MP>),              \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kH2NnLds));      \
    hipLaunchKernelGGL((k_h2_nn<E, MP>), grid, dim3(kH2NnThreads), kH2NnLds, ctx->stream, M, N,   \
                       Kp, P, ldp, bimg, C, ldc, rounds, ex);                                    \
  } while (0)
  if (relu_dropout) {
    if (a_rows) NTS_H2NN(true, true); else NTS_H2NN(true, false);
  } else {
    if (a_rows) NTS_H2NN(false, true); else NTS_H2NN(false, false);
  }
#undef NTS_H2NN
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

extern "C" int nts_hip_gemm_h2_tn_gather(nts_hip_ctx* ctx, int M, int N, int K, const uint32_t* P,
                                         uint64_t ldp, const float* rs, const uint32_t* a_rows,
                                         const float* B, uint64_t ldb, const float* X, uint64_t ldx,
                                         float bscale, float* C, uint64_t ldc) {
  NTS_CHECK_ARG(ctx, "NULL context");
  NTS_CHECK_ARG(M > 0 && N > 0 && N % 16 == 0 && N <= 1024 && K >= 0, "shape");
  NTS_CHECK_ARG(ldp >= (uint64_t)M && (uintptr_t)P % 4 == 0, "pair table layout");
  NTS_CHECK_ARG(ldb >= (uint64_t)N && ldb % 4 == 0 && (uintptr_t)B % 16 == 0, "B layout");
  NTS_CHECK_ARG(!X || (ldx >= (uint64_t)N && ldx % 4 == 0 && (uintptr_t)X % 16 == 0), "X layout");
  NTS_CHECK_ARG(!a_rows || (uintptr_t)a_rows % 16 == 0, "a_rows must be 16-byte aligned");
  NTS_CHECK_ARG(ldc >= (uint64_t)N, "ldc");
  NTS_CHECK_ARG(K == 0 || (P && rs && B && C), "NULL buffer");
  if (K == 0) {
    NTS_HIP_TRY(hipMemset2DAsync(C, ldc * sizeof(float), 0, (size_t)N * sizeof(float), (size_t)M,
                                 ctx->stream));
    return NTS_OK;
  }
  // v2 (TPW 2) keeps the chunk's row ids + scales in LDS (8 B per row): past
  // 8192-row chunks (a reduction > ~700 K rows at this N) the v1 kernel runs
  bool v1 = false;
  int TPW = 0, nmb = 0, splits = 0, kchunk = 0;
  const int T = (M + 15) / 16, nnb = (N + 127) / 128, ksteps = (K + 31) / 32;
  for (int pass = 0; pass < 2; ++pass) {
    TPW = v1 ? 3 : 2;
    nmb = (T + 8 * TPW - 1) / (8 * TPW);
    splits = std::max(1, std::min(256 / (nmb * nnb), ksteps / 4));
    kchunk = ((ksteps + splits - 1) / splits) * 32;
    splits = (K + kchunk - 1) / kchunk;
    if (v1 || kchunk <= 8192) break;
    v1 = true;
  }
  const int tn2_lds = kH2TnLds + 8 * kchunk;
  const uint64_t stride = (uint64_t)M * N;
  const size_t cm_bytes = ((size_t)N * 4 + 255) / 256 * 256;
  const size_t rsg_bytes = ((size_t)K * 4 + 255) / 256 * 256;
  const size_t part_bytes = splits > 1 ? stride * splits * sizeof(float) : 0;
  NTS_RET(ensure_scratch(ctx, cm_bytes + rsg_bytes + part_bytes + 256));
  uint32_t* cmax = (uint32_t*)ctx->scratch;
  float* rsg = (float*)((char*)ctx->scratch + cm_bytes);
  float* out = C;
  uint64_t ldo = ldc;
  if (splits > 1) {
    out = (float*)((char*)ctx->scratch + cm_bytes + rsg_bytes);
    ldo = N;
  }
  // column max of rs[row] * op(B) (bounded by the unmasked B * bscale), and
  // the B rows' scales gathered for the kernel
  NTS_RET(colmax(ctx, B, ldb, (uint64_t)K, N, rs, a_rows, cmax, rsg));
  H2Extra ex;
  ex.amap = a_rows;
  ex.rs = rs;
  ex.rsg = rsg;
  ex.cmax = cmax;
  ex.bx = X;
  ex.ldbx = ldx;
  ex.bscale = bscale;
  NTS_CHECK_ARG(!X || bscale > 0.f, "bscale must be > 0");
  const dim3 grid(nmb * nnb * splits);
#define NTS_H2TN(BM, MP)                                                                         \
  do {                                                                                           \
    if (v1) {                                                                                    \
      NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_h2_tn<3, BM, MP>),        \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, kH2TnLds));    \
      hipLaunchKernelGGL((k_h2_tn<3, BM, MP>), grid, dim3(kH2TnThreads), kH2TnLds, ctx->stream, M, \
                         N, K, P, ldp, B, ldb, out, ldo, kchunk, splits > 1 ? stride : (uint64_t)0, \
                         nmb, nnb, ex);                                                          \
    } else {                                                                                     \
      NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_h2_tn2<2, BM, MP>),       \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, tn2_lds));     \
      hipLaunchKernelGGL((k_h2_tn2<2, BM, MP>), grid, dim3(kH2TnThreads), tn2_lds, ctx->stream, M, \
                         N, K, P, ldp, B, ldb, out, ldo, kchunk, splits > 1 ? stride : (uint64_t)0, \
                         nmb, nnb, ex);                                                          \
    }                                                                                            \
  } while (0)
  if (X) {
    if (a_rows) NTS_H2TN(true, true); else NTS_H2TN(true, false);
  } else {
    if (a_rows) NTS_H2TN(false, true); else NTS_H2TN(false, false);
  }
#undef NTS_H2TN
  NTS_LAUNCH_CHECK();
  if (splits == 1) return NTS_OK;
  return sum_splits(ctx->stream, out, splits, stride, M, N, C, ldc);
}

extern "C" int nts_hip_h2_split_rows_planar(nts_hip_ctx* ctx, uint64_t R, uint32_t K, const float* X,
                                            uint64_t ldx, uint32_t Kp, uint16_t* Q, uint64_t ldq,
                                            float* rs) {
  NTS_CHECK_ARG(ctx, "NULL context");
  NTS_CHECK_ARG(Kp >= K && Kp % 32 == 0 && ldq >= 2 * (uint64_t)Kp && ldq % 8 == 0, "Kp / ldq");
  NTS_CHECK_ARG(ldx >= K, "ldx < K");
  NTS_CHECK_ARG(R == 0 || (X && Q && rs), "NULL buffer");
  NTS_CHECK_ARG((uintptr_t)Q % 16 == 0, "Q must be 16-byte aligned");
  if (R == 0) return NTS_OK;
  hipLaunchKernelGGL(k_h2_split_rows_planar, dim3((uint32_t)((R + 3) / 4)), dim3(256), 0, ctx->stream, R,
                     K, X, ldx, Kp, Q, ldq, rs);
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

// TN v4 on the planar table (k_h2_tn4): N % 128 == 0, M <= 8 * 5 * 16 = 640,
// rows of <= 640 pair words (Kp <= 640).  Scratch: [column max][row scales][partials].
static int h2p_tn_gather(nts_hip_ctx* ctx, int M, int N, int K, const uint16_t* Q, uint64_t ldq, int Kp,
                         const float* rs, const uint32_t* a_rows, const float* B, uint64_t ldb, float* C,
                         uint64_t ldc, const uint32_t* part_max, uint32_t rows_per_part) {
  constexpr int TPW = 5;
  NTS_CHECK_ARG(ctx, "NULL context");
  NTS_CHECK_ARG(M > 0 && M <= 8 * TPW * 16 && N > 0 && N % 128 == 0 && K >= 0, "shape");
  NTS_CHECK_ARG(Kp % 32 == 0 && Kp >= M && Kp <= 640 && ldq >= 2 * (uint64_t)Kp && ldq % 8 == 0 &&
                    (uintptr_t)Q % 16 == 0, "planar table layout");
  NTS_CHECK_ARG(ldb >= (uint64_t)N && ldb % 4 == 0 && (uintptr_t)B % 16 == 0, "B layout");
  NTS_CHECK_ARG(ldc >= (uint64_t)N, "ldc");
  NTS_CHECK_ARG(K == 0 || (Q && rs && B && C), "NULL buffer");
  if (K == 0) {
    NTS_HIP_TRY(hipMemset2DAsync(C, ldc * sizeof(float), 0, (size_t)N * sizeof(float), (size_t)M,
                                 ctx->stream));
    return NTS_OK;
  }
  const int nnb = N / 128;
  const int pitch = (4 * Kp + 511) / 512 * 512;
  const int ksteps = (K + 15) / 16;
  int splits = std::max(1, std::min(gemm_cus() / nnb, ksteps / 8));
  int kchunk = ((ksteps + splits - 1) / splits) * 16;
  if (kchunk > 960) kchunk = 960;  // the chunk's ids + row scales in LDS (8 B per row)
  splits = (K + kchunk - 1) / kchunk;
  const int lds = 3 * 16 * pitch + 3 * kH2Tn3BRaw + 2 * kH2Tn3BPl + 512 + 8 * kchunk;
  NTS_CHECK_ARG(lds <= 160 * 1024, "LDS");
  const uint64_t stride = (uint64_t)M * N;
  const size_t part_bytes = splits > 1 ? stride * splits * sizeof(float) : 0;
  float* out = C;
  uint64_t ldo = ldc;
  if (splits > 1) {
    NTS_RET(ensure_scratch(ctx, part_bytes + 256));
    out = (float*)ctx->scratch;
    ldo = N;
  }
  H2Extra ex;  // column scales per chunk: from the producer's per-part maxima, else a pre-pass
  ex.amap = a_rows;
  ex.rs = rs;
  ex.cparts = part_max;
  ex.rpp = rows_per_part;
  ex.nparts_ld = (uint64_t)N;
#ifdef NTS_PROBE_BUILD  // timing probes (scripts/probe): results are garbage
  static const int diag = [] {
    const char* e = getenv("NTS_TN4_DIAG");
    return e ? atoi(e) : 0;
  }();
#endif
#ifndef NTS_TN4_RP  // row-aligned DMA pieces (compile-time A/B: -DNTS_TN4_RP=0)
#define NTS_TN4_RP 1
#endif
  constexpr bool rp = NTS_TN4_RP != 0;
#define NTS_TN4(D, ...)                                                                            \
  do {                                                                                             \
    NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_h2_tn4<TPW, D, ##__VA_ARGS__>), \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds));             \
    hipLaunchKernelGGL((k_h2_tn4<TPW, D, ##__VA_ARGS__>), dim3(nnb * splits), dim3(kH2Tn3Threads), lds, \
                       ctx->stream, M, K, reinterpret_cast<const char*>(Q), ldq * sizeof(uint16_t), \
                       pitch, 2 * Kp, B, ldb, out, ldo, kchunk,                                    \
                       splits > 1 ? stride : (uint64_t)0, nnb, ex);                                \
  } while (0)
#ifdef NTS_PROBE_BUILD
  if (diag == 1) NTS_TN4(1);
  else if (diag == 2) NTS_TN4(2);
  else if (diag == 4) NTS_TN4(4);
  else
#endif
  if (rp && pitch == 2560) NTS_TN4(0, true);
  else NTS_TN4(0);
#undef NTS_TN4
  NTS_LAUNCH_CHECK();
  if (splits == 1) return NTS_OK;
  return sum_splits(ctx->stream, out, splits, stride, M, N, C, ldc);
}

extern "C" int nts_hip_gemm_h2p_tn_gather(nts_hip_ctx* ctx, int M, int N, int K, const uint16_t* Q,
                                          uint64_t ldq, int Kp, const float* rs, const uint32_t* a_rows,
                                          const float* B, uint64_t ldb, float* C, uint64_t ldc) {
  return h2p_tn_gather(ctx, M, N, K, Q, ldq, Kp, rs, a_rows, B, ldb, C, ldc, nullptr, 0);
}

// as nts_hip_gemm_h2p_tn_gather with per-part column maxima of |B| given (part
// p = B rows [p R, (p+1) R), N words each, e.g. by nts_hip_spmm_csr_bwd_colmax):
// the kernel skips its per-chunk pre-pass over B (one read of B instead of two)
extern "C" int nts_hip_gemm_h2p_tn_gather_cm(nts_hip_ctx* ctx, int M, int N, int K, const uint16_t* Q,
                                             uint64_t ldq, int Kp, const float* rs,
                                             const uint32_t* a_rows, const float* B, uint64_t ldb,
                                             float* C, uint64_t ldc, const uint32_t* part_max,
                                             uint32_t rows_per_part) {
  NTS_CHECK_ARG(part_max && rows_per_part > 0, "NULL column maxima");
  return h2p_tn_gather(ctx, M, N, K, Q, ldq, Kp, rs, a_rows, B, ldb, C, ldc, part_max, rows_per_part);
}

// NN v3 on the planar table (k_h2_nn3): N % 128 == 0, Kp <= 640.  The W image
// and its column maxima in scratch, as nts_hip_gemm_h2_gather.
extern "C" int nts_hip_gemm_h2p_gather(nts_hip_ctx* ctx, int relu_dropout, int M, int N, int Kp,
                                       const uint16_t* Q, uint64_t ldq, const float* rs,
                                       const uint32_t* a_rows, const float* W, uint64_t ldw, int K,
                                       float* C, uint64_t ldc, float p, uint64_t seed, uint64_t offset) {
  NTS_CHECK_ARG(ctx, "NULL context");
  NTS_CHECK_ARG(M >= 0 && N > 0 && N % 128 == 0 && K > 0 && Kp >= K && Kp % 32 == 0 &&
                    Kp <= 32 * kH2Nn3KS, "shape");
  NTS_CHECK_ARG(ldq >= 2 * (uint64_t)Kp && ldq % 8 == 0 && (uintptr_t)Q % 16 == 0, "planar table layout");
  NTS_CHECK_ARG(ldw >= (uint64_t)N && ldc >= (uint64_t)N, "ld");
  NTS_CHECK_ARG(ldw % 4 == 0 && (uintptr_t)W % 16 == 0, "W rows must be float4-aligned");
  NTS_CHECK_ARG(M == 0 || (Q && rs && W && C), "NULL buffer");
  NTS_CHECK_ARG(p >= 0.f && p < 1.f, "p must be in [0, 1)");
  if (M == 0) return NTS_OK;
  const int ncb = N / 128, nsteps = Kp / 32;
  const size_t cm_bytes = ((size_t)N * 4 + 255) / 256 * 256;
  const size_t img = (size_t)nsteps * ncb * kH2Img;
  NTS_RET(ensure_scratch(ctx, cm_bytes + img + 256));
  uint32_t* cmax = (uint32_t*)ctx->scratch;
  char* bimg = (char*)ctx->scratch + cm_bytes;
  hipLaunchKernelGGL(k_h2_prep_w, dim3(nsteps, ncb), dim3(512), 0, ctx->stream, W, ldw, K, N, cmax, bimg);
  NTS_LAUNCH_CHECK();
  H2Extra ex;
  ex.keep_threshold = dropout_threshold(p);
  ex.scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  ex.seed = seed;
  ex.offset = offset;
  ex.amap = a_rows;
  ex.rs = rs;
  ex.cmax = cmax;
  const int pitch = (4 * Kp + 511) / 512 * 512;
  const int T = (M + 15) / 16;
  // one block per CU; past the row-id stage's LDS room (8 B per row) more
  // blocks, each with fewer tiles (large bottom frontiers, e.g. C5)
  const int tile_cap = (160 * 1024 - 3 * 16 * pitch) / (2 * 4 * 16);
  NTS_CHECK_ARG(tile_cap >= 1, "row pitch too large for the NN stage");
  int gx = std::max({1, std::min(gemm_cus() / ncb, T), (T + tile_cap - 1) / tile_cap});
  const int max_tiles = (T + gx - 1) / gx;
  const int lds = 3 * 16 * pitch + 2 * 4 * 16 * max_tiles;
  NTS_CHECK_ARG(lds <= 160 * 1024, "row-id stage");
  const dim3 grid(gx, ncb);
#define NTS_H2NN3(E, MP, ...)                                                                     \
  do {                                                                                            \
    NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_h2_nn3<E, MP, ##__VA_ARGS__>), \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds));            \
    hipLaunchKernelGGL((k_h2_nn3<E, MP, ##__VA_ARGS__>), grid, dim3(512), lds, ctx->stream, M, N, Kp,            \
                       reinterpret_cast<const char*>(Q), ldq * sizeof(uint16_t), pitch, 2 * Kp, bimg, C, \
                       ldc, ex);                                                                  \
  } while (0)
#ifdef NTS_PROBE_BUILD  // timing probes (scripts/probe): results are garbage
  static const int diag = [] {
    const char* e = getenv("NTS_NN3_DIAG");
    return e ? atoi(e) : 0;
  }();
#else
  constexpr int diag = 0;
#endif
  // row-aligned LDS-DMA pieces (compile-time A/B: -DNTS_NN3_RP=0 keeps the
  // row-straddling ones)
#ifndef NTS_NN3_RP
#define NTS_NN3_RP 1
#endif
  constexpr bool rp = NTS_NN3_RP != 0;
  // 16-byte row stores from swapped MFMA operands (-DNTS_NN3_TR=1; measured:
  // alone 174-178 -> 168-170 us, in the C2 bench no gain — off by default)
#ifndef NTS_NN3_TR
#define NTS_NN3_TR 0
#endif
  constexpr bool tr = NTS_NN3_TR != 0;
  const bool tr_ok = tr && ldc % 4 == 0 && (uintptr_t)C % 16 == 0;
#ifdef NTS_WITH_H2_NN4
  // four stages (k_h2_nn4) where the table rows carry their scales in a tail
  // (ldq >= 2 Kp + 8 halves: 2560-byte rows) and the step count is compiled
  // in.  Variant builds only (make variant V=nn4 VFLAGS=-DNTS_WITH_H2_NN4):
  // measured no faster than k_h2_nn3 in the C2 bench (r04d: 152.6 vs ~158 us
  // alone, 164.9 vs 170.9 us pipelined)
  if (!relu_dropout && a_rows && pitch == 2560 && ldq >= 2 * (uint64_t)Kp + 8 && nsteps == 19) {
    gx = std::max(gx, (T + 63) / 64);  // <= 64 tiles per block (lane-held row ids)
    constexpr int lds4 = 4 * 16 * 2560;
    NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_h2_nn4<19>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds4));
    hipLaunchKernelGGL((k_h2_nn4<19>), dim3(gx, ncb), dim3(512), lds4, ctx->stream, M, N,
                       reinterpret_cast<const char*>(Q), ldq * sizeof(uint16_t), 2 * Kp, bimg, C,
                       ldc, ex);
    NTS_LAUNCH_CHECK();
    return NTS_OK;
  }
#endif
  // compile-time step counts for the feature widths the driver meets
  // (C2: 602 -> Kp 608); NTS_NN3_DIAG=4 forces the runtime-count loop
  if (relu_dropout) {
    if (a_rows) NTS_H2NN3(true, true); else NTS_H2NN3(true, false);
#ifdef NTS_PROBE_BUILD
  } else if (a_rows && diag == 1) {
    NTS_H2NN3(false, true, 19, 1);
  } else if (a_rows && diag == 2) {
    NTS_H2NN3(false, true, 19, 2);
#endif
  } else if (a_rows && nsteps == 19 && diag != 4 && pitch == 2560 && rp && tr_ok) {
    NTS_H2NN3(false, true, 19, 0, true, true);
  } else if (a_rows && nsteps == 19 && diag != 4 && pitch == 2560 && rp) {
    NTS_H2NN3(false, true, 19, 0, true);
  } else if (a_rows && nsteps == 19 && diag != 4) {
    NTS_H2NN3(false, true, 19);
  } else if (a_rows && nsteps == 20 && diag != 4 && pitch == 2560 && rp && tr_ok) {
    NTS_H2NN3(false, true, 20, 0, true, true);
  } else if (a_rows && nsteps == 20 && diag != 4) {
    NTS_H2NN3(false, true, 20);
  } else {
    if (a_rows) NTS_H2NN3(false, true); else NTS_H2NN3(false, false);
  }
#undef NTS_H2NN3
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

// Dynamic-A NN (k_h2_nnd): K <= 128 with K % 4 == 0 and 16-byte rows, N 128 or
// 256.  W's image and column maxima in scratch (as nts_hip_gemm_h2_gather).
extern "C" int nts_hip_gemm_h2d_act(nts_hip_ctx* ctx, int relu_dropout, int M, int N, int K,
                                    const float* A, uint64_t lda, const float* W, uint64_t ldw,
                                    float* C, uint64_t ldc, float p, uint64_t seed, uint64_t offset,
                                    uint16_t* Q, uint64_t ldq, float* rs) {
  NTS_CHECK_ARG(ctx, "NULL context");
  NTS_CHECK_ARG(M >= 0 && K > 0 && K <= 128 && K % 4 == 0 && (N == 128 || N == 256), "shape");
  NTS_CHECK_ARG(lda >= (uint64_t)K && lda % 4 == 0 && (uintptr_t)A % 16 == 0, "A rows must be 16-byte aligned");
  NTS_CHECK_ARG(ldw >= (uint64_t)N && ldw % 4 == 0 && (uintptr_t)W % 16 == 0 && ldc >= (uint64_t)N, "ld");
  NTS_CHECK_ARG(p >= 0.f && p < 1.f, "p must be in [0, 1)");
  const int nks = (K + 31) / 32;
  NTS_CHECK_ARG(!Q || (rs && ldq >= 2 * (uint64_t)(32 * nks) && ldq % 8 == 0 && (uintptr_t)Q % 16 == 0),
                "pair table output");
  if (M == 0) return NTS_OK;
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  const int ncb = N / 128;
  const size_t cm_bytes = ((size_t)N * 4 + 255) / 256 * 256;
  const size_t img = (size_t)nks * ncb * kH2Img;
  NTS_RET(ensure_scratch(ctx, cm_bytes + img + 256));
  uint32_t* cmax = (uint32_t*)ctx->scratch;
  char* bimg = (char*)ctx->scratch + cm_bytes;
  hipLaunchKernelGGL(k_h2_prep_w, dim3(nks, ncb), dim3(512), 0, ctx->stream, W, ldw, K, N, cmax, bimg);
  NTS_LAUNCH_CHECK();
  H2Extra ex;
  ex.keep_threshold = relu_dropout ? dropout_threshold(p) : 0u;
  ex.scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  ex.seed = seed;
  ex.offset = offset;
  const int T = (M + kH2dTM - 1) / kH2dTM;
  const dim3 grid(std::max(1, std::min(gemm_cus(), T)));  // one block per CU (~156 VGPRs)
#define NTS_H2D(NK, NT, E, QO)                                                                   \
  hipLaunchKernelGGL((k_h2_nnd<NK, NT, E, QO>), grid, dim3(512), 0, ctx->stream, M, K, A, lda,   \
                     bimg, ncb, cmax, C, ldc, Q, ldq, rs, ex)
#define NTS_H2D_NK(NK)                                                                           \
  do {                                                                                           \
    if (N == 256) {                                                                              \
      if (relu_dropout) { if (Q) NTS_H2D(NK, 2, true, true); else NTS_H2D(NK, 2, true, false); } \
      else { if (Q) NTS_H2D(NK, 2, false, true); else NTS_H2D(NK, 2, false, false); }            \
    } else {                                                                                     \
      if (relu_dropout) { if (Q) NTS_H2D(NK, 1, true, true); else NTS_H2D(NK, 1, true, false); } \
      else { if (Q) NTS_H2D(NK, 1, false, true); else NTS_H2D(NK, 1, false, false); }            \
    }                                                                                            \
  } while (0)
  switch (nks) {
    case 1: NTS_H2D_NK(1); break;
    case 2: NTS_H2D_NK(2); break;
    case 3: NTS_H2D_NK(3); break;
    default: NTS_H2D_NK(4);
  }
#undef NTS_H2D_NK
#undef NTS_H2D
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}
