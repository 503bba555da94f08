// fp32 layer GEMMs on the bf16 matrix cores, fp32-accurate (NTS_GEMM_SPLIT3).
//
// gfx950's fp32-input MFMA (v_mfma_f32_16x16x4_f32) runs at 1/16 of the bf16
// rate.  Every fp32 operand x is split exactly into three bf16 pieces
//     x0 = bf16(x),  x1 = bf16(x - x0),  x2 = bf16(x - x0 - x1)
// (round-to-nearest-even each time; x - x0 and x - x0 - x1 are exact in fp32),
// so x0 + x1 + x2 carries x's 24-bit significand (|x - x0 - x1 - x2| <=
// 2^-27 |x|).  A product a·b is then the six bf16 products whose magnitude is
// at least 2^-16 |a b| relative:
//     a0 b0 + a0 b1 + a1 b0 + a0 b2 + a1 b1 + a2 b0
// (dropped: a1 b2, a2 b1, a2 b2, each <= 2^-24 |a b|), each bf16 x bf16
// product exact in the fp32 accumulator of v_mfma_f32_16x16x32_bf16.  Six
// bf16 MFMAs cost 6/16 of one fp32-input MFMA for the same k: 2.7x the fp32
// rate.  The error vs an fp64 GEMM is measured against the native fp32 MFMA
// kernels in tests/test_hip_kernels.py (test_split3_gemm_*).  Values beyond
// bf16's range behave like fp32 except |x| within 2^-8 of FLT_MAX (x0 rounds
// to inf): irrelevant to activations and weights.
//
// Kernels (the same operations and fused extras as gemm.hip's):
//   k_gemm3_nn  C = A B (+ relu/dropout epilogue), A rows optionally gathered
//               through a row map; a 512-thread block streams 32-deep k-slices
//               of B (split and laid out in MFMA fragment order in LDS, double
//               buffered) past 8 waves that each own 2 row tiles x 128 columns.
//   k_s3_tn     C = A^T op(B) (weight gradient; relu/dropout backward fused in
//               the B load), A's k rows optionally gathered: 8-wave blocks
//               over one k-chunk, A^T fragments loaded straight to registers
//               and split there, B staged as bf16 pieces in LDS and read with
//               ds_read_b64_tr_b16, the long reduction split over blocks and
//               summed in a fixed order (sum_splits) — deterministic.
//   k_gemm3_tn  the first-generation TN (NTS_S3_V1=1): a 320 x 128 output
//               tile per block, k-slices of A and B staged transposed into
//               fragment order.
#include "common.hpp"

namespace nts_hip {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kS3Threads = 512;  // 8 waves
constexpr int kS3Frag = 64 * 16;  // bytes of one fragment image (64 lanes x 8 bf16)

// x -> (x0, x1, x2), element-wise over one lane's 8 fragment values
__device__ __forceinline__ void split3(const float (&x)[8], bf16x8& h0, bf16x8& h1, bf16x8& h2) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 a0 = (__bf16)x[j];
    const float r1 = x[j] - (float)a0;
    const __bf16 a1 = (__bf16)r1;
    const float r2 = r1 - (float)a1;
    h0[j] = a0;
    h1[j] = a1;
    h2[j] = (__bf16)r2;
  }
}

// acc += a * b over one 32-deep k-slice, a and b given as split triples
__device__ __forceinline__ f32x4 mfma6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}

// one lane's split triple into a fragment image [piece][lane] (16 B per lane)
__device__ __forceinline__ void put3(char* img, int piece_stride, int lane, const float (&x)[8]) {
  bf16x8 h[3];
  split3(x, h[0], h[1], h[2]);
#pragma unroll
  for (int p = 0; p < 3; ++p) *reinterpret_cast<bf16x8*>(img + p * piece_stride + 16 * lane) = h[p];
}
__device__ __forceinline__ void get3(const char* img, int piece_stride, int lane, bf16x8 (&h)[3]) {
#pragma unroll
  for (int p = 0; p < 3; ++p) h[p] = *reinterpret_cast<const bf16x8*>(img + p * piece_stride + 16 * lane);
}

struct Gemm3Extra {
  uint32_t keep_threshold = 0;  // EPI: relu + inverted dropout (common.hpp dropout_*)
  float scale = 1.f;
  uint64_t seed = 0, offset = 0;
  const float* bx = nullptr;  // BMASK: B = G * bscale where X > 0
  uint64_t ldbx = 0;
  float bscale = 1.f;
  const uint32_t* amap = nullptr;  // gathered A rows (NN: M rows, TN: K rows)
#ifdef NTS_PROBE_BUILD
  int diag = 0;  // NTS_S3_DIAG timing probes (results invalid): 1 no global loads,
                 // 2 no split, 4 no barrier, 8 no MFMA, 16 no B fragment reads
#else
  static constexpr int diag = 0;  // the product library has no timing probes
#endif
};

// ---------------------------------------------------------------------------
// B pre-split (NN): the weight [K x N] as the bf16 fragment image of
// v_mfma_f32_16x16x32_bf16 that the NN kernel's blocks stage into LDS each
// 32-deep k-step:
//   img[s][cb][ct][piece][lane] (16 B) =
//       piece of B[32 s + 8 (lane >> 4) + j][128 cb + 16 ct + (lane & 15)]
// zero past K and N.  One launch per GEMM (the weight changes every step).
constexpr int kS3Img = 8 * 3 * kS3Frag;  // one (step, column block) image: 24 KB

__global__ __launch_bounds__(256) void k_split3_b(const float* __restrict__ B, uint64_t ldb, int K,
                                                  int N, int total, int ncb, char* __restrict__ out) {
  const int id = blockIdx.x * 256 + threadIdx.x;
  if (id >= total) return;
  const int lane = id & 63, ct = (id >> 6) & 7, rest = id >> 9;
  const int cb = rest % ncb, s = rest / ncb;
  const int col = cb * 128 + ct * 16 + (lane & 15);
  const int k0 = 32 * s + 8 * (lane >> 4);
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (col < N && k0 + j < K) ? B[(uint64_t)(k0 + j) * ldb + col] : 0.f;
  put3(out + (size_t)rest * kS3Img + ct * 3 * kS3Frag, kS3Frag, lane, x);
}

// ---------------------------------------------------------------------------
// The global_load_lds instructions are issued from inline asm: hipcc cannot
// tell the stages of one LDS array apart and, for a compiler-visible LDS DMA,
// waits vmcnt(0) before the next ds_read of ANY stage (draining the
// pipeline).  Their completion is counted by hand (s_waitcnt vmcnt(N)); the
// only compiler-visible global loads of the k-loop (the partial last step)
// come after a vmcnt(0).
typedef __attribute__((address_space(3))) void* lds_ptr_t;
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(lds_ptr_t)p;
}
// 16 bytes per lane from `src` to LDS (wave-uniform base `lds`) + 16 * lane
__device__ __forceinline__ void glds16(const void* src, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// NN.  Block = 8 waves (two per SIMD), one column block of 128 per grid.y.
// The M rows are cut into 16-row tiles; wave gw of the grid owns the
// contiguous tiles [gw T / W, (gw+1) T / W) and processes them two at a time
// in `rounds` rounds (one count for all, so a block's waves stay in step
// over the shared B slices; a wave with one tile left runs the one-tile
// path).  Both operands reach LDS by global_load_lds (no VGPR staging), all
// in ONE shared array:
//   B: the pre-split image of step s (24 KB, 3 x 1 KB per wave), 2 stages;
//   A: each wave's 2 x (16 rows x 32 k) fp32 slab of step s, 3 stages, laid
//      out so that lane (i, g)'s fragment A[row i][k0 + 8g .. +7] is the 32
//      bytes at 32 (i + 16 g) of its tile.
// Step s waits (counted vmcnt, raw s_barrier: nothing drains the pipeline)
// for B(s) and A(s), then issues B(s+1) and A(s+2), reads its fragments,
// splits A, and runs 8 column tiles x 6 MFMAs per row tile.  The partial
// last k-step (K % 32) is loaded to registers with clamped loads after the
// pipeline has drained (no over-read past a row).  Each output element is a
// fixed-order chain: deterministic.  Blocks x and x + gridDim.x·y (the
// column blocks of the same rows) sit on the same XCD when gridDim.x % 8 ==
// 0: A's second read hits L2.
constexpr int kS3NnThreads = 512;
constexpr int kS3NnAWave = 2 * 2048;             // one wave's A slab of a step
constexpr int kS3NnA = 8 * kS3NnAWave;           // one A stage
constexpr int kS3NnLds = 2 * kS3Img + 3 * kS3NnA;  // 48 + 96 KB

template <bool EPI, bool AMAP>
__global__ __launch_bounds__(kS3NnThreads, 1) void k_gemm3_nn(int M, int N, int K,
                                                             const float* __restrict__ A, uint64_t lda,
                                                             const char* __restrict__ bimg,
                                                             float* __restrict__ C, uint64_t ldc,
                                                             int rounds, Gemm3Extra ex) {
  extern __shared__ __attribute__((aligned(16))) char s3nn[];
  char* const sb = s3nn;               // [2][kS3Img]
  char* const sa = s3nn + 2 * kS3Img;  // [3][8 waves][2 tiles][2048]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.y * 128;
  const int T = (M + 15) / 16;
  const int64_t W = (int64_t)gridDim.x * 8;
  const int64_t gw = (int64_t)blockIdx.x * 8 + wv;
  const int t_lo = (int)(gw * T / W), t_hi = (int)((gw + 1) * T / W);
  const int nsteps = (K + 31) / 32, nfull = K / 32;
  const size_t bstride = (size_t)gridDim.y * kS3Img;
  const uint32_t lsb = lds_addr(sb), lsa = lds_addr(sa);
  // B image copy role: 3 x 1 KB per wave per step
  const char* bsrc = bimg + (size_t)blockIdx.y * kS3Img + wv * 1024 + 16 * lane;
  // A glds role: lane l loads row (l >> 1) & 15, floats 8 (l >> 5) + 4 (l & 1) (+ 16 q)
  const int gr = (lane >> 1) & 15, gpo = 8 * (lane >> 5) + 4 * (lane & 1);
  const float* arow[2];
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
    if (ex.diag & 1) return;
    const uint32_t dst = lsb + (s & 1) * kS3Img + wv * 1024;
    const char* src = bsrc + (size_t)s * bstride;
#pragma unroll
    for (int p = 0; p < 3; ++p) glds16(src + 8192 * p, dst + 8192 * p);
  };
  auto issue_a = [&](int s) {
    if (ex.diag & 1) return;
    const uint32_t dst = lsa + (s % 3) * kS3NnA + wv * kS3NnAWave;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int q = 0; q < 2; ++q) glds16(arow[rt] + 32 * s + 16 * q, dst + rt * 2048 + q * 1024);
  };
  f32x4 acc[2][8];
  // split the row tiles' fragments and run the MFMAs of step s against B(s)
  auto mma = [&](int s, const float (&x)[2][8], bool two) {
    bf16x8 a[2][3];
    if (ex.diag & 2) {
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int p = 0; p < 3; ++p) a[rt][p] = *reinterpret_cast<const bf16x8*>(&x[rt][0]);
    } else {
      split3(x[0], a[0][0], a[0][1], a[0][2]);
      split3(x[1], a[1][0], a[1][1], a[1][2]);
    }
    if (ex.diag & 8) return;
    const char* img = sb + (s & 1) * kS3Img;
    if (ex.diag & 16) {  // no B reads: the A pieces stand in for B
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
        acc[0][ct] = mfma6(a[0], a[1], acc[0][ct]);
        acc[1][ct] = mfma6(a[1], a[0], acc[1][ct]);
      }
      return;
    }
    if (two) {
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
        bf16x8 b[3];
        get3(img + ct * 3 * kS3Frag, kS3Frag, lane, b);
        acc[0][ct] = mfma6(a[0], b, acc[0][ct]);
        acc[1][ct] = mfma6(a[1], b, acc[1][ct]);
      }
    } else {
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
        bf16x8 b[3];
        get3(img + ct * 3 * kS3Frag, kS3Frag, lane, b);
        acc[0][ct] = mfma6(a[0], b, acc[0][ct]);
      }
    }
  };

  for (int rd = 0; rd < rounds; ++rd) {
    const int nt = min(2, max(0, t_hi - (t_lo + 2 * rd)));  // this wave's tiles this round
    set_rows(rd);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) acc[rt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    issue_b(0);
    if (nfull > 0) issue_a(0);
    if (nfull > 1) issue_a(1);
    for (int s = 0; s < nsteps; ++s) {
      // B(s) and A(s) landed (A(s+1), issued after B(s), may stay in flight)
#ifdef NTS_S3NN_COUNTED  // (A/B build: the counted wait)
      if (s + 1 < nfull) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else  // drained: the LDS-DMA loads need not retire in issue order (k_x3_tn, round 6)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
      if (!(ex.diag & 4)) raw_barrier();
      if (s + 1 < nsteps) issue_b(s + 1);
      if (s + 2 < nfull) issue_a(s + 2);
      float x[2][8];
      if (s < nfull) {
        const char* as = sa + (s % 3) * kS3NnA + wv * kS3NnAWave + 32 * (i + 16 * g);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
          const float4 u = *reinterpret_cast<const float4*>(as + rt * 2048);
          const float4 v = *reinterpret_cast<const float4*>(as + rt * 2048 + 16);
          x[rt][0] = u.x; x[rt][1] = u.y; x[rt][2] = u.z; x[rt][3] = u.w;
          x[rt][4] = v.x; x[rt][5] = v.y; x[rt][6] = v.z; x[rt][7] = v.w;
        }
      } else {  // the partial step: clamped loads of the fragment layout, masked
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
          const int t = min(t_lo + 2 * rd + rt, T - 1);
          const int64_t row = (int64_t)t * 16 + i;
          const uint64_t rr = (uint64_t)(row < M ? row : M - 1);
          const float* pr = A + (AMAP ? (uint64_t)ex.amap[rr] : rr) * lda;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int k = 32 * s + 8 * g + j;
            const float v = pr[min(k, K - 1)];
            x[rt][j] = k < K ? v : 0.f;
          }
        }
      }
      if (nt > 0) mma(s, x, nt == 2);
    }
    raw_barrier();  // every wave is done with the B stages before the next round's
    // epilogue: acc[rt][ct][v] = C[16 t + 4 g + v][n0 + 16 ct + i]
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      if (rt >= nt) continue;
      const int64_t r4 = (int64_t)(t_lo + 2 * rd + rt) * 16 + 4 * g;
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
        const uint32_t col = (uint32_t)(n0 + 16 * ct + i);
        if ((int)col >= N) continue;
        float o[4] = {acc[rt][ct][0], acc[rt][ct][1], acc[rt][ct][2], acc[rt][ct][3]};
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
// NN for short reductions (K <= 128, dense rows: the aggregate-first bottom
// layers of the products-shaped C3 / C4, Z = relu/dropout(Y W0) with Y
// [~140 K x 100]).  k_gemm3_nn streams the W image step by step and pipelines
// A through LDS over the k-loop; with <= 4 k-steps a round that is all
// prologue (110 us for C3's layer, no faster than the fp32-input kernel).
// Here each block keeps its column block's WHOLE image (nsteps x 24 KB) in
// LDS for its lifetime and each wave loops over 32-row tiles (grid-strided),
// A loaded straight to registers:
// per k-step the two row tiles' fragments split in registers, 8 column tiles
// x 6 MFMAs each (the pieces, products, k order and instruction of
// k_gemm3_nn: bit-identical), relu/dropout in the epilogue.
// two waves per SIMD (<= 256 registers each: no next-tile A in registers; the
// other wave covers the loads) so one wave's epilogue VALU — the dropout
// Philox rounds, as many cycles as the tile's MFMAs — overlaps the other's
// MFMAs
constexpr int kX3KThreads = 512;
constexpr int kX3KSteps = 4;  // K <= 128

// lane i and its neighbour i ^ 1 hold the two columns of one Philox column
// pair (dropout_words keys (row / 4, col / 2)): each computes one of two
// column tiles' words and takes the other's from its neighbour (DPP swap)
__device__ __forceinline__ uint32_t x3k_swap(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}

template <bool EPI>
__global__ __launch_bounds__(kX3KThreads, 1) void k_x3_nnk(int M, int N, int K,
                                                          const float* __restrict__ A, uint64_t lda,
                                                          const char* __restrict__ bimg,
                                                          float* __restrict__ C, uint64_t ldc,
                                                          Gemm3Extra ex) {
  extern __shared__ __attribute__((aligned(16))) char x3k[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int cb = blockIdx.y, ncb = gridDim.y, n0 = cb * 128;
  const int nsteps = (K + 31) / 32;
  // the column block's image of every step: [s][ct][piece][lane], by LDS DMA
  // (1 KB a wave instruction, no registers; inline asm, so the wait is ours)
  {
    const int wu = __builtin_amdgcn_readfirstlane(wv);
    const uint32_t lds0 = lds_addr(x3k);
    for (int c = wu; c < nsteps * (kS3Img / 1024); c += kX3KThreads / 64) {
      const int o = c * 1024, s = o / kS3Img, r = o - s * kS3Img;
      glds16(bimg + ((size_t)s * ncb + cb) * kS3Img + r + 16 * lane, lds0 + (uint32_t)o);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const int T = (M + 31) / 32;
  const int W = gridDim.x * (kX3KThreads / 64), gw = blockIdx.x * (kX3KThreads / 64) + wv;
  // lane (i, g)'s fragments of a tile: rows 32 t + 16 rt + i, k = 32 s + 8 g + j
  auto load = [&](int t, float (&x)[2][kX3KSteps][8]) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int64_t row = (int64_t)t * 32 + 16 * rt + i;
      const float* pr = A + (uint64_t)(row < M ? row : M - 1) * lda;
#pragma unroll
      for (int s = 0; s < kX3KSteps; ++s) {
        const int k0 = 32 * s + 8 * g;
        if (k0 + 8 <= K) {
          const float4 u = *reinterpret_cast<const float4*>(pr + k0);
          const float4 v = *reinterpret_cast<const float4*>(pr + k0 + 4);
          x[rt][s][0] = u.x; x[rt][s][1] = u.y; x[rt][s][2] = u.z; x[rt][s][3] = u.w;
          x[rt][s][4] = v.x; x[rt][s][5] = v.y; x[rt][s][6] = v.z; x[rt][s][7] = v.w;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float val = pr[min(k0 + j, K - 1)];
            x[rt][s][j] = k0 + j < K ? val : 0.f;
          }
        }
      }
    }
  };
  for (int t = gw; t < T; t += W) {
    float cur[2][kX3KSteps][8];
    load(t, cur);
    f32x4 acc[2][8];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) acc[rt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kX3KSteps; ++s) {
      if (s < nsteps) {
        bf16x8 a[2][3];
        split3(cur[0][s], a[0][0], a[0][1], a[0][2]);
        split3(cur[1][s], a[1][0], a[1][1], a[1][2]);
        const char* img = x3k + s * kS3Img;
#pragma unroll
        for (int ct = 0; ct < 8; ++ct) {
          bf16x8 b[3];
          get3(img + ct * 3 * kS3Frag, kS3Frag, lane, b);
          acc[0][ct] = mfma6(a[0], b, acc[0][ct]);
          acc[1][ct] = mfma6(a[1], b, acc[1][ct]);
        }
      }
    }
    // epilogue: acc[rt][ct][v] = C[32 t + 16 rt + 4 g + v][n0 + 16 ct + i];
    // per column-tile pair one Philox call a lane, shared with the neighbour
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int64_t r4 = (int64_t)t * 32 + 16 * rt + 4 * g;
#pragma unroll
      for (int cp = 0; cp < 4; ++cp) {
        uint4 wd[2];
        if constexpr (EPI) {
          const int ctm = 2 * cp + (i & 1);  // the tile this lane's call serves
          const uint4 w = dropout_words((uint64_t)r4, (uint32_t)(n0 + 16 * ctm + i), ex.seed, ex.offset);
          const uint4 o = make_uint4(x3k_swap(w.x), x3k_swap(w.y), x3k_swap(w.z), x3k_swap(w.w));
          wd[0] = (i & 1) ? o : w;
          wd[1] = (i & 1) ? w : o;
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int ct = 2 * cp + h;
          const uint32_t col = (uint32_t)(n0 + 16 * ct + i);
          if ((int)col >= N) continue;
          float o[4] = {acc[rt][ct][0], acc[rt][ct][1], acc[rt][ct][2], acc[rt][ct][3]};
          if constexpr (EPI) {
            const uint32_t wv4[4] = {wd[h].x, wd[h].y, wd[h].z, wd[h].w};
#pragma unroll
            for (int v = 0; v < 4; ++v)
              o[v] = (dropout_bits(wv4[v], col) >= ex.keep_threshold && o[v] > 0.f) ? o[v] * ex.scale : 0.f;
          }
#pragma unroll
          for (int v = 0; v < 4; ++v)
            if (r4 + v < M) C[(uint64_t)(r4 + v) * ldc + col] = o[v];
        }
      }
    }
  }
}

bool x3_nnk_ok(int M, int N, int K, const float* A, uint64_t lda) {
  return K >= 1 && K <= 32 * kX3KSteps && M >= 4096 && N >= 1 && lda >= (uint64_t)K && lda % 4 == 0 &&
         (uintptr_t)A % 16 == 0;
}

// ---------------------------------------------------------------------------
// TN: C[M x N] = A[K x M]^T op(B)[K x N].  Block = 8 waves, output tile 160
// rows (10 row tiles) x 128 columns; wave (wm, wn) = (wv & 1, wv >> 1) owns
// row tiles 5 wm .. 5 wm + 4 and column tiles 2 wn, 2 wn + 1 (40
// accumulators).  Per 32-deep k-step thread t (c = t & 127, kg = t >> 7)
// loads the 8 k rows 8 kg .. 8 kg + 7 of A at columns r0 + c (and r0 + 128 + c
// for c < 32) and of B at column n0 + c: each (column, kg) is exactly one
// lane's fragment (lane = (column & 15) + 16 kg), split and stored with 3
// ds_write_b128.  Two LDS stages (108 KB); the loads of step s+2 are issued
// during step s.  Waves 0-3 run MFMAs then stage, waves 4-7 stage then run
// MFMAs, so each SIMD's two waves overlap the split (VALU) with the MFMAs
// (one barrier per step).  With a row map the row ids of step s+3 are read
// during step s.
constexpr int kS3TnRows = 160;
struct S3TnSmem {
  char a[2][10 * 3 * kS3Frag];  // [stage][rt][piece][lane]
  char b[2][8 * 3 * kS3Frag];   // [stage][ct][piece][lane]
};

template <bool BMASK, bool AMAP>
__global__ __launch_bounds__(kS3Threads, 1) void k_gemm3_tn(int M, int N, int K, const float* __restrict__ A,
                                                           uint64_t lda, const float* __restrict__ B,
                                                           uint64_t ldb, float* __restrict__ C,
                                                           uint64_t ldc, int kchunk,
                                                           uint64_t split_stride, int nrg, int ncb,
                                                           Gemm3Extra ex) {
  extern __shared__ __attribute__((aligned(16))) char s3raw[];
  S3TnSmem& sm = *reinterpret_cast<S3TnSmem*>(s3raw);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv & 1, wn = wv >> 1;
  const bool lead = wv < 4;
  const int rg = blockIdx.x % nrg;
  const int cb = (blockIdx.x / nrg) % ncb;
  const int split = blockIdx.x / (nrg * ncb);
  const int r0 = rg * kS3TnRows, n0 = cb * 128;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int nsteps = kbeg < kend ? (kend - kbeg + 31) / 32 : 0;
  const int c = tid & 127, kg = tid >> 7;
  const bool two = c < 32;  // second A column r0 + 128 + c
  const bool aok0 = r0 + c < M, aok1 = two && r0 + 128 + c < M;
  const int acol0 = aok0 ? r0 + c : 0, acol1 = aok1 ? r0 + 128 + c : 0;
  const bool bok = n0 + c < N;
  const float* bcol = B + (bok ? n0 + c : 0);
  const float* xcol = BMASK ? ex.bx + (bok ? n0 + c : 0) : nullptr;
  uint32_t rnext[8];  // A row ids of the next step to load
  auto map_rows = [&](int s, uint32_t (&rr)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = min(kbeg + 32 * s + 8 * kg + j, K - 1);
      rr[j] = AMAP ? ex.amap[k] : (uint32_t)k;
    }
  };
  // two register staging sets (step parity): the loads of step s+3 are issued
  // during step s and written to LDS during step s+2
  struct Stage {
    float a0[8], a1[8], b[8], x[BMASK ? 8 : 1];
  };
  Stage sg0, sg1;
  auto load = [&](int s, Stage& q) {
    if (ex.diag & 1) return;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float* arow = A + (uint64_t)rnext[j] * lda;
      q.a0[j] = arow[acol0];
      q.a1[j] = arow[acol1];  // unconditional (a select here makes hipcc wait per load)
      const uint64_t k = (uint64_t)min(kbeg + 32 * s + 8 * kg + j, K - 1);
      q.b[j] = bcol[k * ldb];
      if constexpr (BMASK) q.x[j] = xcol[k * ex.ldbx];
    }
  };
  auto store = [&](int s, const Stage& q) {
    if (ex.diag & 2) return;
    const int st = s & 1;
    const int kl = kend - (kbeg + 32 * s + 8 * kg);  // valid k rows of this thread's 8
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (aok0 && j < kl) ? q.a0[j] : 0.f;
    put3(sm.a[st] + (c >> 4) * 3 * kS3Frag, kS3Frag, (c & 15) + 16 * kg, x);
    if (two) {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (aok1 && j < kl) ? q.a1[j] : 0.f;
      put3(sm.a[st] + (8 + (c >> 4)) * 3 * kS3Frag, kS3Frag, (c & 15) + 16 * kg, x);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float bb = q.b[j];
      if constexpr (BMASK) bb = q.x[j] > 0.f ? bb * ex.bscale : 0.f;
      x[j] = (bok && j < kl) ? bb : 0.f;
    }
    put3(sm.b[st] + (c >> 4) * 3 * kS3Frag, kS3Frag, (c & 15) + 16 * kg, x);
  };
  f32x4 acc[5][2];
#pragma unroll
  for (int q = 0; q < 5; ++q)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) acc[q][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int s) {
    if (ex.diag & 8) return;
    const int st = s & 1;
    bf16x8 b[2][3], a[2][3];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) get3(sm.b[st] + (2 * wn + ct) * 3 * kS3Frag, kS3Frag, lane, b[ct]);
    get3(sm.a[st] + (5 * wm) * 3 * kS3Frag, kS3Frag, lane, a[0]);
#pragma unroll
    for (int q = 0; q < 5; ++q) {  // row tile q+1's fragments are read during q's MFMAs
      if (q + 1 < 5) get3(sm.a[st] + (5 * wm + q + 1) * 3 * kS3Frag, kS3Frag, lane, a[(q + 1) & 1]);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) acc[q][ct] = mfma6(a[q & 1], b[ct], acc[q][ct]);
    }
  };
  // prologue: step 0 staged, steps 1 and 2 in flight
  if (nsteps > 0) {
    map_rows(0, rnext);
    load(0, sg0);
    store(0, sg0);
    map_rows(1, rnext);
    if (nsteps > 1) load(1, sg1);
    map_rows(2, rnext);
    if (nsteps > 2) load(2, sg0);
    map_rows(3, rnext);
  }
  __syncthreads();
  // step s: stage s+1 from set (s+1)&1, refill it with step s+3
  auto step = [&](int s, Stage& q) {
    if (lead) {
      compute(s);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (s + 1 < nsteps) store(s + 1, q);
    if (s + 3 < nsteps) {
      load(s + 3, q);
      map_rows(s + 4, rnext);
    }
    if (!lead) {
      __builtin_amdgcn_sched_barrier(0);
      compute(s);
    }
    __syncthreads();
  };
  for (int s = 0; s < nsteps; s += 2) {
    step(s, sg1);
    if (s + 1 < nsteps) step(s + 1, sg0);
  }
  // acc[q][ct][v] = C[r0 + 16 (5 wm + q) + 4 g + v][n0 + 16 (2 wn + ct) + i]
  const int i = lane & 15, g = lane >> 4;
  float* Cb = C + (uint64_t)split * split_stride;
#pragma unroll
  for (int q = 0; q < 5; ++q)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int row = r0 + 16 * (5 * wm + q) + 4 * g + v;
      if (row >= M) continue;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const int col = n0 + 16 * (2 * wn + ct) + i;
        if (col < N) Cb[(uint64_t)row * ldc + col] = acc[q][ct][v];
      }
    }
}

// ---------------------------------------------------------------------------
// TN v2 (the default for TN; NTS_S3_V1=1 selects k_gemm3_tn above): two
// waves per SIMD, every operand software-pipelined in registers ahead of its
// MFMAs, the split of step s+1 beside the MFMAs of step s (the loads and
// splits of the last steps are skipped by uniform branches: clamped
// unconditional ones measured slower here, their live ranges spill).
// TN: C[M x N] = A[K x M]^T op(B)[K x N] (weight gradient; A's K rows
// optionally gathered through a row map, op(B) = B or the relu/dropout
// backward B * bscale where X > 0).  An 8-wave block takes one k-chunk, a
// range of A's 16-column tiles (M-dimension tiles split evenly over the
// blocks, then over the waves, at most TPW per wave; a missing tile is a
// clamped duplicate that is not stored) and 128 columns of B.  The chunks'
// partial tiles are summed in a fixed order (sum_splits): deterministic.
//   A^T fragments come straight from global memory into registers: lane
//     (i, g) of tile t loads A[k0 + 8g + j][16 t + i] (j = 0..7, one dword
//     each, rows through the map; ids a step before the values, the values
//     two steps before their MFMAs) and splits them one step ahead;
//   B rows are loaded 8 floats per thread, masked, split and written to LDS
//     as three bf16 images with plain 256-byte rows (16-byte chunks
//     XOR-swizzled), double-buffered, and read back TRANSPOSED as MFMA B
//     fragments by ds_read_b64_tr_b16 (k rows 8g..8g+3 and 8g+4..8g+7 of the
//     fragment's 16 columns).
constexpr int kS3TnV2Threads = 512;
constexpr int kS3TnV2Img = 32 * 256;            // one piece of one step: 32 rows x 128 bf16
constexpr int kS3TnV2Lds = 2 * 3 * kS3TnV2Img;  // 2 stages x 3 pieces = 48 KB

// byte offset of 16-byte chunk `ch` (0..15) of row `row` in a [32][256 B] image
__device__ __forceinline__ int s3_tr_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <int TPW, bool BMASK, bool AMAP>
__global__ __launch_bounds__(kS3TnV2Threads, 1) void k_s3_tn(int M, int N, int K,
                                                             const float* __restrict__ A, uint64_t lda,
                                                             const float* __restrict__ B, uint64_t ldb,
                                                             float* __restrict__ C, uint64_t ldc,
                                                             int kchunk, uint64_t split_stride,
                                                             int nmb, int nnb, Gemm3Extra ex) {
  extern __shared__ __attribute__((aligned(16))) char s3tn[];  // [2][3][kS3TnV2Img]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, g = lane >> 4;
  const int mb = blockIdx.x % nmb;
  const int nb = (blockIdx.x / nmb) % nnb;
  const int split = blockIdx.x / (nmb * nnb);
  const int n0 = nb * 128;
  const int T = (M + 15) / 16;
  const int b_lo = mb * T / nmb, b_cnt = (mb + 1) * T / nmb - b_lo;
  const int w_lo = b_lo + wv * b_cnt / 8, w_hi = b_lo + (wv + 1) * b_cnt / 8;  // this wave's tiles
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int nsteps = kbeg < kend ? (kend - kbeg + 31) / 32 : 0;

  int acol[TPW];  // this lane's A column per tile (clamped)
#pragma unroll
  for (int t = 0; t < TPW; ++t) acol[t] = min(16 * min(w_lo + t, max(w_hi - 1, w_lo)) + i, M - 1);
  // B staging role: row br = tid >> 4 of the step, columns bc .. bc + 7
  const int br = tid >> 4, bc = 8 * (tid & 15);
  const bool bok = n0 + bc < N;  // N % 16 == 0
  const float* bcol = B + (bok ? n0 + bc : 0);
  const float* xcol = BMASK ? ex.bx + (bok ? n0 + bc : 0) : nullptr;

  f32x4 acc[TPW][8];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int ct = 0; ct < 8; ++ct) acc[t][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint32_t rid[2][8];   // A row ids of two steps
  float xa[TPW][8];     // raw A^T fragments of the next step (per tile)
  bf16x8 pa[TPW][3];    // split pieces of the current step
  float4 braw[2], xraw[BMASK ? 2 : 1];

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
  // one tile's fragment of step s (rows past the chunk zeroed: the pad may hold anything)
  auto load_x = [&](int s, const uint32_t (&r)[8], int t) {
    const int k0 = kbeg + 32 * s + 8 * g;
#pragma unroll
    for (int j = 0; j < 8; ++j) xa[t][j] = A[(uint64_t)r[j] * lda + acol[t]];
    if (k0 + 8 > kend) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (k0 + j >= kend) xa[t][j] = 0.f;
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
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ok ? v[u] : 0.f;
    bf16x8 q0, q1, q2;
    split3(v, q0, q1, q2);
    char* dst = s3tn + buf * 3 * kS3TnV2Img + s3_tr_off(br, bc / 8);
    *reinterpret_cast<bf16x8*>(dst) = q0;
    *reinterpret_cast<bf16x8*>(dst + kS3TnV2Img) = q1;
    *reinterpret_cast<bf16x8*>(dst + 2 * kS3TnV2Img) = q2;
  };
  // transposed fragment reads: lane 4q+p of each 16-lane group addresses row
  // r0 + q, columns 4p .. 4p+3 of the column tile (chunk 2 ct + (p >> 1), +8 B)
  const int tq = (lane & 15) >> 2, tp = lane & 3;
  const int off_lo = s3_tr_off(8 * g + tq, tp >> 1) + 8 * (tp & 1);
  const int off_hi = s3_tr_off(8 * g + 4 + tq, tp >> 1) + 8 * (tp & 1);
  auto read_b = [&](int buf, int ct, bf16x8 (&b)[3]) {
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) {
      const char* img = s3tn + (buf * 3 + pc) * kS3TnV2Img;
      // chunk 2 ct + c: the XOR swizzle acts on the low 4 chunk bits, and
      // 2 ct only touches bits the row-dependent XOR also touches, so apply
      // it to the chunk index (ch ^ f) = (2ct + c) ^ f = 2ct ^ (c ^ f) for c < 2
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s16x4*)(img + (off_lo ^ (32 * ct))));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s16x4*)(img + (off_hi ^ (32 * ct))));
      const s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      b[pc] = __builtin_bit_cast(bf16x8, c);
    }
  };

  if (nsteps > 0) {
    load_ids(0, rid[0]);
    if (nsteps > 1) load_ids(1, rid[1]);
#pragma unroll
    for (int t = 0; t < TPW; ++t) load_x(0, rid[0], t);
#pragma unroll
    for (int t = 0; t < TPW; ++t) split3(xa[t], pa[t][0], pa[t][1], pa[t][2]);
    if (nsteps > 1)
#pragma unroll
      for (int t = 0; t < TPW; ++t) load_x(1, rid[1], t);
    if (nsteps > 2) load_ids(2, rid[0]);
    load_b(0);
    store_b(0, 0);
    if (nsteps > 1) load_b(1);
  }
  // step s: B pieces of s in buffer s&1, A pieces of s in pa, raw A of s+1 in
  // xa, ids of s+2 in rid[s&1], raw B of s+1 in braw.  Tile by tile: the
  // tile's 8 x 6 MFMAs, then its pieces of s+1 (split beside the next tile's
  // MFMAs) and the loads of its fragment of s+2.
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
        bf16x8 b[3];
        read_b(P, ct, b);
        acc[t][ct] = mfma6(pa[t], b, acc[t][ct]);
      }
      if (s + 1 < nsteps) split3(xa[t], pa[t][0], pa[t][1], pa[t][2]);
      if (s + 2 < nsteps) load_x(s + 2, rid[P], t);
    }
  };
  for (int s = 0; s < nsteps; s += 2) {
    step(s, std::integral_constant<int, 0>());
    if (s + 1 < nsteps) step(s + 1, std::integral_constant<int, 1>());
  }
  // acc[t][ct][v] = C[16 (w_lo + t) + 4 g + v][n0 + 16 ct + i]
  float* Cb = C + (uint64_t)split * split_stride;
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
        if (col < N) Cb[(uint64_t)row * ldc + col] = acc[t][ct][v];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// launchers (called by gemm.hip's dispatcher when the context's GEMM mode is
// NTS_GEMM_SPLIT3 and the shape qualifies)

// NN: the A rows are read by 16-byte global_load_lds (row pitch and base
// 16-byte aligned)
bool gemm3_nn_ok(int M, int N, int K, const float* A, uint64_t lda) {
  return M >= 256 && K >= 1 && N % 16 == 0 && lda % 4 == 0 && (uintptr_t)A % 16 == 0;
}
bool gemm3_tn_ok(int M, int N, int K) { return M >= 1 && K >= 256 && N % 16 == 0; }

// NTS_S3_V1=1: the first-generation TN kernel (k_gemm3_tn), for A/B.  (A
// second-generation NN kernel with the same register pipeline as k_s3_tn
// measured equal to k_gemm3_nn on the gathered shape and slower on the dense
// one — DESIGN §3 — so NN keeps k_gemm3_nn.)
static bool use_v1() {  // compile-time A/B: -DNTS_S3_V1=1
#ifdef NTS_S3_V1
  return NTS_S3_V1 != 0;
#else
  return false;
#endif
}

int gemm3_nn(nts_hip_ctx* ctx, bool epi, int M, int N, int K, const float* A, uint64_t lda,
             const uint32_t* amap, const float* B, uint64_t ldb, float* C, uint64_t ldc,
             uint32_t keep_threshold, float scale, uint64_t seed, uint64_t offset) {
  Gemm3Extra ex;
  ex.keep_threshold = keep_threshold;
  ex.scale = scale;
  ex.seed = seed;
  ex.offset = offset;
  ex.amap = amap;
#ifdef NTS_PROBE_BUILD
  static const int diag = [] {
    const char* e = getenv("NTS_S3_DIAG");
    return e ? atoi(e) : 0;
  }();
  ex.diag = diag;
#endif
  const int ncb = (N + 127) / 128;
  const int nsteps = (K + 31) / 32;
  // the weight's fragment image (scratch: the NN call uses no other scratch)
  const size_t img = (size_t)nsteps * ncb * kS3Img;
  NTS_RET(ensure_scratch(ctx, img + 256));
  char* bimg = (char*)ctx->scratch;
  const int total = nsteps * ncb * 512;  // (s, cb, ct, lane)
  hipLaunchKernelGGL(k_split3_b, dim3((total + 255) / 256), dim3(256), 0, ctx->stream, B, ldb, K,
                     N, total, ncb, bimg);
  NTS_LAUNCH_CHECK();
#ifndef NTS_NO_X3  // (variant builds: -DNTS_NO_X3 keeps k_gemm3_nn for A/B)
  // the row-gathered NN (k_x3_nn / k_x3_nn7); dense rows reach k_x3_nn7 (and
  // its relu/dropout epilogue) only under NTS_GEMM_SPLIT3_ALL: on C3's dense
  // 100-wide bottom layer it measured 124 us vs 60 us on k_h2_nnd (round 6)
  if ((amap && x3_nn_ok(M, N, K, A, lda)) ||
      (ctx->gemm_mode == NTS_GEMM_SPLIT3_ALL && x3_nn7_ok(M, N, K, A, lda)))
    return x3_nn(ctx, epi, M, N, K, A, lda, amap, bimg, C, ldc, keep_threshold, scale, seed, offset);
#endif
  if (!amap && x3_nnk_ok(M, N, K, A, lda)) {  // short reductions, dense rows
    const int G = std::max(1, std::min(256 / ncb, ((M + 31) / 32 + 7) / 8));
    const int lds = nsteps * kS3Img;
#define NTS_X3K(E)                                                                                 \
  do {                                                                                             \
    NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_x3_nnk<E>),                  \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds));             \
    hipLaunchKernelGGL((k_x3_nnk<E>), dim3(G, ncb), dim3(kX3KThreads), lds, ctx->stream, M, N, K, A, \
                       lda, bimg, C, ldc, ex);                                                     \
  } while (0)
    if (epi) NTS_X3K(true); else NTS_X3K(false);
#undef NTS_X3K
    NTS_LAUNCH_CHECK();
    return NTS_OK;
  }
  // one 8-wave block per CU over all column blocks (row blocks a multiple of 8:
  // XCD pairing), no more blocks than 16-tile rounds
  const int T = (M + 15) / 16;
  int gx = std::max(8, (256 / ncb) / 8 * 8);
  gx = std::min(gx, std::max(8, ((T + 15) / 16 + 7) / 8 * 8));
  const int64_t W = (int64_t)gx * 8;
  const int max_tiles = (int)((T + W - 1) / W);
  const int rounds = (max_tiles + 1) / 2;
  const dim3 grid(gx, ncb);
#define NTS_G3NN(E, MP)                                                                     \
  do {                                                                                          \
    NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm3_nn<E, MP>),         \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kS3NnLds));     \
    hipLaunchKernelGGL((k_gemm3_nn<E, MP>), grid, dim3(kS3NnThreads), kS3NnLds, ctx->stream, M, N, \
                       K, A, lda, bimg, C, ldc, rounds, ex);                                    \
  } while (0)
  if (epi) {
    if (amap) NTS_G3NN(true, true); else NTS_G3NN(true, false);
  } else {
    if (amap) NTS_G3NN(false, true); else NTS_G3NN(false, false);
  }
#undef NTS_G3NN
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

int gemm3_tn(nts_hip_ctx* ctx, int M, int N, int K, const float* A, uint64_t lda,
             const uint32_t* amap, const float* B, uint64_t ldb, const float* X, uint64_t ldx,
             float bscale, float* C, uint64_t ldc) {
  Gemm3Extra ex;
#ifdef NTS_PROBE_BUILD
  static const int diag = [] {
    const char* e = getenv("NTS_S3_DIAG");
    return e ? atoi(e) : 0;
  }();
  ex.diag = diag;
#endif
  ex.amap = amap;
  ex.bx = X;
  ex.ldbx = ldx;
  ex.bscale = bscale;
#ifndef NTS_NO_X3  // (variant builds: -DNTS_NO_X3 keeps k_s3_tn for A/B)
  if (amap && !X && x3_tn_ok(M, N, K, A, lda, B, ldb))
    return x3_tn(ctx, M, N, K, A, lda, amap, B, ldb, C, ldc);
#endif
  const bool v2_ok = ldb % 4 == 0 && (uintptr_t)B % 16 == 0 &&
                     (!X || (ldx % 4 == 0 && (uintptr_t)X % 16 == 0)) &&
                     (!amap || (uintptr_t)amap % 16 == 0);
  if (!use_v1() && v2_ok) {
    // v2: 8-wave blocks of up to 8 x TPW column tiles of A x 128 columns,
    // the reduction split so that one block lands on every CU
    constexpr int TPW = 3;
    const int T = (M + 15) / 16;
    const int nmb = (T + 8 * TPW - 1) / (8 * TPW), nnb = (N + 127) / 128;
    const int ksteps = (K + 31) / 32;
    int splits = std::max(1, std::min(256 / (nmb * nnb), ksteps / 4));
    const int kchunk = ((ksteps + splits - 1) / splits) * 32;
    splits = (K + kchunk - 1) / kchunk;
    const uint64_t stride = (uint64_t)M * N;
    float* out = C;
    uint64_t ldo = ldc;
    if (splits > 1) {
      NTS_RET(ensure_scratch(ctx, stride * splits * sizeof(float) + 256));
      out = (float*)ctx->scratch;
      ldo = N;
    }
    const dim3 grid(nmb * nnb * splits);
#define NTS_S3TN(BM, MP)                                                                          \
  do {                                                                                            \
    NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_s3_tn<TPW, BM, MP>),          \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kS3TnV2Lds));      \
    hipLaunchKernelGGL((k_s3_tn<TPW, BM, MP>), grid, dim3(kS3TnV2Threads), kS3TnV2Lds, ctx->stream, M, \
                       N, K, A, lda, B, ldb, out, ldo, kchunk, splits > 1 ? stride : (uint64_t)0,   \
                       nmb, nnb, ex);                                                             \
  } while (0)
    if (X) {
      if (amap) NTS_S3TN(true, true); else NTS_S3TN(true, false);
    } else {
      if (amap) NTS_S3TN(false, true); else NTS_S3TN(false, false);
    }
#undef NTS_S3TN
    NTS_LAUNCH_CHECK();
    if (splits == 1) return NTS_OK;
    return sum_splits(ctx->stream, out, splits, stride, M, N, C, ldc);
  }
  const int nrg = (M + kS3TnRows - 1) / kS3TnRows, ncb = (N + 127) / 128;
  int splits = std::max(1, std::min(256 / (nrg * ncb), (K + 4 * 32 - 1) / (4 * 32)));
  const int kchunk = ((K + splits - 1) / splits + 31) / 32 * 32;
  splits = (K + kchunk - 1) / kchunk;
  const dim3 grid(nrg * ncb * splits);
  const size_t lds = sizeof(S3TnSmem);
  const bool direct = splits == 1;
  const uint64_t stride = (uint64_t)M * N;
  float* out = C;
  uint64_t ldo = ldc;
  if (!direct) {
    NTS_RET(ensure_scratch(ctx, stride * splits * sizeof(float) + 256));
    out = (float*)ctx->scratch;
    ldo = N;
  }
#define NTS_G3TN(BM, MP)                                                                         \
  do {                                                                                           \
    NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm3_tn<BM, MP>),          \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));      \
    hipLaunchKernelGGL((k_gemm3_tn<BM, MP>), grid, dim3(kS3Threads), lds, ctx->stream, M, N, K, A, \
                       lda, B, ldb, out, ldo, kchunk, direct ? (uint64_t)0 : stride, nrg, ncb, ex); \
  } while (0)
  if (X) {
    if (amap) NTS_G3TN(true, true); else NTS_G3TN(true, false);
  } else {
    if (amap) NTS_G3TN(false, true); else NTS_G3TN(false, false);
  }
#undef NTS_G3TN
  NTS_LAUNCH_CHECK();
  if (direct) return NTS_OK;
  return sum_splits(ctx->stream, out, splits, stride, M, N, C, ldc);
}

}  // namespace nts_hip
