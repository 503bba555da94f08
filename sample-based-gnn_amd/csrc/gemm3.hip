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
//   k_gemm3_tn  C = A^T op(B) (weight gradient; relu/dropout backward fused in
//               the B load), A's k rows optionally gathered: a 320 x 128
//               output tile per block, k-slices of A and B staged transposed
//               into fragment order, the long reduction split over blocks and
//               summed in a fixed order (sum_splits) — deterministic.
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
  int diag = 0;  // NTS_S3_DIAG timing probes (results invalid): 1 no global loads,
                 // 2 no split, 4 no barrier, 8 no MFMA, 16 no B fragment reads
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
      if (s + 1 < nfull) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
// launchers (called by gemm.hip's dispatcher when the context's GEMM mode is
// NTS_GEMM_SPLIT3 and the shape qualifies)

// NN: the A rows are read by 16-byte global_load_lds (row pitch and base
// 16-byte aligned)
bool gemm3_nn_ok(int M, int N, int K, const float* A, uint64_t lda) {
  return M >= 256 && K >= 1 && N % 16 == 0 && lda % 4 == 0 && (uintptr_t)A % 16 == 0;
}
bool gemm3_tn_ok(int M, int N, int K) { return M >= 1 && K >= 256 && N % 16 == 0; }

int gemm3_nn(nts_hip_ctx* ctx, bool epi, int M, int N, int K, const float* A, uint64_t lda,
             const uint32_t* amap, const float* B, uint64_t ldb, float* C, uint64_t ldc,
             uint32_t keep_threshold, float scale, uint64_t seed, uint64_t offset) {
  Gemm3Extra ex;
  ex.keep_threshold = keep_threshold;
  ex.scale = scale;
  ex.seed = seed;
  ex.offset = offset;
  ex.amap = amap;
  static const int diag = [] {
    const char* e = getenv("NTS_S3_DIAG");
    return e ? atoi(e) : 0;
  }();
  ex.diag = diag;
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
  // one 8-wave block per CU over all column blocks (row blocks a multiple of 8:
  // XCD pairing), no more blocks than 16-tile rounds
  const int T = (M + 15) / 16;
  int gx = std::max(8, (256 / ncb) / 8 * 8);
  gx = std::min(gx, std::max(8, ((T + 15) / 16 + 7) / 8 * 8));
  const int64_t W = (int64_t)gx * 8;
  const int max_tiles = (int)((T + W - 1) / W);
  const int rounds = (max_tiles + 1) / 2;
  const dim3 grid(gx, ncb);
#define NTS_G3NN(E, MP)                                                                       \
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
  static const int diag = [] {
    const char* e = getenv("NTS_S3_DIAG");
    return e ? atoi(e) : 0;
  }();
  ex.diag = diag;
  ex.amap = amap;
  ex.bx = X;
  ex.ldbx = ldx;
  ex.bscale = bscale;
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
