// fp32 GEMMs of the GCN layer update on the matrix cores (exact fp32 products,
// fp32 accumulate: v_mfma_f32_32x32x2_f32 / v_mfma_f32_16x16x4_f32).
//
// The layer GEMMs are tall-skinny: Z = Y W with Y [~150K x 602], W [602 x 128]
// (Parameter::forward, core/NtsScheduler.hpp:859-862) and the weight gradient
// dW = Y^T dZ (reduction over the ~150K sampled rows).  The library TN kernel
// runs these at ~36-45 TF/s; here:
//   NN, W slice fits LDS (K <= 608): k_gemm_wres — the weight's column slice
//       stays resident in LDS for the whole launch, A rows stream straight to
//       registers, no barrier in the main loop (see its comment).
//   TN with M >= 320, N % 128 == 0: k_gemm_tn_big — a 640 x 128 output tile
//       per block in accumulators, k-chunks split over blocks.
//   otherwise: k_gemm — block 64 rows x 128 cols, 4 waves of 32 x 64 on
//       v_mfma_f32_32x32x2_f32, A and B k-slices staged in LDS (double
//       buffered, register prefetch two steps deep).
//   Split reductions: partial tiles summed by k_sum_splits_tree in a fixed
//       tree order (deterministic, no atomics).
#include "common.hpp"

#include <type_traits>

namespace nts_hip {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kGT = 256;   // threads per block
constexpr int kBM = 64;    // block rows: 2 wave rows x 32
constexpr int kBN = 128;   // block cols: 2 wave cols x 2 MFMA tiles of 32
constexpr int kBK = 32;    // k per step (16 MFMA 32x32x2 k-pairs)
constexpr int kAP = 36;    // NN A tile pitch (floats): ds_read_b128 conflict-free

// Shared-memory image of one k-step (double buffered).
//   NN: As[m][k] (pitch kAP)      -> lane reads 16 consecutive k: 4 x ds_read_b128
//   TN: At[k][m]                  -> lane reads A[k][m] for 16 k:   16 x ds_read_b32
//   Bs[k][j][r][t] = B[k0+k][n0 + 64j + 32t + r]  (t = 0,1)  -> one ds_read_b64
//       gives a lane both column tiles of its wave column j, conflict-free.
struct GemmSmem {
  float a[2][kBM * kAP];
  float b[2][kBK * kBN];
};

// zero (mk == 0) or keep (mk == ~0) a value without a branch or a select on
// the loaded data's arrival
__device__ __forceinline__ float msk(float v, uint32_t mk) {
  return __uint_as_float(__float_as_uint(v) & mk);
}

// Per-thread tile movers.  Global -> registers for one k-step (8 A floats +
// 16 B floats per thread, every wave instruction reading whole 128-byte row
// segments), registers -> LDS at the end of the step.  Loads are branch-free
// with addresses clamped into the operands (k past K reads a valid element;
// its LDS image is zeroed by mask), so the compiler counts outstanding loads
// (vmcnt(N)) across steps instead of draining the queue: the two-deep
// prefetch relies on it.  Row/column bases are computed once per block.
// amap != nullptr: row r of the A operand is row amap[r] of the given matrix
// (NN: the M rows; TN: the K rows) — the transform-first bottom layer reads
// the feature table through the sampled layer's `source`.
template <bool TRANS_A, int AVEC>
struct ATile {
  static constexpr int NP = 8 / AVEC;  // loads per thread per step
  const float* base[TRANS_A ? 1 : NP];
  const uint32_t* amap;
  int kc;      // NN: this thread's k column in the step;  TN: its first k row
  int sdst;    // LDS offset of the first element
  __device__ ATile(const float* A, uint64_t lda, int M, int K, int64_t m0, const uint32_t* map)
      : amap(map) {
    const int tid = threadIdx.x;
    if (!TRANS_A) {  // A[m][k]: 64 rows x 32 k, rows tid/(32/AVEC) + (256/(32/AVEC)) p
      constexpr int per = 32 / AVEC;
      kc = (tid % per) * AVEC;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int64_t m = m0 + tid / per + (256 / per) * p;
        const uint64_t mm = (uint64_t)(m < M ? m : M - 1);
        base[p] = A + (amap ? (uint64_t)amap[mm] : mm) * lda;
      }
      sdst = (tid / per) * kAP + kc;
    } else {  // A[k][m]: 32 k x 64 m, k rows tid/(64/AVEC) + (256/(64/AVEC)) p
      constexpr int per = 64 / AVEC;
      const int64_t m = m0 + (tid % per) * AVEC;
      base[0] = A + (m < M ? m : M - AVEC);
      kc = tid / per;
      sdst = kc * kBM + (tid % per) * AVEC;
    }
    (void)K;
  }
  __device__ __forceinline__ void load(uint64_t lda, int K, int k0, float (&v)[8]) const {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const float* src;
      if (!TRANS_A) {
        const int k = min(k0 + kc, K - AVEC);
        src = base[p] + k;
      } else {
        const int k = min(k0 + kc + (256 / (64 / AVEC)) * p, K - 1);
        src = base[0] + (amap ? (uint64_t)amap[k] : (uint64_t)k) * lda;
      }
      if (AVEC == 4) {
        const float4 x = *reinterpret_cast<const float4*>(src);
        v[4 * p] = x.x; v[4 * p + 1] = x.y; v[4 * p + 2] = x.z; v[4 * p + 3] = x.w;
      } else if (AVEC == 2) {
        const float2 x = *reinterpret_cast<const float2*>(src);
        v[2 * p] = x.x; v[2 * p + 1] = x.y;
      } else {
        v[p] = *src;
      }
    }
  }
  __device__ __forceinline__ void store(float* __restrict__ sa, int K, int k0,
                                        const float (&v)[8]) const {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      float* dst;
      uint32_t mk;
      if (!TRANS_A) {
        dst = sa + sdst + (256 / (32 / AVEC)) * p * kAP;
        mk = k0 + kc < K ? ~0u : 0u;
      } else {
        dst = sa + sdst + (256 / (64 / AVEC)) * p * kBM;
        mk = k0 + kc + (256 / (64 / AVEC)) * p < K ? ~0u : 0u;
      }
      if (AVEC == 4)
        *reinterpret_cast<float4*>(dst) = make_float4(msk(v[4 * p], mk), msk(v[4 * p + 1], mk),
                                                      msk(v[4 * p + 2], mk), msk(v[4 * p + 3], mk));
      else if (AVEC == 2)
        *reinterpret_cast<float2*>(dst) = make_float2(msk(v[2 * p], mk), msk(v[2 * p + 1], mk));
      else
        *dst = msk(v[p], mk);
    }
  }
};

// B k-slice [32 x 128] into the permuted image Bs[k][j][r][t] (col 64j+32t+r).
// BFULL (N % 128 == 0, the usual hidden width): thread quad g = tid + 256i
// (k = g/32, j = (g%32)/16, m = g%16) loads the float2 pairs at columns
// 64j+2m and 64j+32+2m, which are exactly the 4 consecutive image slots
// (r = 2m, 2m+1; t = 0, 1): 8 float2 loads + 4 ds_write_b128 per step.
// Otherwise thread (kk = tid>>5, r = tid&31) moves k-rows kk + 8p, columns
// r + 32t (clamped): 16 loads + 8 ds_write_b64.
template <bool BFULL, bool BMASK>
struct BTile {
  static constexpr int NX = BMASK ? 16 : 1;
  const float* base;
  const float* xbase;  // BMASK: the forward output X (same shape as B)
  int coff[4];
  int kk, r;
  __device__ BTile(const float* B, const float* X, int N, int n0) {
    const int tid = threadIdx.x;
    if (BFULL) {
      kk = tid >> 5;  // k row of quad i: kk + 8i
      const int qq = tid & 31;
      r = (qq >> 4) * 64 + 2 * (qq & 15);  // c0 (relative to n0); image slot 4*qq
      base = B + n0 + r;
      xbase = BMASK ? X + n0 + r : nullptr;
    } else {
      kk = tid >> 5;
      r = tid & 31;
      base = B;
      xbase = X;
#pragma unroll
      for (int t = 0; t < 4; ++t) coff[t] = min(n0 + r + 32 * t, N - 1);
    }
  }
  __device__ __forceinline__ void load1(const float* b, uint64_t ld, int K, int k0,
                                        float* v) const {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const float* row = b + (uint64_t)min(k0 + kk + 8 * p, K - 1) * ld;
      if (BFULL) {
        const float2 x0 = *reinterpret_cast<const float2*>(row);
        const float2 x1 = *reinterpret_cast<const float2*>(row + 32);
        v[4 * p] = x0.x; v[4 * p + 1] = x1.x; v[4 * p + 2] = x0.y; v[4 * p + 3] = x1.y;
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) v[4 * p + t] = row[coff[t]];
      }
    }
  }
  __device__ __forceinline__ void load(uint64_t ldb, uint64_t ldx, int K, int k0, float (&v)[16],
                                       float (&vx)[NX]) const {
    load1(base, ldb, K, k0, v);
    if constexpr (BMASK) load1(xbase, ldx, K, k0, vx);
  }
  // B value as staged: k >= K -> 0; BMASK: G * scale where X > 0, else 0
  // (relu + dropout backward: X = dropout(relu(Z)) > 0 exactly where dZ != 0)
  __device__ __forceinline__ float val(const float (&v)[16], const float (&vx)[NX], int q,
                                       uint32_t mk, float bscale) const {
    if constexpr (BMASK) return vx[q] > 0.f ? msk(v[q], mk) * bscale : 0.f;
    return msk(v[q], mk);
  }
  __device__ __forceinline__ void store(float* __restrict__ sb, int K, int k0,
                                        const float (&v)[16], const float (&vx)[NX],
                                        float bscale) const {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const uint32_t mk = k0 + kk + 8 * p < K ? ~0u : 0u;
      float* row = sb + (kk + 8 * p) * kBN;
      if (BFULL) {
        *reinterpret_cast<float4*>(row + 4 * (threadIdx.x & 31)) =
            make_float4(val(v, vx, 4 * p, mk, bscale), val(v, vx, 4 * p + 1, mk, bscale),
                        val(v, vx, 4 * p + 2, mk, bscale), val(v, vx, 4 * p + 3, mk, bscale));
      } else {
        *reinterpret_cast<float2*>(row + 2 * r) =
            make_float2(val(v, vx, 4 * p, mk, bscale), val(v, vx, 4 * p + 1, mk, bscale));
        *reinterpret_cast<float2*>(row + 64 + 2 * r) =
            make_float2(val(v, vx, 4 * p + 2, mk, bscale), val(v, vx, 4 * p + 3, mk, bscale));
      }
    }
  }
};

// Fused extras of one launch.
//   EPI:   C = keep(row, col) ? relu(AB) * scale : 0 — ReLU + inverted dropout;
//          keep from Philox4x32-10 (key = seed, counter = {row>>2, col, offset})
//          word row&3 >= keep_threshold (p * 2^32): P(keep) = 1 - p.
//   BMASK: B = G * bscale where X > 0 (the backward of EPI, X its output).
struct GemmExtra {
  uint32_t keep_threshold = 0;
  float scale = 1.f;
  uint64_t seed = 0, offset = 0;
  const float* bx = nullptr;
  uint64_t ldbx = 0;
  float bscale = 1.f;
  const uint32_t* amap = nullptr;  // gathered A rows (see ATile)
};

// C_tile = op(A) B over k in [kbeg, kend); result written to C (ldc) or to a
// partial slab.  grid: x = M tiles, y = N tiles, z = k splits.
// Wave w: rows 32*(w&1) .. +32 of the block tile, columns 64*(w>>1) .. +64.
template <bool TRANS_A, int AVEC, bool BFULL, bool EPI, bool BMASK>
__global__ __launch_bounds__(kGT, 3) void k_gemm(int M, int N, int K, const float* __restrict__ A,
                                                 uint64_t lda, const float* __restrict__ B,
                                                 uint64_t ldb, float* __restrict__ C, uint64_t ldc,
                                                 int kchunk, uint64_t split_stride, GemmExtra ex) {
  __shared__ GemmSmem sm;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int wr = 32 * (w & 1), wc = w >> 1;
  const int64_t m0 = (int64_t)blockIdx.x * kBM;
  const int n0 = blockIdx.y * kBN;
  const int kbeg = blockIdx.z * kchunk;
  const int kend = min(K, kbeg + kchunk);
  f32x16 acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  const ATile<TRANS_A, AVEC> at(A, lda, M, kend, m0, ex.amap);
  const BTile<BFULL, BMASK> bt(B, ex.bx, N, n0);
  constexpr int NX = BTile<BFULL, BMASK>::NX;

  // Two register staging sets: the global loads of k-step j+2 are issued at
  // the start of step j (two steps of MFMA work cover the HBM latency), the
  // set holding step j+1 is written to the other LDS buffer at its end.
  float av0[8], bv0[16], av1[8], bv1[16], bx0[NX], bx1[NX];
  const int nsteps = kbeg < kend ? (kend - kbeg + kBK - 1) / kBK : 0;
  auto compute = [&](int cur) {
    float a[16];
    if (!TRANS_A) {
      const float4* ap = reinterpret_cast<const float4*>(sm.a[cur] + (wr + r) * kAP + 16 * h);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = ap[q];
        a[4 * q] = x.x; a[4 * q + 1] = x.y; a[4 * q + 2] = x.z; a[4 * q + 3] = x.w;
      }
    } else {
      const float* ap = sm.a[cur] + (16 * h) * kBM + wr + r;
#pragma unroll
      for (int s = 0; s < 16; ++s) a[s] = ap[s * kBM];
    }
    const float2* bp = reinterpret_cast<const float2*>(sm.b[cur] + (16 * h) * kBN + 64 * wc) + r;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const float2 b = bp[s * (kBN / 2)];
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b.x, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b.y, acc[1], 0, 0, 0);
    }
  };
  if (nsteps > 0) {
    at.load(lda, kend, kbeg, av0);
    bt.load(ldb, ex.ldbx, kend, kbeg, bv0, bx0);
    at.load(lda, kend, kbeg + kBK, av1);
    bt.load(ldb, ex.ldbx, kend, kbeg + kBK, bv1, bx1);
    at.store(sm.a[0], kend, kbeg, av0);
    bt.store(sm.b[0], kend, kbeg, bv0, bx0, ex.bscale);
  }
  __syncthreads();
  int j = 0;
  for (; j + 2 <= nsteps; j += 2) {
    const int k0 = kbeg + j * kBK;
    // step j: LDS buffer 0, loads of step j+2 -> set 0, set 1 (step j+1) -> buffer 1
    // (sched_barrier: keep the loads at the head of the step and the stores at
    // its tail — the scheduler would otherwise sink the loads below the MFMAs)
    at.load(lda, kend, k0 + 2 * kBK, av0);
    bt.load(ldb, ex.ldbx, kend, k0 + 2 * kBK, bv0, bx0);
    __builtin_amdgcn_sched_barrier(0);
    compute(0);
    __builtin_amdgcn_sched_barrier(0);
    at.store(sm.a[1], kend, k0 + kBK, av1);
    bt.store(sm.b[1], kend, k0 + kBK, bv1, bx1, ex.bscale);
    __syncthreads();
    // step j+1: LDS buffer 1, loads of step j+3 -> set 1, set 0 (step j+2) -> buffer 0
    at.load(lda, kend, k0 + 3 * kBK, av1);
    bt.load(ldb, ex.ldbx, kend, k0 + 3 * kBK, bv1, bx1);
    __builtin_amdgcn_sched_barrier(0);
    compute(1);
    __builtin_amdgcn_sched_barrier(0);
    at.store(sm.a[0], kend, k0 + 2 * kBK, av0);
    bt.store(sm.b[0], kend, k0 + 2 * kBK, bv0, bx0, ex.bscale);
    __syncthreads();
  }
  if (j < nsteps) compute(0);  // odd step count: the last step is already in buffer 0
  // epilogue: acc[t][i] -> (row = 8*(i>>2) + 4*h + (i&3), col = 32t + r) of the wave tile
  float* Cb = C + (uint64_t)blockIdx.z * split_stride;
  const int64_t wrow0 = m0 + wr;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int col = n0 + 64 * wc + 32 * t + r;
    if (col >= N) continue;
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // 4 consecutive rows: one Philox call
      const int64_t r4 = wrow0 + 8 * g + 4 * h;
      float o[4] = {acc[t][4 * g], acc[t][4 * g + 1], acc[t][4 * g + 2], acc[t][4 * g + 3]};
      if constexpr (EPI) {
        const uint4 rnd = dropout_words((uint64_t)r4, (uint32_t)col, ex.seed, ex.offset);
        const uint32_t wd[4] = {rnd.x, rnd.y, rnd.z, rnd.w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
          o[q] = (dropout_bits(wd[q], (uint32_t)col) >= ex.keep_threshold && o[q] > 0.f)
                     ? o[q] * ex.scale : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (r4 + q < M) Cb[(uint64_t)(r4 + q) * ldc + col] = o[q];
    }
  }
}

// ---------------------------------------------------------------------------
// NN with the weight slice resident in LDS (k_gemm_wres).
//
// The layer GEMM multiplies a tall activation [M x K] (M ~ 10^5) by a small
// weight [K x N].  A 1024-thread block (16 waves, one block per CU) copies
// the column slice W[:, n0 .. n0+NCOL) into LDS ONCE (K <= 624 at NCOL = 64,
// K <= 312 at NCOL = 128) and then streams row tiles of A with no barrier in
// the main loop:
//   * v_mfma_f32_16x16x4_f32; lane (i, g) = (lane & 15, lane >> 4);
//   * a wave task = 32 rows (2 row tiles) x NCOL columns (NCOL/16 col tiles);
//   * lane (i, g) loads A[row i][k0 + 8g .. k0 + 8g + 7] of a 32-deep k-block
//     straight to registers (128 contiguous bytes per row per k-block) —
//     the k order inside a k-block is a free permutation shared with B:
//     MFMA t of the block sums k = k0 + 8g + t over the four lane groups;
//   * B operands come from LDS (lgkmcnt), so the only vector-memory queue
//     entries are A's: the next k-block's rows are loaded a whole k-block
//     (64 MFMAs) ahead without any in-order vmcnt stall;
//   * LDS image sB[k][64q + 4i + jj] = W[k][n0 + (NCOL/16) i + 4q + jj]: one
//     ds_read_b128 per (k, q) per lane, conflict-free under gfx950's b128
//     lane grouping.
// Column blocks of the same row tile run on the same XCD (block b and the
// blocks b + 8·c), so the second read of an A tile is an L2/MALL hit.
// Numerics: every output is one k-ordered fp32 fma chain (exact products),
// fixed by the shapes — deterministic.
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kWresRT = 1;  // 16-row tiles per wave task
// 16 waves (4 per SIMD, <= 128 VGPRs) at NCOL = 64; 8 waves at NCOL = 128,
// whose 32 accumulator registers more per lane need the larger budget
template <int NCOL>
constexpr int wres_threads() { return NCOL == 128 ? 512 : 1024; }

// Raw loads of one 32-deep k-block of the wave's A rows (no masking: a select
// on the loaded value would make the compiler wait for the load right away).
template <int AVEC>
__device__ __forceinline__ void wres_load_a(const float* const (&arow)[kWresRT], int kb, int g,
                                            float (&a)[kWresRT][8]) {
  const int kbase = 32 * kb + 8 * g;
#pragma unroll
  for (int rt = 0; rt < kWresRT; ++rt) {
    const float* p = arow[rt] + kbase;
    if (AVEC == 4) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float4 x = reinterpret_cast<const float4*>(p)[q];
        a[rt][4 * q] = x.x; a[rt][4 * q + 1] = x.y; a[rt][4 * q + 2] = x.z; a[rt][4 * q + 3] = x.w;
      }
    } else if (AVEC == 2) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float2 x = reinterpret_cast<const float2*>(p)[q];
        a[rt][2 * q] = x.x; a[rt][2 * q + 1] = x.y;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) a[rt][q] = p[q];
    }
  }
}

// The last (partial) k-block, issued before the main loop: raw loads at
// clamped addresses (no select on the values here, see above) ...
__device__ __forceinline__ void wres_load_tail(const float* const (&arow)[kWresRT], int K, int kb,
                                               int g, float (&a)[kWresRT][8]) {
  const int kbase = 32 * kb + 8 * g;
#pragma unroll
  for (int rt = 0; rt < kWresRT; ++rt)
#pragma unroll
    for (int e = 0; e < 8; ++e) a[rt][e] = arow[rt][min(kbase + e, K - 1)];
}
// ... masked only when used (k >= K contributes 0 * padding)
__device__ __forceinline__ void wres_mask_tail(int K, int kb, int g, float (&a)[kWresRT][8]) {
  const int kbase = 32 * kb + 8 * g;
#pragma unroll
  for (int rt = 0; rt < kWresRT; ++rt)
#pragma unroll
    for (int e = 0; e < 8; ++e) a[rt][e] = msk(a[rt][e], kbase + e < K ? ~0u : 0u);
}

template <int NCOL>
__device__ __forceinline__ void wres_mfma(const float* __restrict__ bb, const float (&a)[kWresRT][8],
                                          f32x4 (&acc)[kWresRT][NCOL / 16]) {
  constexpr int CQ = NCOL / 64;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    f32x4 b[CQ];
#pragma unroll
    for (int q = 0; q < CQ; ++q) b[q] = *reinterpret_cast<const f32x4*>(bb + t * NCOL + 64 * q);
#pragma unroll
    for (int rt = 0; rt < kWresRT; ++rt)
#pragma unroll
      for (int q = 0; q < CQ; ++q)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          acc[rt][4 * q + jj] =
              __builtin_amdgcn_mfma_f32_16x16x4f32(a[rt][t], b[q][jj], acc[rt][4 * q + jj], 0, 0, 0);
  }
}

template <int NCOL, int AVEC, bool EPI, int DEPTH, bool XT>
__global__ __launch_bounds__(wres_threads<NCOL>()) void k_gemm_wres(
    int M, int N, int K, int nkb, const float* __restrict__ A, uint64_t lda,
    const float* __restrict__ B, uint64_t ldb, float* __restrict__ C, uint64_t ldc, int ncb,
    int vec_store, GemmExtra ex) {
  extern __shared__ __attribute__((aligned(16))) float sB[];
  constexpr int CT = NCOL / 16;  // 16-column tiles per wave task
  constexpr int CQ = CT / 4;     // ds_read_b128 per k
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int cb = (blockIdx.x >> 3) % ncb;
  const int bi = ((blockIdx.x >> 3) / ncb) * 8 + (blockIdx.x & 7);
  const int bpc = gridDim.x / ncb;
  const int n0 = cb * NCOL;
  const int Kp = nkb * 32;
  constexpr int WT = wres_threads<NCOL>();
  const int rows_per_task = 16 * kWresRT;
  const int ntask = (M + rows_per_task - 1) / rows_per_task;
  const int nwaves = bpc * (WT / 64);
  const int nfull = K / 32;
  auto rows_of = [&](int task, const float* (&ar)[kWresRT]) {
    const int64_t m0 = (int64_t)min(task, ntask - 1) * rows_per_task;
#pragma unroll
    for (int rt = 0; rt < kWresRT; ++rt) {
      const int64_t r = m0 + 16 * rt + i;
      const uint64_t rr = (uint64_t)(r < M ? r : M - 1);
      ar[rt] = A + (ex.amap ? (uint64_t)ex.amap[rr] : rr) * lda;
    }
  };
  // XT (cross-task prefetch, needs nfull % DEPTH == 0): the loads that would
  // re-read a task's last block fetch the next task's first blocks instead,
  // and the first task's are issued before the weight slice is staged
  const bool xt = XT && nfull >= DEPTH && nfull % DEPTH == 0;
  float a[DEPTH][kWresRT][8], at[kWresRT][8];
  int task = wv * bpc + bi;
  const float* arow[kWresRT];
  rows_of(task, arow);
  if (xt && task < ntask) {
#pragma unroll
    for (int d = 0; d + 1 < DEPTH; ++d) wres_load_a<AVEC>(arow, d, g, a[d]);
  }
  // fill in float4 pieces: local columns 4c4 .. 4c4+3 land on 4 consecutive
  // image slots (c = CT ii + j with j % 4 == 0 .. 3)
  if (ldb % 4 == 0 && ((uintptr_t)B & 15) == 0) {
#pragma unroll 4
    for (int e = tid; e < Kp * (NCOL / 4); e += WT) {
      const int k = e / (NCOL / 4), c = 4 * (e % (NCOL / 4));
      const int ii = c / CT, j = c % CT;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < K) v = *reinterpret_cast<const float4*>(B + (uint64_t)k * ldb + n0 + c);
      *reinterpret_cast<float4*>(sB + k * NCOL + 64 * (j >> 2) + 4 * ii) = v;
    }
  } else {
    for (int e = tid; e < Kp * NCOL; e += WT) {
      const int k = e / NCOL, c = e % NCOL;
      const int ii = c / CT, j = c % CT;
      const float v = k < K ? B[(uint64_t)k * ldb + n0 + c] : 0.f;
      sB[k * NCOL + 64 * (j >> 2) + 4 * ii + (j & 3)] = v;
    }
  }
  __syncthreads();
  (void)N;
  // the next task's row pointers are resolved a whole task ahead (with a row
  // map, a dependent load each) and handed over at the end of the task
  const float* nrow[kWresRT];
  rows_of(task + nwaves, nrow);
  for (; task < ntask; task += nwaves) {
    const int64_t m0 = (int64_t)task * rows_per_task;
    f32x4 acc[kWresRT][CT];
#pragma unroll
    for (int rt = 0; rt < kWresRT; ++rt)
#pragma unroll
      for (int j = 0; j < CT; ++j) acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // full k-blocks (32 (kb+1) <= K) are read unmasked into DEPTH rotating
    // register sets: the loads of blocks kb+1 .. kb+DEPTH-1 are in flight
    // during block kb's MFMAs; the partial last block is read masked.
    const float* bb = sB + 8 * g * NCOL + 4 * i;
    const bool tail = nfull < nkb;
    if (tail) wres_load_tail(arow, K, nfull, g, at);
    if (!xt && nfull > 0) {
#pragma unroll
      for (int d = 0; d + 1 < DEPTH; ++d) wres_load_a<AVEC>(arow, min(d, nfull - 1), g, a[d]);
    }
    int kb = 0;
    for (; kb + DEPTH <= nfull; kb += DEPTH) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        // unconditional (clamped / next task) so that every path through the
        // loop has the same queue of loads: the compiler then waits with a
        // count, not vmcnt(0)
        const int j = kb + d + DEPTH - 1;
        if (xt) {
          const bool own = j < nfull;
          const float* src[kWresRT];
#pragma unroll
          for (int rt = 0; rt < kWresRT; ++rt) src[rt] = own ? arow[rt] : nrow[rt];
          wres_load_a<AVEC>(src, own ? j : j - nfull, g, a[(d + DEPTH - 1) % DEPTH]);
        } else {
          wres_load_a<AVEC>(arow, min(j, nfull - 1), g, a[(d + DEPTH - 1) % DEPTH]);
        }
        __builtin_amdgcn_sched_barrier(0);
        wres_mfma<NCOL>(bb + 32 * (kb + d) * NCOL, a[d], acc);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // remaining full blocks: a[r] holds block kb + r
#pragma unroll
    for (int r = 0; r + 1 < DEPTH; ++r)
      if (kb + r < nfull) wres_mfma<NCOL>(bb + 32 * (kb + r) * NCOL, a[r], acc);
    if (tail) {
      wres_mask_tail(K, nfull, g, at);
      wres_mfma<NCOL>(bb + 32 * nfull * NCOL, at, acc);
    }
#pragma unroll
    for (int rt = 0; rt < kWresRT; ++rt) arow[rt] = nrow[rt];
    rows_of(task + 2 * nwaves, nrow);
    // epilogue: acc[rt][j][v] = C[m0 + 16 rt + 4 g + v][n0 + CT i + j]
#pragma unroll
    for (int rt = 0; rt < kWresRT; ++rt) {
      const int64_t r4 = m0 + 16 * rt + 4 * g;
      float o[4][CT];
#pragma unroll
      for (int j = 0; j < CT; ++j) {
#pragma unroll
        for (int v = 0; v < 4; ++v) o[v][j] = acc[rt][j][v];
      }
      if constexpr (EPI) {  // columns CT i + 2q, +1 share one generator call
#pragma unroll
        for (int q = 0; q < CT / 2; ++q) {
          const uint32_t col = (uint32_t)(n0 + CT * i + 2 * q);
          const uint4 rnd = dropout_words((uint64_t)r4, col, ex.seed, ex.offset);
          const uint32_t wd[4] = {rnd.x, rnd.y, rnd.z, rnd.w};
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              float& x = o[v][2 * q + h];
              x = (dropout_bits(wd[v], col + h) >= ex.keep_threshold && x > 0.f) ? x * ex.scale
                                                                                 : 0.f;
            }
        }
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        if (r4 + v >= M) continue;
        float* crow = C + (uint64_t)(r4 + v) * ldc + n0 + CT * i;
        if (vec_store) {
#pragma unroll
          for (int q = 0; q < CQ; ++q)
            *reinterpret_cast<float4*>(crow + 4 * q) =
                make_float4(o[v][4 * q], o[v][4 * q + 1], o[v][4 * q + 2], o[v][4 * q + 3]);
        } else {
#pragma unroll
          for (int j = 0; j < CT; ++j) crow[j] = o[v][j];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// TN with a block-sized output tile in accumulators (k_gemm_tn_big):
// C[M,N] = A[K,M]^T op(B)[K,N] — the weight gradient, M = layer input width
// (~602), N = 128, K = sampled rows (~10^5).  A 512-thread block owns a
// 640 x 128 output tile for one k-chunk: wave w keeps rows 80 w .. 80 w + 79
// x all 128 columns in 40 v_mfma_f32_16x16x4_f32 accumulators (rows
// interleaved over the lane index: row = 80 w + 5 i + rt, col = 8 i + j).
// Each 16-deep k-step is staged coalesced into LDS (A rows [16 x 640], the
// masked B rows [16 x 128]); per 4 k a lane reads 5 + 8 operand floats from
// LDS for 40 MFMAs (the old 64 x 128 tile read one LDS value per MFMA).
// Pitches make both reads conflict-free: LDY = 656 (rows of 4 lane groups
// land on disjoint b32 banks at stride 5), LDG = 132.  Partial tiles of the
// k-chunks are summed in a fixed order (k_sum_splits_tree).
// RT = 1 (a 128 x 128 tile, the narrow layers' weight gradient: 100 or 128
// output rows): LDY = 160 puts the two lane groups of a b32 read on disjoint
// bank halves.
constexpr int kTbWaves = 8;
constexpr int kTbKS = 16;                       // k rows per step
constexpr int kTbLDG = 132;
template <int RT>
constexpr int tb_rows() { return kTbWaves * 16 * RT; }  // 640 at RT = 5
template <int RT>
constexpr int tb_ldy() { return RT == 5 ? 656 : RT == 1 ? 160 : tb_rows<RT>() + 16; }

// NB = 3 (STAGGER): waves 4-7 run half a k-step behind waves 0-3 (they
// finish step st-1's second half after the barrier that ends step st-1), so
// the two waves sharing a SIMD are not in lockstep at the barrier and the LDS
// stores (MI355X_MICROARCH.md, workgroup rule 9).  A third LDS buffer keeps
// step st-1 readable while step st+1 is stored.  Every output element keeps
// the same k order: results are bit-identical to NB = 2.
template <int NB, int RT>
struct TbSmem {
  float y[NB][kTbKS * tb_ldy<RT>()];
  float g[NB][kTbKS * kTbLDG];
};

template <bool BMASK, int AVEC, bool STAGGER, int RT = 5>
__global__ __launch_bounds__(kTbWaves * 64, 1) void k_gemm_tn_big(
    int M, int N, int K, const float* __restrict__ A, uint64_t lda, const float* __restrict__ B,
    uint64_t ldb, float* __restrict__ C, uint64_t ldc, int kchunk, uint64_t split_stride,
    int nrg, int ncb, GemmExtra ex) {
  extern __shared__ __attribute__((aligned(16))) float smem_raw[];
  constexpr int NB = STAGGER ? 3 : 2;
  constexpr int kTbRT = RT, kTbRows = tb_rows<RT>(), kTbLDY = tb_ldy<RT>();
  TbSmem<NB, RT>& sm = *reinterpret_cast<TbSmem<NB, RT>*>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int rg = blockIdx.x % nrg;
  const int cb = (blockIdx.x / nrg) % ncb;
  const int split = blockIdx.x / (nrg * ncb);
  const int r0 = rg * kTbRows, n0 = cb * 128;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int nsteps = kbeg < kend ? (kend - kbeg + kTbKS - 1) / kTbKS : 0;
  // staging roles: A element pairs e = tid + 512 p -> (k row e / 320, cols 2 (e % 320) + {0,1});
  // B/X float4 q = tid -> (k row q / 32, cols 4 (q % 32) .. +3)
  constexpr int NAV = kTbRows / AVEC;                  // vectors per staged A row
  constexpr int NAL = kTbKS * NAV / (kTbWaves * 64);  // A loads per thread per step
  // one register staging set: the loads of step st+1 are issued before the
  // MFMAs of step st (which read LDS only) and written to the other LDS
  // buffer after them
  float av[NAL * AVEC];
  float4 bv, xv;
  const int bk = tid / 32, bc = 4 * (tid % 32);
  // A row of each staged element; with a row map these are dependent loads,
  // resolved one step ahead (the map of step st+2 is read with step st+1)
  uint32_t arow[NAL];
  auto map_rows = [&](int step) {
    const int kb = kbeg + step * kTbKS;
#pragma unroll
    for (int p = 0; p < NAL; ++p) {
      const int kk = min(kb + (tid + kTbWaves * 64 * p) / NAV, K - 1);
      arow[p] = ex.amap ? ex.amap[kk] : (uint32_t)kk;
    }
  };
  map_rows(0);
  auto load = [&](int step) {
    const int kb = kbeg + step * kTbKS;
#pragma unroll
    for (int p = 0; p < NAL; ++p) {
      const int e = tid + kTbWaves * 64 * p;
      // AVEC = 4 reads may run into the row padding (lda >= M rounded up to
      // 4); columns >= M are zeroed when staged
      const int c = min(r0 + AVEC * (e % NAV), AVEC == 4 ? (int)lda - 4 : M - AVEC);
      const float* src = A + (uint64_t)arow[p] * lda + c;
      if (AVEC == 4) {
        const float4 x = *reinterpret_cast<const float4*>(src);
        av[4 * p] = x.x; av[4 * p + 1] = x.y; av[4 * p + 2] = x.z; av[4 * p + 3] = x.w;
      } else if (AVEC == 2) {
        const float2 x = *reinterpret_cast<const float2*>(src);
        av[2 * p] = x.x; av[2 * p + 1] = x.y;
      } else {
        av[p] = *src;
      }
    }
    const int kk = min(kb + bk, K - 1);
    bv = *reinterpret_cast<const float4*>(B + (uint64_t)kk * ldb + n0 + bc);
    if constexpr (BMASK) xv = *reinterpret_cast<const float4*>(ex.bx + (uint64_t)kk * ex.ldbx + n0 + bc);
    map_rows(step + 1);
  };
  auto store = [&](int step, float* sy, float* sg) {
    const int kb = kbeg + step * kTbKS;
#pragma unroll
    for (int p = 0; p < NAL; ++p) {
      const int e = tid + kTbWaves * 64 * p;
      const int kr = e / NAV, c = AVEC * (e % NAV);
#pragma unroll
      for (int q = 0; q < AVEC; ++q) {
        const bool ok = (kb + kr < kend) && (r0 + c + q < M);
        sy[kr * kTbLDY + c + q] = ok ? av[AVEC * p + q] : 0.f;
      }
    }
    const bool okk = kb + bk < kend;
    float b4[4] = {bv.x, bv.y, bv.z, bv.w};
    if constexpr (BMASK) {
      const float x4[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) b4[q] = x4[q] > 0.f ? b4[q] * ex.bscale : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) b4[q] = okk ? b4[q] : 0.f;
    *reinterpret_cast<float4*>(sg + bk * kTbLDG + bc) = make_float4(b4[0], b4[1], b4[2], b4[3]);
  };
  f32x4 acc[kTbRT][8];
#pragma unroll
  for (int rt = 0; rt < kTbRT; ++rt)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // k sub-steps t0 .. t1-1 of one staged step (4 k each)
  auto compute = [&](const float* sy, const float* sg, int t0, int t1) {
    const float* ya = sy + g * kTbLDY + wv * 16 * kTbRT + kTbRT * i;
    const float* gb = sg + g * kTbLDG + 8 * i;
#pragma unroll
    for (int t = t0; t < t1; ++t) {
      float a[kTbRT];
#pragma unroll
      for (int rt = 0; rt < kTbRT; ++rt) a[rt] = ya[4 * t * kTbLDY + rt];
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(gb + 4 * t * kTbLDG);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(gb + 4 * t * kTbLDG + 4);
#pragma unroll
      for (int rt = 0; rt < kTbRT; ++rt) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rt], b0[j], acc[rt][j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[rt][4 + j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rt], b1[j], acc[rt][4 + j], 0, 0, 0);
      }
    }
  };
  constexpr int TH = kTbKS / 8;  // half a step
  const bool lag = STAGGER && wv >= kTbWaves / 2;
  if (nsteps > 0) {
    load(0);
    store(0, sm.y[0], sm.g[0]);
  }
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    const int cur = st % NB, nxt = (st + 1) % NB, prv = (st + NB - 1) % NB;
    load(st + 1);  // clamped rows past the chunk; masked (zero) when stored
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!STAGGER) {
      compute(sm.y[cur], sm.g[cur], 0, 2 * TH);
    } else {
      // two half steps through one (not unrolled) body: lead waves cur/0, cur/TH;
      // lagging waves prv/TH (none at st = 0), cur/0
#pragma unroll 1
      for (int ph = 0; ph < 2; ++ph) {
        if (lag && ph == 0 && st == 0) continue;
        const int b = (lag && ph == 0) ? prv : cur;
        const int t0 = lag ? (ph == 0 ? TH : 0) : ph * TH;
        compute(sm.y[b] + 4 * t0 * kTbLDY, sm.g[b] + 4 * t0 * kTbLDG, 0, TH);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (st + 1 < nsteps) store(st + 1, sm.y[nxt], sm.g[nxt]);
    __syncthreads();
  }
  if (lag && nsteps > 0) {
    const int last = (nsteps - 1) % NB;
    compute(sm.y[last], sm.g[last], TH, 2 * TH);
  }
  // acc[rt][j][v] = C[r0 + 80 wv + 5 (4 g + v) + rt][n0 + 8 i + j]
  float* Cb = C + (uint64_t)split * split_stride;
  const bool vec = (ldc % 4 == 0) && ((uintptr_t)Cb % 16 == 0);
#pragma unroll
  for (int v = 0; v < 4; ++v)
#pragma unroll
    for (int rt = 0; rt < kTbRT; ++rt) {
      const int row = r0 + wv * 16 * kTbRT + kTbRT * (4 * g + v) + rt;
      if (row >= M) continue;
      float* crow = Cb + (uint64_t)row * ldc + n0 + 8 * i;
      if (vec) {
        reinterpret_cast<float4*>(crow)[0] =
            make_float4(acc[rt][0][v], acc[rt][1][v], acc[rt][2][v], acc[rt][3][v]);
        reinterpret_cast<float4*>(crow)[1] =
            make_float4(acc[rt][4][v], acc[rt][5][v], acc[rt][6][v], acc[rt][7][v]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) crow[j] = acc[rt][j][v];
      }
    }
  (void)N;
}

// C = sum over `splits` partial slabs [M x N] (ld N), as a fixed-shape tree:
// thread s of a TPE-lane group sums splits s, s+TPE, ... in order (8 loads in
// flight, the tail batch predicated), then the group combines its TPE sums
// pairwise by shuffles (deterministic; every element with TPE-way parallel
// loads instead of one serial chain).  VEC = 4: float4 elements (N % 4 == 0,
// C 16-byte aligned rows), else floats.
template <int VEC, int TPE>
__global__ __launch_bounds__(256) void k_sum_splits_tree(const float* __restrict__ part,
                                                         int splits, uint64_t stride, int M,
                                                         int N, float* __restrict__ C,
                                                         uint64_t ldc) {
  using T = typename std::conditional<VEC == 4, float4, float>::type;
  constexpr int B = 8;
  const int s = threadIdx.x % TPE;
  const uint64_t e = (uint64_t)blockIdx.x * (256 / TPE) + threadIdx.x / TPE;
  const uint64_t total = (uint64_t)M * N / VEC;
  const T* p = reinterpret_cast<const T*>(part);
  const uint64_t st = stride / VEC;
  auto add = [](T& a, const T& b) {
    if constexpr (VEC == 4) {
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    } else {
      a += b;
    }
  };
  auto zero = []() {
    if constexpr (VEC == 4) return make_float4(0.f, 0.f, 0.f, 0.f); else return 0.f;
  };
  T acc = zero();
  if (e < total) {
    for (int z = s; z < splits; z += B * TPE) {
      T v[B];
#pragma unroll
      for (int u = 0; u < B; ++u)
        v[u] = z + TPE * u < splits ? p[(uint64_t)(z + TPE * u) * st + e] : zero();
#pragma unroll
      for (int u = 0; u < B; ++u)
        if (z + TPE * u < splits) add(acc, v[u]);
    }
  }
#pragma unroll
  for (int o = TPE / 2; o >= 1; o >>= 1) {
    if constexpr (VEC == 4) {
      acc.x += __shfl_down(acc.x, o, TPE);
      acc.y += __shfl_down(acc.y, o, TPE);
      acc.z += __shfl_down(acc.z, o, TPE);
      acc.w += __shfl_down(acc.w, o, TPE);
    } else {
      acc += __shfl_down(acc, o, TPE);
    }
  }
  if (s == 0 && e < total) {
    const uint64_t el = e * VEC;
    *reinterpret_cast<T*>(C + (el / N) * ldc + (el % N)) = acc;
  }
}

// Many splits (the row-split weight-gradient GEMMs: 256 slabs): wave w of a
// 16-wave block sums splits w, w + 16, ... of 64 consecutive float4 elements
// (one lane each: every load a coalesced 1 KB row piece of one slab, 8 in
// flight), then wave 0 adds the 16 wave sums in wave order through LDS.
// Deterministic (a fixed order per split count).
constexpr int kSsWaves = 16;
__global__ __launch_bounds__(kSsWaves * 64) void k_sum_splits_rows(const float4* __restrict__ part,
                                                                   int splits, uint64_t st4,
                                                                   uint64_t total, int N4,
                                                                   float* __restrict__ C,
                                                                   uint64_t ldc) {
  constexpr int B = 8;
  __shared__ float4 red[kSsWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t e = (uint64_t)blockIdx.x * 64 + lane;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < total) {
    for (int z = w; z < splits; z += B * kSsWaves) {
      float4 v[B];
#pragma unroll
      for (int u = 0; u < B; ++u)
        v[u] = z + kSsWaves * u < splits ? part[(uint64_t)(z + kSsWaves * u) * st4 + e]
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < B; ++u)
        if (z + kSsWaves * u < splits) {
          acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
        }
    }
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && e < total) {
    float4 r = red[0][lane];
#pragma unroll
    for (int k = 1; k < kSsWaves; ++k) {
      const float4 q = red[k][lane];
      r.x += q.x; r.y += q.y; r.z += q.z; r.w += q.w;
    }
    const uint64_t row = e / N4, col = (e % N4) * 4;
    *reinterpret_cast<float4*>(C + row * ldc + col) = r;
  }
}

// Sum `splits` partial slabs (stride floats apart, ld N) into C.
int sum_splits(hipStream_t st, const float* part, int splits, uint64_t stride, int M, int N,
               float* C, uint64_t ldc) {
  const bool v4 = N % 4 == 0 && ldc % 4 == 0 && (uintptr_t)C % 16 == 0;
  const bool wide = splits > 256;  // 64 lanes per element, else 16
  const uint64_t elems = stride / (v4 ? 4 : 1);
  if (v4 && splits >= 64 && stride % 4 == 0 && (uintptr_t)part % 16 == 0) {
    const uint64_t total = (uint64_t)M * N / 4;
    hipLaunchKernelGGL(k_sum_splits_rows, dim3(std::max(1u, ceil_div(total, 64))),
                       dim3(kSsWaves * 64), 0, st, reinterpret_cast<const float4*>(part), splits,
                       stride / 4, total, N / 4, C, ldc);
    NTS_LAUNCH_CHECK();
    return NTS_OK;
  }
  const uint32_t g = std::max(1u, ceil_div(elems, wide ? 4 : 16));
#define NTS_SS(V, T)                                                                         \
  hipLaunchKernelGGL((k_sum_splits_tree<V, T>), dim3(g), dim3(256), 0, st, part, splits, stride, \
                     M, N, C, ldc)
  if (v4) {
    if (wide) NTS_SS(4, 64); else NTS_SS(4, 16);
  } else {
    if (wide) NTS_SS(1, 64); else NTS_SS(1, 16);
  }
#undef NTS_SS
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

static bool tn_big_ok(int M, int N, const float* B, uint64_t ldb, const GemmExtra& ex, bool bmask) {
  // RT = 1 for <= 128 output rows (compile-time A/B: -DNTS_TN_NARROW=0)
#ifndef NTS_TN_NARROW
#define NTS_TN_NARROW 1
#endif
  constexpr bool narrow = NTS_TN_NARROW != 0;
  if (!(M >= 320 || (narrow && M <= 128)) || N % 128 != 0 || ldb % 4 != 0 || (uintptr_t)B % 16 != 0)
    return false;
  if (bmask && (ex.ldbx % 4 != 0 || (uintptr_t)ex.bx % 16 != 0)) return false;
  return true;
}

template <bool BMASK>
static int launch_tn_big(nts_hip_ctx* ctx, int M, int N, int K, const float* A, uint64_t lda,
                         const float* B, uint64_t ldb, float* C, uint64_t ldc,
                         const GemmExtra& ex) {
  hipStream_t st = ctx->stream;
  const bool rt1 = M <= 128;
  const int nrg = (M + (rt1 ? tb_rows<1>() : tb_rows<5>()) - 1) / (rt1 ? tb_rows<1>() : tb_rows<5>());
  const int ncb = N / 128;
  // narrow tiles hold ~55 KB of LDS and ~70 VGPRs: two blocks fit a CU, and
  // the second doubles the gathered rows in flight (A/B: -DNTS_TN_NARROW_BLOCKS=n)
#ifndef NTS_TN_NARROW_BLOCKS
#define NTS_TN_NARROW_BLOCKS 512
#endif
  constexpr int narrow_blocks = NTS_TN_NARROW_BLOCKS;
  const int target = rt1 ? narrow_blocks : 256;
  int splits = std::max(1, std::min(target / (nrg * ncb), (K + 4 * kTbKS - 1) / (4 * kTbKS)));
  const int kchunk = ((K + splits - 1) / splits + kTbKS - 1) / kTbKS * kTbKS;
  splits = (K + kchunk - 1) / kchunk;
  const dim3 grid(nrg * ncb * splits);
#ifndef NTS_TN_STAGGER  // compile-time A/B: -DNTS_TN_STAGGER=0
#define NTS_TN_STAGGER 1
#endif
  constexpr bool stagger = NTS_TN_STAGGER != 0;
  const size_t lds = rt1 ? (stagger ? sizeof(TbSmem<3, 1>) : sizeof(TbSmem<2, 1>))
                        : (stagger ? sizeof(TbSmem<3, 5>) : sizeof(TbSmem<2, 5>));
  const bool a4 = lda % 4 == 0 && lda >= (uint64_t)(M + 3) / 4 * 4 && (uintptr_t)A % 16 == 0;
  const bool a2 = M % 2 == 0 && lda % 2 == 0 && (uintptr_t)A % 8 == 0;
  const bool direct = splits == 1;
  const uint64_t stride = (uint64_t)M * N;
  float* out = C;
  uint64_t ldo = ldc;
  if (!direct) {
    NTS_RET(ensure_scratch(ctx, stride * splits * sizeof(float) + 256));
    out = (float*)ctx->scratch;
    ldo = N;
  }
#define NTS_TB_R(AV, SG, R)                                                                     \
  do {                                                                                          \
    NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_tn_big<BMASK, AV, SG, R>), \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));     \
    hipLaunchKernelGGL((k_gemm_tn_big<BMASK, AV, SG, R>), grid, dim3(kTbWaves * 64), lds, st, M, N, \
                       K, A, lda, B, ldb, out, ldo, kchunk, direct ? (uint64_t)0 : stride, nrg, \
                       ncb, ex);                                                                \
  } while (0)
#define NTS_TB_S(AV, SG)                  \
  do {                                    \
    if (rt1) NTS_TB_R(AV, SG, 1);         \
    else NTS_TB_R(AV, SG, 5);             \
  } while (0)
#define NTS_TB(AV)                               \
  do {                                           \
    if (stagger) NTS_TB_S(AV, true);             \
    else NTS_TB_S(AV, false);                    \
  } while (0)
  if (a4) NTS_TB(4); else if (a2) NTS_TB(2); else NTS_TB(1);
#undef NTS_TB
#undef NTS_TB_S
#undef NTS_TB_R
  NTS_LAUNCH_CHECK();
  if (direct) return NTS_OK;
  return sum_splits(st, out, splits, stride, M, N, C, ldc);
}

template <bool TRANS_A, bool EPI, bool BMASK>
static int launch(hipStream_t st, int M, int N, int K, const float* A, uint64_t lda,
                  const float* B, uint64_t ldb, float* C, uint64_t ldc, int splits, int kchunk,
                  uint64_t split_stride, const GemmExtra& ex) {
  dim3 grid(ceil_div(M, kBM), ceil_div(N, kBN), splits);
  // vector width of the A tile loads: rows of the loaded dimension must stay aligned
  const int inner = TRANS_A ? M : K;
  int avec = 1;
  if (inner % 4 == 0 && lda % 4 == 0 && (uintptr_t)A % 16 == 0) avec = 4;
  else if (inner % 2 == 0 && lda % 2 == 0 && (uintptr_t)A % 8 == 0) avec = 2;
  bool bfull = N % kBN == 0 && ldb % 2 == 0 && (uintptr_t)B % 8 == 0;
  if (BMASK) bfull = bfull && ex.ldbx % 2 == 0 && (uintptr_t)ex.bx % 8 == 0;
#define NTS_GEMM(AV, BF)                                                                      \
  hipLaunchKernelGGL((k_gemm<TRANS_A, AV, BF, EPI, BMASK>), grid, dim3(kGT), 0, st, M, N, K, \
                     A, lda, B, ldb, C, ldc, kchunk, split_stride, ex)
  if (avec == 4) { if (bfull) NTS_GEMM(4, true); else NTS_GEMM(4, false); }
  else if (avec == 2) { if (bfull) NTS_GEMM(2, true); else NTS_GEMM(2, false); }
  else { if (bfull) NTS_GEMM(1, true); else NTS_GEMM(1, false); }
#undef NTS_GEMM
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

// Column slice width of k_gemm_wres for this shape (0: not applicable).
static int wres_ncol(int M, int N, int K) {
  if (M < 2048 || K < 1) return 0;
  if (K <= 288 && N % 128 == 0) return 128;
  if (K <= 608 && N % 64 == 0) return 64;
  return 0;
}

template <bool EPI>
static int launch_wres(hipStream_t st, int ncol, int M, int N, int K, const float* A, uint64_t lda,
                       const float* B, uint64_t ldb, float* C, uint64_t ldc, const GemmExtra& ex) {
  const int nkb = (K + 31) / 32;
  const int ncb = N / ncol;
  const int per = std::max(1, 32 / ncb);  // blocks per (XCD, column block)
  const int grid = 8 * ncb * per;
  const size_t lds = (size_t)nkb * 32 * ncol * sizeof(float);
  // vector width of the A row loads of the full k-blocks (the partial last
  // block is read element-wise): only the row pitch and base alignment matter
  int avec = 1;
  if (lda % 4 == 0 && (uintptr_t)A % 16 == 0) avec = 4;
  else if (lda % 2 == 0 && (uintptr_t)A % 8 == 0) avec = 2;
  const int vs = (ldc % 4 == 0 && (uintptr_t)C % 16 == 0) ? 1 : 0;
#ifndef NTS_WRES_DEPTH  // compile-time A/B: -DNTS_WRES_DEPTH=3, -DNTS_WRES_XT=0
#define NTS_WRES_DEPTH 2
#endif
#ifndef NTS_WRES_XT
#define NTS_WRES_XT 1
#endif
  constexpr int depth = NTS_WRES_DEPTH;
  constexpr bool xtask = NTS_WRES_XT != 0;
#define NTS_WRES_D(NC, AV, D, X)                                                                \
  do {                                                                                          \
    NTS_HIP_TRY(hipFuncSetAttribute(                                                            \
        reinterpret_cast<const void*>(&k_gemm_wres<NC, AV, EPI, D, X>),                         \
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                                 \
    hipLaunchKernelGGL((k_gemm_wres<NC, AV, EPI, D, X>), dim3(grid), dim3(wres_threads<NC>()),  \
                       lds, st, M, N, K, nkb, A, lda, B, ldb, C, ldc, ncb, vs, ex);             \
  } while (0)
#define NTS_WRES(NC, AV)                                            \
  do {                                                              \
    if (depth == 3) {                                               \
      if (xtask) NTS_WRES_D(NC, AV, 3, true); else NTS_WRES_D(NC, AV, 3, false); \
    } else {                                                        \
      if (xtask) NTS_WRES_D(NC, AV, 2, true); else NTS_WRES_D(NC, AV, 2, false); \
    }                                                               \
  } while (0)
  if (ncol == 128) {
    if (avec == 4) NTS_WRES(128, 4); else if (avec == 2) NTS_WRES(128, 2); else NTS_WRES(128, 1);
  } else {
    if (avec == 4) NTS_WRES(64, 4); else if (avec == 2) NTS_WRES(64, 2); else NTS_WRES(64, 1);
  }
#undef NTS_WRES
#undef NTS_WRES_D
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

// Kernel selection (NTS_GEMM_TILED=1 forces the LDS-tiled kernel everywhere,
// for A/B comparisons).
static bool force_tiled() {  // compile-time A/B: -DNTS_GEMM_TILED=1
#ifdef NTS_GEMM_TILED
  return NTS_GEMM_TILED != 0;
#else
  return false;
#endif
}

// One GEMM: split the reduction when the output grid alone cannot fill the
// chip (partials summed in a fixed order by sum_splits: deterministic).  EPI
// needs the complete sum, so it never splits.
template <bool EPI, bool BMASK>
static int gemm(nts_hip_ctx* ctx, bool trans_a, int M, int N, int K, const float* A, uint64_t lda,
                const float* B, uint64_t ldb, float* C, uint64_t ldc, const GemmExtra& ex) {
  hipStream_t st = ctx->stream;
  if (K == 0) {  // empty reduction: C = 0 (and relu/dropout of 0 is 0)
    for (int i = 0; i < M; ++i) NTS_HIP_TRY(hipMemsetAsync(C + (uint64_t)i * ldc, 0, N * 4, st));
    return NTS_OK;
  }
  // The split kernels pay off on wide reductions / wide outputs (the C2
  // bottom layer, K = M = 602); narrow ones (products-shaped F = 100) run
  // faster on the fp32-input MFMA kernels (C3: 0.716 vs 0.740 ms/step).
  // Round 6: short dense reductions (K <= 128) on k_x3_nnk, which keeps the
  // whole W image in LDS.
#ifndef NTS_NO_X3K  // (A/B build: -DNTS_NO_X3K keeps these on the fp32-input kernels)
  const bool nnk = !trans_a && !BMASK && !ex.amap && x3_nnk_ok(M, N, K, A, lda);
#else
  const bool nnk = false;
#endif
#ifndef NTS_NO_X3K
  // ... and the masked weight gradient of such a layer (dW = Y^T (dZ ⊙ [Z >
  // 0]) s, M <= 128 output rows) on k_x3_tn's one-tile form with the mask rows
  // beside dZ's (the row pitch must cover 32 ceil(M / 32) floats)
  if (trans_a && BMASK && !EPI && ctx->gemm_mode != NTS_GEMM_F32 &&
      x3_tn_bm_ok(M, N, K, A, lda, B, ldb, ex.bx, ex.ldbx))
    return x3_tn(ctx, M, N, K, A, lda, ex.amap, B, ldb, C, ldc, ex.bx, ex.ldbx, ex.bscale);
#endif
  if (ctx->gemm_mode == NTS_GEMM_SPLIT3_ALL ||
      (ctx->gemm_mode == NTS_GEMM_SPLIT3 && ((trans_a ? M : K) >= 256 || nnk))) {
    if (!trans_a && !BMASK && gemm3_nn_ok(M, N, K, A, lda))
      return gemm3_nn(ctx, EPI, M, N, K, A, lda, ex.amap, B, ldb, C, ldc, ex.keep_threshold,
                      ex.scale, ex.seed, ex.offset);
    if (trans_a && !EPI && gemm3_tn_ok(M, N, K))
      return gemm3_tn(ctx, M, N, K, A, lda, ex.amap, B, ldb, BMASK ? ex.bx : nullptr, ex.ldbx,
                      ex.bscale, C, ldc);
  }
  if (!force_tiled()) {
    if (!trans_a && !BMASK) {
      const int ncol = wres_ncol(M, N, K);
      if (ncol) return launch_wres<EPI>(st, ncol, M, N, K, A, lda, B, ldb, C, ldc, ex);
    }
    if (trans_a && !EPI && tn_big_ok(M, N, B, ldb, ex, BMASK))
      return launch_tn_big<BMASK>(ctx, M, N, K, A, lda, B, ldb, C, ldc, ex);
  }
  const int tiles = (int)(ceil_div(M, kBM) * ceil_div(N, kBN));
  int splits = 1;
  const int ksteps = (K + kBK - 1) / kBK;
  // 3 blocks per CU are resident (LDS): aim the split grid at 768 blocks
  if (!EPI && tiles < 384) splits = std::max(1, std::min(768 / tiles, ksteps / 4));
  const int kchunk = ((ksteps + splits - 1) / splits) * kBK;
  splits = (K + kchunk - 1) / kchunk;
  if (splits == 1)
    return trans_a ? launch<true, EPI, BMASK>(st, M, N, K, A, lda, B, ldb, C, ldc, 1, kchunk, 0, ex)
                   : launch<false, EPI, BMASK>(st, M, N, K, A, lda, B, ldb, C, ldc, 1, kchunk, 0, ex);
  const uint64_t stride = (uint64_t)M * N;
  NTS_RET(ensure_scratch(ctx, stride * splits * sizeof(float) + 256));
  float* part = (float*)ctx->scratch;
  const int rc =
      trans_a ? launch<true, EPI, BMASK>(st, M, N, K, A, lda, B, ldb, part, N, splits, kchunk, stride, ex)
              : launch<false, EPI, BMASK>(st, M, N, K, A, lda, B, ldb, part, N, splits, kchunk, stride, ex);
  if (rc != NTS_OK) return rc;
  return sum_splits(st, part, splits, stride, M, N, C, ldc);
}

}  // namespace nts_hip

using namespace nts_hip;

#define NTS_GEMM_ARGS_CHECK(trans_a)                                            \
  NTS_CHECK_ARG(ctx && C, "NULL argument");                                     \
  NTS_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "negative size");                   \
  if (M == 0 || N == 0) return NTS_OK;                                          \
  NTS_CHECK_ARG((A && B) || K == 0, "NULL operand");                            \
  NTS_CHECK_ARG(ldb >= (uint64_t)N && ldc >= (uint64_t)N, "leading dimension"); \
  NTS_CHECK_ARG((trans_a) ? lda >= (uint64_t)M : lda >= (uint64_t)K, "lda");    \
  NTS_HIP_TRY(hipSetDevice(ctx->device))

extern "C" int nts_hip_gemm_f32(nts_hip_ctx* ctx, int trans_a, int M, int N, int K,
                                const float* A, uint64_t lda, const float* B, uint64_t ldb,
                                float* C, uint64_t ldc) {
  NTS_GEMM_ARGS_CHECK(trans_a);
  return trans_a ? gemm<false, false>(ctx, true, M, N, K, A, lda, B, ldb, C, ldc, GemmExtra())
                 : gemm<false, false>(ctx, false, M, N, K, A, lda, B, ldb, C, ldc, GemmExtra());
}

extern "C" int nts_hip_gemm_gather_f32(nts_hip_ctx* ctx, int M, int N, int K, const float* A,
                                       uint64_t lda, const uint32_t* a_rows, const float* B,
                                       uint64_t ldb, float* C, uint64_t ldc) {
  NTS_GEMM_ARGS_CHECK(false);
  NTS_CHECK_ARG(a_rows || K == 0, "NULL row map");
  GemmExtra ex;
  ex.amap = a_rows;
  return gemm<false, false>(ctx, false, M, N, K, A, lda, B, ldb, C, ldc, ex);
}

extern "C" int nts_hip_gemm_tn_gather_f32(nts_hip_ctx* ctx, int M, int N, int K, const float* A,
                                          uint64_t lda, const uint32_t* a_rows, const float* B,
                                          uint64_t ldb, float* C, uint64_t ldc) {
  NTS_GEMM_ARGS_CHECK(true);
  NTS_CHECK_ARG(a_rows || K == 0, "NULL row map");
  GemmExtra ex;
  ex.amap = a_rows;
  return gemm<false, false>(ctx, true, M, N, K, A, lda, B, ldb, C, ldc, ex);
}

extern "C" int nts_hip_gemm_relu_dropout_f32(nts_hip_ctx* ctx, int M, int N, int K, const float* A,
                                             uint64_t lda, const float* B, uint64_t ldb, float* C,
                                             uint64_t ldc, float p, uint64_t seed,
                                             uint64_t offset) {
  NTS_GEMM_ARGS_CHECK(false);
  NTS_CHECK_ARG(p >= 0.f && p <= 1.f, "dropout probability must be in [0, 1]");
  GemmExtra ex;
  ex.seed = seed;
  ex.offset = offset;
  ex.keep_threshold = dropout_threshold(p);
  ex.scale = p >= 1.f ? 0.f : 1.0f / (1.0f - p);  // p = 1: everything dropped (torch: zeros)
  return gemm<true, false>(ctx, false, M, N, K, A, lda, B, ldb, C, ldc, ex);
}

extern "C" int nts_hip_gemm_tn_masked_f32(nts_hip_ctx* ctx, int M, int N, int K, const float* A,
                                          uint64_t lda, const float* B, uint64_t ldb,
                                          const float* X, uint64_t ldx, float scale, float* C,
                                          uint64_t ldc) {
  NTS_GEMM_ARGS_CHECK(true);
  NTS_CHECK_ARG(X || K == 0, "NULL mask operand");
  NTS_CHECK_ARG(ldx >= (uint64_t)N, "ldx");
  GemmExtra ex;
  ex.bx = X;
  ex.ldbx = ldx;
  ex.bscale = scale;
  return gemm<false, true>(ctx, true, M, N, K, A, lda, B, ldb, C, ldc, ex);
}
