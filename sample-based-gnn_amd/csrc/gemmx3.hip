// fp32-exact row-gathered GEMMs of the transform-first bottom layer on the
// bf16 matrix cores (the headline's arithmetic, NTS_GEMM_SPLIT3).
//
// The operands are the fp32 feature table itself (no pair table): every fp32
// value x is split exactly into three bf16 pieces inside the kernel,
//     x0 = bf16(x),  x1 = bf16(x - x0),  x2 = bf16(x - x0 - x1)   (RNE each)
// so x0 + x1 + x2 == x for every finite fp32 (24 significant bits, the
// exponent range of fp32), and a product a b is the six bf16 products
//     a0 b0 + a0 b1 + a1 b0 + a0 b2 + a1 b1 + a2 b0
// (dropped: a1 b2, a2 b1, a2 b2, each <= 2^-24 |a b|), exact in the fp32
// accumulator — the split of gemm3.hip, i.e. the reference's fp32
// `x.matmul(W)` (core/NtsScheduler.hpp:859-862) to fp32 accuracy.
//
// What these kernels change against gemm3.hip's k_gemm3_nn / k_s3_tn is the
// access pattern: WHOLE gathered feature rows (2,432 B of 602 floats) are
// streamed into LDS by global_load_lds, row-aligned 1-KiB pieces, three
// stages (two steps in flight), the row ids staged in LDS — the pattern that
// measured 5.9 TB/s for the pair tables (scripts/probe/stream_probe.hip) —
// instead of 128-byte slices of 16 rows per k-step (k_gemm3_nn) or dword
// column gathers (k_s3_tn).
//
//   k_x3_tn  dW = X[amap]^T dH: one block per chunk of the gathered rows
//            covers EVERY output row (the structure of gemmh2.hip's k_h2_tn4):
//            per 16-row step, each wave reads its X^T fragments with
//            ds_read_b32 (32 consecutive columns per half-wave: conflict-free)
//            and its dH fragments likewise, splits them in registers, and runs
//            v_mfma_f32_32x32x16_bf16 x 6 per 32x32 tile; the chunks'
//            partials are summed in a fixed order (sum_splits): deterministic.
#include "common.hpp"
#include <type_traits>

namespace nts_hip {

typedef __bf16 x3bf8 __attribute__((ext_vector_type(8)));
typedef float x3f16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void* x3_lds_ptr;

__device__ __forceinline__ uint32_t x3_lds(const void* p) { return (uint32_t)(uintptr_t)(x3_lds_ptr)p; }
// 16 bytes per lane from `src` to LDS (wave-uniform base `lds`) + 16 * lane;
// inline asm: a compiler-visible LDS DMA makes hipcc drain every stage (see
// gemm3.hip), so completion is counted by hand with s_waitcnt vmcnt
__device__ __forceinline__ void x3_glds16(const void* src, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}
__device__ __forceinline__ void x3_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// x -> (x0, x1, x2), element-wise over one lane's 8 fragment values
__device__ __forceinline__ void x3_split(const float (&x)[8], x3bf8 (&h)[3]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 a0 = (__bf16)x[j];
    const float r1 = x[j] - (float)a0;
    const __bf16 a1 = (__bf16)r1;
    h[0][j] = a0;
    h[1][j] = a1;
    h[2][j] = (__bf16)(r1 - (float)a1);
  }
}

// acc += a b over one 16-deep k-slice of a 32x32 tile (small products first)
__device__ __forceinline__ x3f16 x3_mfma6(const x3bf8 (&a)[3], const x3bf8 (&b)[3], x3f16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}

// ---------------------------------------------------------------------------
// TN: C[M x N] = X[amap[k]][0..M)^T B[k][0..N) over the gathered rows k of
// [kbeg, kend) (one chunk per block; N in 128-column blocks).  M <= 608: an
// X row of Kp = 32 ceil(M / 32) floats is RB = 4 Kp bytes, PR = ceil(RB /
// 1024) row-aligned DMA pieces per row.
// LDS: X stages [3][16][RB]; raw dH stages [2][16][128 floats]; dH's three
// bf16 planes [2 buffers][3][16][128] (256-byte rows, 16-byte chunks
// XOR-swizzled for ds_read_b64_tr_b16, the layout of gemmh2.hip's TN); row ids.
// Wave wv: wn = wv & 1 takes columns 64 wn .. +63 (two 32-column tiles), wm =
// wv >> 1 a quarter of the 32-row output tiles (at most TPW).
// Per 16-row step s, after the wait (this wave's X(s) and dH(s+1) pieces; the
// 2 PR pieces of X(s+1) may stay in flight) and the barrier:
//   issue dH(s+2) into the raw stage dH(s) left, X(s+2) into the stage X(s-1)
//     left (row ids read one step ahead);
//   split dH(s+1) (rows past the chunk zeroed) into the other plane buffer,
//     one float4 per thread (visible to every wave after the next barrier);
//   B fragments of step s from the planes written during step s-1 (tr reads);
//   A fragments of tile t: lane (c, h) reads X[16 s + 8 h + j][32 (m_lo + t) +
//     c], j = 0..7 (ds_read_b32, 32 consecutive dwords per half-wave) for tile
//     t+1 while tile t's 12 MFMAs run, and splits them (rows past the chunk
//     are duplicates of its last row, multiplied by zeroed dH rows; the
//     table's pad columns only reach output rows >= M, never stored).
constexpr int kX3Threads = 512;
constexpr int kX3BRaw = 16 * 512;   // one step of fp32 dH rows (128 columns)
constexpr int kX3BPl = 16 * 256;    // one bf16 plane of a step

__device__ __forceinline__ int x3_tr_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

typedef short x3s4 __attribute__((ext_vector_type(4)));
typedef short x3s8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) x3s4 x3_lds_s4;

// exact split of two fp32 values into three packed bf16 pairs (RNE each; the
// per-pair form of x3_split, so the pieces can be scheduled pair by pair)
typedef __bf16 x3bf2 __attribute__((ext_vector_type(2)));
typedef float x3f2 __attribute__((ext_vector_type(2)));
typedef uint32_t x3u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void x3_split2(float x0, float x1, uint32_t& p0, uint32_t& p1, uint32_t& p2) {
  const x3bf2 h = __builtin_convertvector((x3f2){x0, x1}, x3bf2);
  const x3f2 hf = __builtin_convertvector(h, x3f2);
  const float r0 = x0 - hf[0], r1 = x1 - hf[1];
  const x3bf2 m = __builtin_convertvector((x3f2){r0, r1}, x3bf2);
  const x3f2 mf = __builtin_convertvector(m, x3f2);
  const x3bf2 l = __builtin_convertvector((x3f2){r0 - mf[0], r1 - mf[1]}, x3bf2);
  p0 = __builtin_bit_cast(uint32_t, h);
  p1 = __builtin_bit_cast(uint32_t, m);
  p2 = __builtin_bit_cast(uint32_t, l);
}

// DIAG (timing probes, NTS_X3_DIAG in the probe build only; results are
// garbage): 1 no MFMAs, 2 no A splits, 4 no DMA after the prologue, 8 no A
// fragment reads, 16 no wait for the DMA, 32 no slab stores
//
// Instruction schedule of a step (one wave): the head (the wait, the
// barrier, dH(s+2)'s DMA, the B fragments, tile 0's A fragment split) and
// then, per 32-row tile t, TWELVE slots, each one MFMA of tile t (the two
// n-tiles' chains alternate) followed by a fixed share of the other work:
// tile t+2's eight A reads, one of tile t+1's four split pairs, and —
// spread over tiles 0..2 — X(s+2)'s six DMA pieces, the block's split of
// dH(s+1) into the planes, and the row ids of step s+3.  sched_barrier(0)
// between slots keeps that order: the wave issues its VALU and LDS work in
// the shadow of its own MFMAs (in-order issue would otherwise run a tile's
// twelve MFMAs, then its VALU, then its reads, none overlapping).
// BM (round 6, dense rows): B = dH ⊙ [Xm > 0] · bscale — the relu/dropout
// backward of an aggregate-first bottom layer (C3 / C4, M = 100) fused: the
// Xm rows of each step ride beside dH's (one more DMA per wave, issued before
// the X pieces, so the counted waits are unchanged) and mask it at the split.
template <int TPW, int PR, int DIAG = 0, bool BM = false>
__global__ __launch_bounds__(kX3Threads, 1) void k_x3_tn(int M, int K, const float* __restrict__ X,
                                                        uint64_t ldx, const uint32_t* __restrict__ amap,
                                                        const float* __restrict__ B, uint64_t ldb,
                                                        float* __restrict__ C, uint64_t ldc, int kchunk,
                                                        uint64_t split_stride, int nnb,
                                                        const float* __restrict__ Xm, uint64_t ldxm,
                                                        float bscale) {
  static_assert(2 * PR <= 6, "X DMA pieces per wave and step");
  extern __shared__ __attribute__((aligned(16))) char x3tn[];
  const int Kp = (M + 31) / 32 * 32, RB = 4 * Kp, RW = Kp;  // LDS row: bytes, floats
  const int xstage = 16 * RB;
  char* const sx = x3tn;                         // [3][16][RB]
  char* const sbr = sx + 3 * xstage;             // [2][kX3BRaw]
  char* const sbp = sbr + 2 * kX3BRaw;           // [2][3][kX3BPl]
  char* const sbm = sbp + 6 * kX3BPl;            // BM: [2][kX3BRaw] raw Xm rows
  uint32_t* const sid = reinterpret_cast<uint32_t*>(sbm + (BM ? 2 * kX3BRaw : 0));  // [16 (nsteps + 3)]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nb = blockIdx.x % nnb, split = blockIdx.x / nnb;
  const int n0 = nb * 128;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk), klast = kend - kbeg - 1;
  if (klast < 0) return;  // (block-uniform)
  const int nsteps = (kend - kbeg + 15) / 16;
  // ids past the chunk: its last row again (every step's DMA, real or not,
  // reads valid rows, so the per-wave piece counts stay uniform)
  for (int k = tid; k < 16 * (nsteps + 3); k += kX3Threads)
    sid[k] = amap ? amap[kbeg + min(k, klast)] : (uint32_t)(kbeg + min(k, klast));
  __syncthreads();
  const uint32_t lsx = x3_lds(sx), lsbr = x3_lds(sbr), lsbm = x3_lds(sbm);
#ifdef NTS_X3_PRIO
  if (wv >= 4) __builtin_amdgcn_s_setprio(1);  // A/B: static priority for the younger half
#endif
  // this wave's DMA rows of a step: 2 wv, 2 wv + 1
  auto ids_read = [&](int s) { return *reinterpret_cast<const uint2*>(sid + 16 * s + 2 * wv); };
  auto ids_uni = [&](uint2 u) {
    return make_uint2(__builtin_amdgcn_readfirstlane(u.x), __builtin_amdgcn_readfirstlane(u.y));
  };
  auto issue_x1 = [&](int s, uint2 id, int q) {  // piece q of this wave's X(s) pieces
    if ((DIAG & 4) && s >= 2) return;
    const int row = 2 * wv + q / PR, part = q % PR;
    const int off = 1024 * part + 16 * lane;
    const char* src = reinterpret_cast<const char*>(X + (uint64_t)(q < PR ? id.x : id.y) * ldx) + off;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(lsx + (s % 3) * xstage + row * RB + 1024 * part);
    if (off < RB) x3_glds16(src, dst);  // lane 0 always issues: the wave's count is exact
  };
  auto issue_b = [&](int s) {
    if ((DIAG & 4) && s >= 2) return;
    const int row = 2 * wv + (lane >> 5);
    const int k = kbeg + min(16 * s + row, klast);
    x3_glds16(B + (uint64_t)k * ldb + n0 + 4 * (lane & 31), lsbr + (s & 1) * kX3BRaw + 1024 * wv);
    if constexpr (BM)
      x3_glds16(Xm + (uint64_t)k * ldxm + n0 + 4 * (lane & 31), lsbm + (s & 1) * kX3BRaw + 1024 * wv);
  };
  // dH(s) raw -> three bf16 planes (buffer s & 1): row sr, columns sc .. sc+3
  const int sr = tid >> 5, sc = 4 * (tid & 31);
  const int soff = x3_tr_off(sr, sc / 8) + 8 * ((sc / 4) & 1);
  auto splitb_read = [&](int s) {
    float4 v = *reinterpret_cast<const float4*>(sbr + (s & 1) * kX3BRaw + 512 * sr + 4 * sc);
    if constexpr (BM) {
      const float4 m = *reinterpret_cast<const float4*>(sbm + (s & 1) * kX3BRaw + 512 * sr + 4 * sc);
      v.x = m.x > 0.f ? v.x * bscale : 0.f;
      v.y = m.y > 0.f ? v.y * bscale : 0.f;
      v.z = m.z > 0.f ? v.z * bscale : 0.f;
      v.w = m.w > 0.f ? v.w * bscale : 0.f;
    }
    return v;
  };
  auto splitb_write = [&](int s, float4 v) {
    const bool ok = 16 * s + sr <= klast;
    uint32_t q0[2], q1[2], q2[2];
    x3_split2(ok ? v.x : 0.f, ok ? v.y : 0.f, q0[0], q1[0], q2[0]);
    x3_split2(ok ? v.z : 0.f, ok ? v.w : 0.f, q0[1], q1[1], q2[1]);
    char* dst = sbp + (s & 1) * 3 * kX3BPl + soff;
    *reinterpret_cast<uint2*>(dst) = make_uint2(q0[0], q0[1]);
    *reinterpret_cast<uint2*>(dst + kX3BPl) = make_uint2(q1[0], q1[1]);
    *reinterpret_cast<uint2*>(dst + 2 * kX3BPl) = make_uint2(q2[0], q2[1]);
  };
  const int wn = wv & 1, wm = wv >> 1;
  const int T32 = (M + 31) / 32;
  const int m_lo = wm * T32 / 4, nmt = (wm + 1) * T32 / 4 - m_lo;
  const int c = lane & 31, h = lane >> 5;
  // 32x32x16 B fragments from the planes: lane (c, h) holds rows 8h .. 8h+7 of
  // column c, read as two transposed 4-row halves by its 16-lane group
  const int half = (lane >> 4) & 1, tq = (lane & 15) >> 2, tp = lane & 3;
  int boff[2][2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int ch = (2 * (64 * wn + 32 * nt + 16 * half + 4 * tp)) / 16;
    boff[nt][0] = x3_tr_off(8 * h + tq, ch) + 8 * (tp & 1);
    boff[nt][1] = x3_tr_off(8 * h + tq + 4, ch) + 8 * (tp & 1);
  }
  // the A^T fragment column of each tile slot (tiles past nmt repeat the
  // wave's last one: computed, never stored)
  int xcol[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) xcol[t] = 32 * max(0, min(m_lo + min(t, nmt - 1), T32 - 1)) + 8 * h * RW + c;
  x3f16 acc[TPW][2];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[t][nt][v] = 0.f;
  // prologue: dH(0) split into planes 0; then dH(1), X(0), X(1) in flight
  issue_b(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  x3_barrier();
  splitb_write(0, splitb_read(0));
  issue_b(1);
  {
    const uint2 i0 = ids_uni(ids_read(0)), i1 = ids_uni(ids_read(1));
#pragma unroll
    for (int q = 0; q < 2 * PR; ++q) issue_x1(0, i0, q);
#pragma unroll
    for (int q = 0; q < 2 * PR; ++q) issue_x1(1, i1, q);
  }
  uint2 idn = ids_uni(ids_read(2));
  for (int s = 0; s < nsteps; ++s) {
    // every DMA of this wave drained (vmcnt(0)), not just the ones this step
    // reads (vmcnt(2 PR), which leaves X(s+1)'s pieces in flight): with the
    // counted wait the one-tile form (its dH split 5 slots after the wait)
    // read a stale step about one run in four — 6 of 23 vs 0 of 23 drained
    // (scripts/dbg_tn.py) — so the count is not safe to rely on; C2 pays
    // nothing for the drain (0.828-0.831 vs 0.829-0.832 ms/step, r06_y.sh)
#ifdef NTS_X3TN_COUNTED  // (A/B build: the counted wait)
    if constexpr (DIAG & 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (!(DIAG & 16)) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PR) : "memory");
#else
    if constexpr (!(DIAG & 16)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    x3_barrier();
    issue_b(s + 2);
    const char* pl = sbp + (s & 1) * 3 * kX3BPl;
    x3bf8 bq[2][3];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const x3s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((x3_lds_s4*)(pl + p * kX3BPl + boff[nt][0]));
        const x3s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((x3_lds_s4*)(pl + p * kX3BPl + boff[nt][1]));
        const x3s8 w = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bq[nt][p] = __builtin_bit_cast(x3bf8, w);
      }
    const float* xs = reinterpret_cast<const float*>(sx + (s % 3) * xstage);
    float xr[2][8];      // raw A^T fragments, tile t in slot t & 1
    uint32_t ap[2][3][4];  // split pieces, tile t in slot t & 1: [piece][pair]
    auto rd = [&](int t, int j) {
      if constexpr (DIAG & 8) return (float)(t + j) * (float)lane;
      else return xs[xcol[t] + j * RW];
    };
    auto sp = [&](int t, int jp) {  // pair jp of tile t's split
      if constexpr (DIAG & 2) {
        ap[t & 1][0][jp] = ap[t & 1][1][jp] = ap[t & 1][2][jp] = __float_as_uint(xr[t & 1][2 * jp]);
      } else {
        x3_split2(xr[t & 1][2 * jp], xr[t & 1][2 * jp + 1], ap[t & 1][0][jp], ap[t & 1][1][jp],
                  ap[t & 1][2][jp]);
      }
    };
#pragma unroll
    for (int j = 0; j < 8; ++j) xr[0][j] = rd(0, j);
    if constexpr (TPW > 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) xr[1][j] = rd(1, j);
    }
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) sp(0, jp);
    const uint2 idx = idn;  // X(s+2)'s rows
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    uint2 idr = make_uint2(0u, 0u);
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      x3bf8 a[3];
#pragma unroll
      for (int p = 0; p < 3; ++p)
        a[p] = __builtin_bit_cast(x3bf8, (x3u4){ap[t & 1][p][0], ap[t & 1][p][1], ap[t & 1][p][2], ap[t & 1][p][3]});
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        __builtin_amdgcn_sched_barrier(0);
        {  // slot k: product k / 2 (small first) of n-tile k & 1
          const int nt = k & 1, pr = k >> 1;
          const int pa = pr == 0 ? 2 : pr == 1 ? 1 : pr == 2 ? 0 : pr == 3 ? 1 : 0;
          const int pb = pr == 0 ? 0 : pr == 1 ? 1 : pr == 2 ? 2 : pr == 3 ? 0 : pr == 4 ? 1 : 0;
          if constexpr (DIAG & 1) acc[t][nt][0] += (float)a[pa][0] + (float)bq[nt][pb][3];
          else acc[t][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[pa], bq[nt][pb], acc[t][nt], 0, 0, 0);
        }
        if (t + 2 < TPW && k < 8) xr[t & 1][k] = rd(t + 2, k);
        if (t + 1 < TPW && (k == 3 || k == 5 || k == 7 || k == 9)) sp(t + 1, (k - 3) / 2);
        if (t == 0 && (k & 1) && k / 2 < 2 * PR) issue_x1(s + 2, idx, k / 2);
        // (fewer than three tiles: these slots move into tile 0 / 1)
        constexpr int tB = TPW >= 2 ? 1 : 0, kBr = TPW >= 2 ? 1 : 5, kBw = TPW >= 2 ? 8 : 9;
        constexpr int tI = TPW >= 3 ? 2 : 0, kIr = TPW >= 3 ? 1 : 6, kIw = TPW >= 3 ? 10 : 11;
        if (t == tB && k == kBr) bv = splitb_read(s + 1);
        if (t == tB && k == kBw) splitb_write(s + 1, bv);  // (past the last step: never read)
        if (t == tI && k == kIr) idr = ids_read(s + 3);
        if (t == tI && k == kIw) idn = ids_uni(idr);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS DMA outlives the block
  x3_barrier();
  // acc[t][nt][v] = C[32 (m_lo + t) + 8 (v / 4) + 4 h + v % 4][n0 + 64 wn + 32 nt + c]
  float* Cb = C + (uint64_t)split * split_stride;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int col = n0 + 64 * wn + 32 * nt + c;
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      if (t >= nmt) continue;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = 32 * (m_lo + t) + 8 * (v / 4) + 4 * h + (v % 4);
        if (row < M && (!(DIAG & 32) || acc[t][nt][v] == 1234.5f)) Cb[(uint64_t)row * ldc + col] = acc[t][nt][v];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// NN: C[M x N] = X[amap[m]][0..K) W (+ relu/dropout): the work split and LDS
// plan of gemm3.hip's k_gemm3_nn — 8-wave blocks, one 128-column block per
// grid.y, 16-row tiles, wave gw of the grid owning the contiguous tiles [gw T
// / W, (gw+1) T / W) two at a time in `rounds` rounds; per 32-deep k-step
// the W fragment image (k_split3_b, 24 KB: 2 stages) and each wave's 2 x (16
// rows x 32 floats) A slab (3 stages) by LDS DMA, counted vmcnt, one raw
// barrier — with every k-step read as a whole (the rows' pad past K is
// zeroed at the split, so the table's row pitch must cover Kp) and the MFMA
// loop scheduled slot by slot: per column tile 12 MFMAs (the two row tiles'
// chains alternating), the next column tile's three B fragment reads in the
// shadow of the first three.  The A slab is wave-private, so the next step's
// fragments are read and split during the current step (a mid-step wait for
// its 4 pieces at column tile 4, split pairs in tiles 5-6, two register sets
// by step parity): 267 vs 273 us at C2 on one box (scripts/r05_q.sh).  Each output element's sum is k_gemm3_nn's
// (same split, same piece order, same k order, same instruction): the
// results are bit-identical.
constexpr int kX3NnImg = 8 * 3 * 1024;       // one (step, column block) W image
constexpr int kX3NnAWave = 2 * 2048;         // one wave's A slab of a step
constexpr int kX3NnA = 8 * kX3NnAWave;       // one A stage
constexpr int kX3NnLds = 2 * kX3NnImg + 3 * kX3NnA;  // 48 + 96 KB
struct X3Epi {
  uint32_t keep_threshold = 0;  // EPI: relu + inverted dropout (common.hpp dropout_*)
  float scale = 1.f;
  uint64_t seed = 0, offset = 0;
};

typedef float x3f4 __attribute__((ext_vector_type(4)));

// DIAG (timing probes, NTS_X3_DIAG in the probe build only; results are
// garbage): 1 no MFMAs, 2 no A splits, 4 no DMA after each round's first
// steps, 8 no B fragment reads
template <bool EPI, int DIAG = 0>
__global__ __launch_bounds__(kX3Threads, 1) void k_x3_nn(int M, int N, int K, const float* __restrict__ X,
                                                        uint64_t ldx, const uint32_t* __restrict__ amap,
                                                        const char* __restrict__ bimg,
                                                        float* __restrict__ C, uint64_t ldc, int rounds,
                                                        X3Epi ep) {
  extern __shared__ __attribute__((aligned(16))) char x3nn[];
  char* const sb = x3nn;                 // [2][kX3NnImg]
  char* const sa = x3nn + 2 * kX3NnImg;  // [3][8 waves][2 tiles][2048]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, q = lane >> 4;
  const int nb = blockIdx.y, n0 = nb * 128;
  const int T = (M + 15) / 16;
  const int64_t Wn = (int64_t)gridDim.x * 8, gw = (int64_t)blockIdx.x * 8 + wv;
  const int t_lo = (int)(gw * T / Wn), t_hi = (int)((gw + 1) * T / Wn);
  const int nsteps = (K + 31) / 32;
  const size_t bstride = (size_t)gridDim.y * kX3NnImg;
  const uint32_t lsb = x3_lds(sb), lsa = x3_lds(sa);
#ifdef NTS_X3_PRIO
  if (wv >= 4) __builtin_amdgcn_s_setprio(1);  // A/B: static priority for the younger half
#endif
  const char* bsrc = bimg + (size_t)nb * kX3NnImg + wv * 1024 + 16 * lane;
  // A DMA role: lane l loads row (l >> 1) & 15, floats 8 (l >> 5) + 4 (l & 1) (+ 16 h)
  const int gr = (lane >> 1) & 15, gpo = 8 * (lane >> 5) + 4 * (lane & 1);
  const float* arow[2];
  auto set_rows = [&](int rd) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int t = min(t_lo + 2 * rd + rt, T - 1);
      const int64_t row = (int64_t)t * 16 + gr;
      const uint64_t rr = (uint64_t)(row < M ? row : M - 1);
      arow[rt] = X + (amap ? (uint64_t)amap[rr] : rr) * ldx + gpo;
    }
  };
  auto issue_b = [&](int s) {
    if ((DIAG & 4) && s >= 2) return;
    const uint32_t dst = lsb + (s & 1) * kX3NnImg + wv * 1024;
    const char* src = bsrc + (size_t)s * bstride;
#pragma unroll
    for (int p = 0; p < 3; ++p) x3_glds16(src + 8192 * p, dst + 8192 * p);
  };
  auto issue_a = [&](int s) {
    if ((DIAG & 4) && s >= 2) return;
    const uint32_t dst = lsa + (s % 3) * kX3NnA + wv * kX3NnAWave;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int h = 0; h < 2; ++h) x3_glds16(arow[rt] + 32 * s + 16 * h, dst + rt * 2048 + h * 1024);
  };
  x3f4 acc[2][8];
  float xr[2][8];           // raw A fragments (one step, per row tile)
  uint32_t ap[2][2][3][4];  // split A pieces: [step parity][row tile][piece][pair]
  // A(s) fragments: lane (i, q) of tile rt holds A[row i][32 s + 8 q .. +7]
  // (this wave's own slab: only its own DMA count guards it, no barrier)
  auto read_a = [&](int s, int rt) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const char* as = sa + (s % 3) * kX3NnA + wv * kX3NnAWave + 32 * (i + 16 * q) + rt * 2048;
    const f4v u = *reinterpret_cast<const f4v*>(as);
    const f4v v = *reinterpret_cast<const f4v*>(as + 16);
    const float x[8] = {u[0], u[1], u[2], u[3], v[0], v[1], v[2], v[3]};
#pragma unroll
    for (int j = 0; j < 8; ++j) xr[rt][j] = x[j];
    if (32 * s + 32 > K) {  // the pad past K (the last step only: a uniform branch)
#pragma unroll
      for (int j = 0; j < 8; ++j) xr[rt][j] = 32 * s + 8 * q + j < K ? x[j] : 0.f;
    }
  };
  auto split_a = [&](auto par, int rt, int jp) {
    constexpr int P = decltype(par)::value;
    if constexpr (DIAG & 2) {
      ap[P][rt][0][jp] = ap[P][rt][1][jp] = ap[P][rt][2][jp] = __float_as_uint(xr[rt][2 * jp]);
    } else {
      x3_split2(xr[rt][2 * jp], xr[rt][2 * jp + 1], ap[P][rt][0][jp], ap[P][rt][1][jp], ap[P][rt][2][jp]);
    }
  };
  // one k-step on the split A(s) in ap[P]; A(s+1) is read and split into
  // ap[1-P] in the second half of the column tiles, after a mid-step wait for
  // its 4 pieces (younger in flight: B(s+1)'s 3 and A(s+2)'s 4)
  // NT: the row tiles this wave computes this round (2, or 1 in a round with
  // one tile left: the MFMAs, A reads and splits of the idle tile skipped —
  // its DMA still runs, so the counted waits are the same)
  auto step = [&](int s, auto par, auto ntc) {
    constexpr int P = decltype(par)::value, NT = decltype(ntc)::value;
    if (s > 0) {
      // B(s) landed (A(s) was waited for in step s-1; A(s+1)'s 4 pieces may stay in flight)
      // (drained, not counted: k_x3_tn showed the LDS-DMA loads need not
      // retire in issue order; this kernel serves the gathered NN below
      // k_x3_nn7's 32,768 rows, where the drain costs little)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      x3_barrier();
      if (s + 1 < nsteps) issue_b(s + 1);
      if (s + 2 < nsteps) issue_a(s + 2);
    }
    const char* img = sb + (s & 1) * kX3NnImg;
    auto getb = [&](int ct, int p) {
      if constexpr (DIAG & 8) return x3bf8{};
      else return *reinterpret_cast<const x3bf8*>(img + ct * 3072 + p * 1024 + 16 * lane);
    };
    x3bf8 bf[2][3];
#pragma unroll
    for (int p = 0; p < 3; ++p) bf[0][p] = getb(0, p);
    x3bf8 a[2][3];
#pragma unroll
    for (int rt = 0; rt < NT; ++rt)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        a[rt][p] = __builtin_bit_cast(x3bf8, (x3u4){ap[P][rt][p][0], ap[P][rt][p][1], ap[P][rt][p][2], ap[P][rt][p][3]});
#pragma unroll
    for (int ct = 0; ct < 8; ++ct) {
#pragma unroll
      for (int k = 0; k < 6 * NT; ++k) {
        __builtin_amdgcn_sched_barrier(0);
        {  // slot k: product k / NT (small first) of row tile k % NT
          const int rt = NT == 2 ? (k & 1) : 0, pr = NT == 2 ? (k >> 1) : k;
          const int pa = pr == 0 ? 2 : pr == 1 ? 1 : pr == 2 ? 0 : pr == 3 ? 1 : 0;
          const int pb = pr == 0 ? 0 : pr == 1 ? 1 : pr == 2 ? 2 : pr == 3 ? 0 : pr == 4 ? 1 : 0;
          if constexpr (DIAG & 1) acc[rt][ct][0] += (float)a[rt][pa][0] + (float)bf[ct & 1][pb][1];
          else if constexpr (EPI)
            acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rt][pa], bf[ct & 1][pb], acc[rt][ct], 0, 0, 0);
          else  // C^T = W^T X^T: the same fragments, operands swapped
            acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ct & 1][pb], a[rt][pa], acc[rt][ct], 0, 0, 0);
        }
        if (ct + 1 < 8 && (k == 0 || k == 2 || k == 4)) bf[(ct + 1) & 1][k / 2] = getb(ct + 1, k / 2);
        // (unconditional: past the round's last step this reads and splits a
        // stale stage nobody uses, cheaper than branching every slot)
        if (ct == 4 && k == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // A(s+1) (drained)
        if (ct == 4 && k == 1) read_a(s + 1, 0);
        if constexpr (NT == 2) {
          if (ct == 4 && k == 3) read_a(s + 1, 1);
          if ((ct == 5 || ct == 6) && k % 3 == 1) split_a(std::integral_constant<int, 1 - P>{}, ct - 5, k / 3);
        } else {
          if (ct == 5 && (k & 1)) split_a(std::integral_constant<int, 1 - P>{}, 0, k >> 1);
          if (ct == 6 && k == 1) split_a(std::integral_constant<int, 1 - P>{}, 0, 3);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto round_steps = [&](auto ntc) {
    constexpr int NT = decltype(ntc)::value;
    issue_b(0);
    issue_a(0);
    if (nsteps > 1) issue_a(1);
    // B(0) and A(0) landed (drained)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    x3_barrier();
    if (nsteps > 1) issue_b(1);
    if (nsteps > 2) issue_a(2);
#pragma unroll
    for (int rt = 0; rt < NT; ++rt) read_a(0, rt);
#pragma unroll
    for (int rt = 0; rt < NT; ++rt)
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) split_a(std::integral_constant<int, 0>{}, rt, jp);
    for (int s = 0; s < nsteps; s += 2) {
      step(s, std::integral_constant<int, 0>{}, ntc);
      if (s + 1 < nsteps) step(s + 1, std::integral_constant<int, 1>{}, ntc);
    }
  };
  for (int rd = 0; rd < rounds; ++rd) {
    const int nt = min(2, max(0, t_hi - (t_lo + 2 * rd)));  // this wave's tiles this round
    set_rows(rd);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) acc[rt][ct] = x3f4{0.f, 0.f, 0.f, 0.f};
    // (a round with one tile left — at C2 the last of every wave's four —
    // runs half the MFMAs; the block's waves still meet at every barrier)
#ifdef NTS_X3_NO_NT1  // (A/B build: every round on both tiles)
    round_steps(std::integral_constant<int, 2>{});
#else
    if (nt == 2) round_steps(std::integral_constant<int, 2>{});
    else round_steps(std::integral_constant<int, 1>{});
#endif
    x3_barrier();  // every wave is done with the B stages before the next round's
    if constexpr (!EPI) {
      // transposed accumulators: acc[rt][ct][v] = C[16 t + i][n0 + 16 ct + 4 q + v],
      // one 16-byte store per tile and lane
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        if (rt >= nt) continue;
        const int64_t row = (int64_t)(t_lo + 2 * rd + rt) * 16 + i;
        if (row >= M) continue;
#pragma unroll
        for (int ct = 0; ct < 8; ++ct) {
          const int col = n0 + 16 * ct + 4 * q;
          if (col >= N) continue;
          float* dst = C + (uint64_t)row * ldc + col;
          if (ldc % 4 == 0 && (uintptr_t)C % 16 == 0)
            *reinterpret_cast<x3f4*>(dst) = acc[rt][ct];
          else
#pragma unroll
            for (int v = 0; v < 4; ++v) dst[v] = acc[rt][ct][v];
        }
      }
      continue;
    }
    // epilogue: acc[rt][ct][v] = C[16 t + 4 q + v][n0 + 16 ct + i]
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      if (rt >= nt) continue;
      const int64_t r4 = (int64_t)(t_lo + 2 * rd + rt) * 16 + 4 * q;
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
        const uint32_t col = (uint32_t)(n0 + 16 * ct + i);
        if ((int)col >= N) continue;
        float o[4] = {acc[rt][ct][0], acc[rt][ct][1], acc[rt][ct][2], acc[rt][ct][3]};
        if constexpr (EPI) {
          const uint4 rnd = dropout_words((uint64_t)r4, col, ep.seed, ep.offset);
          const uint32_t wd[4] = {rnd.x, rnd.y, rnd.z, rnd.w};
#pragma unroll
          for (int v = 0; v < 4; ++v)
            o[v] = (dropout_bits(wd[v], col) >= ep.keep_threshold && o[v] > 0.f) ? o[v] * ep.scale : 0.f;
        }
#pragma unroll
        for (int v = 0; v < 4; ++v)
          if (r4 + v < M) C[(uint64_t)(r4 + v) * ldc + col] = o[v];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// NN, round 6: k_x3_nn7 — the product of k_x3_nn (same fragments, same piece
// order, same k order: bit-identical), reorganised so that the W image is
// streamed once per 7 x 16 = 112 rows of every wave instead of once per 32,
// and the gathered rows skip LDS:
//   * 4-wave blocks, one wave per SIMD (up to 512 registers a lane); each
//     wave owns the contiguous 16-row tiles [gw T / W, (gw+1) T / W), in
//     rounds of RT = 7 tiles x 128 columns (224 accumulator registers); the
//     MFMAs of a step are row-tile major (tile t's 48, then tile t+1's);
//   * per 32-deep k-step the block shares one 24 KB W image in LDS (three
//     buffers, 6 LDS-DMA pieces per wave and step, one barrier per step); the
//     B fragments of column tile c+1 are read while column tile c's six MFMAs
//     run (two register sets);
//   * each wave's own A rows are loaded straight to registers (two 16-byte
//     loads per lane, tile and step) one step ahead, and split into the three
//     bf16 pieces one tile ahead of their MFMAs, one split instruction per
//     MFMA slot;
//   * the loads run on across rounds (the next round's first rows are in
//     flight during a round's last step); the accumulators are stored at each
//     round's end.
// VMEM order per step g (W(g) in LDS buffer g % 3): tile t < RT-1 issues
// kX3N7Wp[t] pieces of W(g+1), then the A loads of tile t+1 for step g+1;
// tile RT-1 issues the A loads of tile 0 for step g+2 and, at its start,
// waits for its own W(g+1) pieces (counted by hand: hipcc does not see the
// LDS DMA) and meets the block's barrier — after which W(g+1) is visible and
// every wave is done with step g-1, so buffer (g+2) % 3 (= W(g-1)'s) is free
// for the next step's pieces.  hipcc's own waits for the A registers count
// only its own loads (over-waiting by the W pieces: still >= 4 tiles of
// slack).
constexpr int kX3N7Threads = 256;
constexpr int kX3N7RT = 7;
constexpr int kX3N7Lds = 3 * kX3NnImg;  // 72 KB
// W(g+1) pieces issued per tile (6 per wave and step: 24 KB / 4 waves)
__device__ constexpr int kX3N7Wp[kX3N7RT] = {2, 2, 2, 0, 0, 0, 0};
// after the last W piece (tile 2): tile 2's own A loads and tiles 3..5's
constexpr int kX3N7WWait = 2 * (kX3N7RT - 1 - 2);
// the piece set of each tile (consecutive tiles, the last tile and the next
// step's first included, never share a set)
__device__ constexpr int kX3N7Pb[kX3N7RT] = {0, 1, 2, 0, 1, 2, 1};

// compile-time loop: f(integral_constant<int, I>) for I in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void x3_sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    x3_sfor<B + 1, E>(f);
  }
}

// one of the 44 instructions of the exact split of 8 fp32 values x (one
// lane's A fragment) into three packed bf16 pieces p[0..2][0..3]: the
// instruction sequence of x3_split2 for four pairs in lock step, so that each
// instruction's operands were produced at least four slots earlier
template <int O>
__device__ __forceinline__ void x3_split_op(const float (&x)[8], float (&r)[8], float (&f)[8],
                                            uint32_t (&p)[3][4]) {
  auto pk = [](float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((x3f2){a, b}, x3bf2));
  };
  if constexpr (O < 4) {  // x0 = bf16(x)
    p[0][O] = pk(x[2 * O], x[2 * O + 1]);
  } else if constexpr (O < 12) {  // back to fp32
    constexpr int e = O - 4;
    f[e] = __uint_as_float((e & 1) ? (p[0][e / 2] & 0xffff0000u) : (p[0][e / 2] << 16));
  } else if constexpr (O < 20) {  // r = x - x0 (exact)
    r[O - 12] = x[O - 12] - f[O - 12];
  } else if constexpr (O < 24) {  // x1 = bf16(r)
    p[1][O - 20] = pk(r[2 * (O - 20)], r[2 * (O - 20) + 1]);
  } else if constexpr (O < 32) {
    constexpr int e = O - 24;
    f[e] = __uint_as_float((e & 1) ? (p[1][e / 2] & 0xffff0000u) : (p[1][e / 2] << 16));
  } else if constexpr (O < 40) {  // r - x1 (exact)
    r[O - 32] = r[O - 32] - f[O - 32];
  } else if constexpr (O < 44) {  // x2 = bf16(r - x1) (exact)
    p[2][O - 40] = pk(r[2 * (O - 40)], r[2 * (O - 40) + 1]);
  }
}

// The W image reaches LDS through registers (normal loads, whose waits hipcc
// counts exactly) — not by LDS DMA with a hand-counted wait: k_x3_tn showed
// the DMA counter need not retire in issue order, and the DMA form's counted
// W wait once left a C2-size product not bit-identical to k_gemm3_nn's (round
// 6, r06final).  -DNTS_X3N7_WDMA keeps the DMA form for A/B.
#ifndef NTS_X3N7_WDMA
#define NTS_X3N7_WREG 1
#endif
// B fragments read this many column tiles ahead (NTS_X3N7_BQ: 1 or 2)
#ifndef NTS_X3N7_BQ
#define NTS_X3N7_BQ 1
#endif
// DIAG (timing probes, NTS_X3_DIAG in the probe build only; results are
// garbage): 1 no MFMAs, 2 no splits, 4 no A loads after the prologue, 8 no B
// fragment reads, 16 no W DMA after the prologue (and no wait for it), 32 no
// barrier
// EPI: relu + inverted dropout epilogue (the non-swapped product, k_x3_nn<true>'s
// accumulator layout and mask keys: bit-identical to it)
template <int RT, int DIAG = 0, bool EPI = false>
__global__ __launch_bounds__(kX3N7Threads, 1) void k_x3_nn7(int M, int N, int K, const float* __restrict__ X,
                                                           uint64_t ldx, const uint32_t* __restrict__ amap,
                                                           const char* __restrict__ bimg, float* __restrict__ C,
                                                           uint64_t ldc, int rounds, X3Epi ep) {
  static_assert(RT == kX3N7RT, "the W piece schedule is written for 7 tiles");
  extern __shared__ __attribute__((aligned(16))) char x3n7[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, q = lane >> 4;
  const int nb = blockIdx.y, n0 = nb * 128;
  const int T = (M + 15) / 16;
  const int64_t Wn = (int64_t)gridDim.x * 4, gw = (int64_t)blockIdx.x * 4 + wv;
  const int t_lo = (int)(gw * T / Wn), t_hi = (int)((gw + 1) * T / Wn);
  const int nsteps = (K + 31) / 32;
  const uint64_t bstride = (uint64_t)gridDim.y * kX3NnImg;
  const uint32_t lsw = x3_lds(x3n7) + 6144 * wv;  // this wave's 6 KB share of a W buffer
  const char* bsrc = bimg + (size_t)nb * kX3NnImg + 6144 * wv + 16 * lane;
  // the lane's row id in tile slot rt of round rd (slots past the wave's
  // tiles repeat its last tile: computed, never stored)
  auto row_id = [&](int rd, int rt) -> uint32_t {
    int t = min(t_lo + RT * rd + rt, max(t_hi, t_lo + 1) - 1);
    t = min(t, T - 1);
    int64_t r = (int64_t)t * 16 + i;
    if (r >= M) r = M - 1;
    const uint32_t id = amap ? amap[r] : (uint32_t)r;
    return (DIAG & 64) ? (id & 1023u) : id;  // (probe: an L2-resident working set)
  };
  const float* ptr[RT];  // slot rt's rows (+ 8 q), in the round of its next load
  uint32_t nid[RT];      // the next round's row ids
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) ptr[rt] = X + (uint64_t)row_id(0, rt) * ldx + 8 * q;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) nid[rt] = row_id(1, rt);
#ifndef NTS_X3N7_WREG  // (A/B build -DNTS_X3N7_WDMA: the W image by LDS DMA)
  auto issue_w = [&](int s, int buf, int piece) {  // piece of W(k-step s) into buffer buf
    x3_glds16(bsrc + (size_t)s * bstride + 1024 * piece, lsw + buf * kX3NnImg + 1024 * piece);
  };
#else
  // the W image staged through registers: hipcc counts these loads with the
  // A loads, so its waits for the A registers are exact (an LDS DMA it cannot
  // see made every such wait cover six more loads)
  // (all six pieces of W(g+1) loaded at the start of step g, before the A
  // loads of step g: their wait at the step's last tile then forces no A
  // load of this step — the VMEM counter is in order)
  x3f4 wst[6];
  char* const wdst = x3n7 + 6144 * wv + 16 * lane;
  auto load_w = [&](int s, auto pc) {
    constexpr int piece = decltype(pc)::value;
    wst[piece] = *reinterpret_cast<const x3f4*>(bsrc + (size_t)s * bstride + 1024 * piece);
  };
  // (inline asm: a plain LDS store was hoisted to its load, waiting for it)
  const uint32_t wdst_l = x3_lds(wdst);
  auto store_w = [&](int buf, auto pc) {
    constexpr int piece = decltype(pc)::value;
    const uint32_t addr = wdst_l + buf * kX3NnImg;
    const x3f4 v = wst[piece];
    asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(addr), "v"(v), "n"(1024 * piece) : "memory");
  };
#endif
  float4 raw[RT][2];  // A fragments of one step (tile 0: the next step's)
  auto load_a = [&](int rt, int s) {
    const float* p = ptr[rt] + 32 * s;
    raw[rt][0] = *reinterpret_cast<const float4*>(p);
    raw[rt][1] = *reinterpret_cast<const float4*>(p + 4);
  };
  x3f4 acc[RT][8];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int ct = 0; ct < 8; ++ct) acc[rt][ct] = x3f4{0.f, 0.f, 0.f, 0.f};
  uint32_t pcs[3][3][4];  // split A pieces, tile t in pcs[kX3N7Pb[t]]
  constexpr int NB = NTS_X3N7_BQ + 1;
  x3bf8 bq[NB][3];        // B fragments, column tile c in bq[c % NB]
  float sr[8], sf[8];     // split temporaries
  auto read_b = [&](int buf, int ct, int p) {
    return *reinterpret_cast<const x3bf8*>(x3n7 + buf * kX3NnImg + ct * 3072 + p * 1024 + 16 * lane);
  };
  // the pad past K (a step past it only, wave-uniform): zero the raw values
  auto mask_k = [&](float (&x)[8], int s) {
    if (32 * s + 32 > K) {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = 32 * s + 8 * q + j < K ? x[j] : 0.f;
    }
  };
  auto raw8 = [&](int rt, float (&x)[8]) {
    x[0] = raw[rt][0].x; x[1] = raw[rt][0].y; x[2] = raw[rt][0].z; x[3] = raw[rt][0].w;
    x[4] = raw[rt][1].x; x[5] = raw[rt][1].y; x[6] = raw[rt][1].z; x[7] = raw[rt][1].w;
  };
  // ---- prologue: W(0) -> buffer 0, A(0) of every tile; split tile 0; A(1)
  // of tile 0; W(1) -> buffer 1 (ordered as one step's tile 6 -> tile 0)
#ifndef NTS_X3N7_WREG
#pragma unroll
  for (int p = 0; p < 6; ++p) issue_w(0, 0, p);
#else
  x3_sfor<0, 6>([&](auto pc) {
    load_w(0, pc);
    store_w(0, pc);
  });
#endif
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) load_a(rt, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  x3_barrier();
  {
    float x[8];
    raw8(0, x);
    mask_k(x, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) x3_split2(x[2 * j], x[2 * j + 1], pcs[0][0][j], pcs[0][1][j], pcs[0][2][j]);
  }
  load_a(0, 1);  // (nsteps >= 4)
#pragma unroll
  for (int c = 0; c < NTS_X3N7_BQ; ++c)
#pragma unroll
    for (int p = 0; p < 3; ++p) bq[c][p] = read_b(0, c, p);
  // ---- the steps of every round
  int wb = 0;  // W(g)'s buffer
  for (int rd = 0; rd < rounds; ++rd) {
  for (int s = 0; s < nsteps; ++s) {
    int s1 = s + 1, rd1 = rd;
    if (s1 == nsteps) { s1 = 0; ++rd1; }
    int s2 = s1 + 1, rd2 = rd1;
    if (s2 == nsteps) { s2 = 0; ++rd2; }
    const int wb1 = wb == 2 ? 0 : wb + 1;  // W(g+1)'s buffer
    x3_sfor<0, RT>([&](auto rtc) {
      constexpr int rt = decltype(rtc)::value;
      constexpr int cur = kX3N7Pb[rt], nxt = kX3N7Pb[rt + 1 < RT ? rt + 1 : 0];
      x3bf8 a[3];
#pragma unroll
      for (int p = 0; p < 3; ++p)
        a[p] = __builtin_bit_cast(x3bf8, (x3u4){pcs[cur][p][0], pcs[cur][p][1], pcs[cur][p][2], pcs[cur][p][3]});
      // the raw values this tile splits: tile rt+1 of this step, or (last
      // tile) tile 0 of the next step
      constexpr int srt = rt + 1 < RT ? rt + 1 : 0;
      const int ss = rt + 1 < RT ? s : s1;
      float x[8];
      if constexpr (rt + 1 == RT) {  // W(g+1) landed (own pieces), then the block's
#ifndef NTS_X3N7_WREG
#ifdef NTS_X3N7_WAIT0  // (A/B build: drain every load at the W wait)
        if constexpr (!(DIAG & 16)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
        if constexpr (!(DIAG & 16)) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kX3N7WWait) : "memory");
#endif
#else
        if constexpr (!(DIAG & 16)) x3_sfor<0, 6>([&](auto pc) { store_w(wb1, pc); });
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's W(g+1) stores
#endif
        if constexpr (!(DIAG & 32)) x3_barrier();  // and every wave's
      }
      __builtin_amdgcn_sched_barrier(0);
      raw8(srt, x);
      mask_k(x, ss);
      x3_sfor<0, 48>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        constexpr int ct = k / 6, pr = k % 6;
        __builtin_amdgcn_sched_barrier(0);
        {  // slot k: product pr (small first) of column tile ct
          constexpr int pa = pr == 0 ? 2 : pr == 1 ? 1 : pr == 2 ? 0 : pr == 3 ? 1 : 0;
          constexpr int pb = pr == 0 ? 0 : pr == 1 ? 1 : pr == 2 ? 2 : pr == 3 ? 0 : pr == 4 ? 1 : 0;
          if constexpr (DIAG & 1) acc[rt][ct][0] += (float)a[pa][0] + (float)bq[ct % NB][pb][1];
          else if constexpr (EPI)
            acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[pa], bq[ct % NB][pb], acc[rt][ct], 0, 0, 0);
          else  // C^T = W^T X^T: the same fragments, operands swapped (16-byte row stores)
            acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[ct % NB][pb], a[pa], acc[rt][ct], 0, 0, 0);
        }
        // the next column tile's B fragments (slots 6 ct .. 6 ct + 2): W(g)'s,
        // or after the last column tile of the last tile W(g+1)'s column tile 0
        if constexpr (pr < 3) {
          constexpr int cn = ct + NTS_X3N7_BQ;  // the column tile read (8, 9: the next tile's 0, 1)
          if constexpr (DIAG & 8) {
          } else if constexpr (cn < 8) bq[cn % NB][pr] = read_b(wb, cn, pr);
          else if constexpr (rt + 1 < RT) bq[(cn - 8) % NB][pr] = read_b(wb, cn - 8, pr);
          else bq[(cn - 8) % NB][pr] = read_b(wb1, cn - 8, pr);
        }
        // one split instruction per slot (slots 1..44)
        if constexpr (DIAG & 2) {
          if constexpr (k >= 1 && k <= 12) pcs[nxt][(k - 1) / 4][(k - 1) % 4] = __float_as_uint(x[(k - 1) % 8]);
        } else if constexpr (k >= 1 && k <= 44) x3_split_op<k - 1>(x, sr, sf, pcs[nxt]);
        if constexpr (rt + 1 < RT) {
          // W(g+1) pieces (buffer (g+1) % 3 held W(g-2): free since every
          // wave passed step g-1's barrier)
#ifndef NTS_X3N7_WREG
          if constexpr (!(DIAG & 16) && kX3N7Wp[rt] > 0 && (k == 4 || k == 28)) issue_w(s1, wb1, 2 * rt + (k == 28));
#else
          // W(g+1) (tile 0, slots 2..7), stored into buffer (g+1) % 3 at tile RT-1
          if constexpr (!(DIAG & 16) && rt == 0 && k >= 2 && k < 8)
            load_w(s1, std::integral_constant<int, (k >= 2 && k < 8 ? k - 2 : 0)>{});
#endif
        }
        // the split's r = x - x0 ran (slot 20): the raw registers are free
        if constexpr (k == 22 && !(DIAG & 4)) {
          if constexpr (rt + 1 < RT) {
            if (s1 == 0 && rd1 < rounds) ptr[srt] = X + (uint64_t)nid[srt] * ldx + 8 * q;
            load_a(srt, s1);
          } else {
            if (s2 == 0 && rd2 < rounds) ptr[0] = X + (uint64_t)nid[0] * ldx + 8 * q;
            load_a(0, s2);
          }
        }
      });
      __builtin_amdgcn_sched_barrier(0);
    });
    wb = wb1;
  }
    // round end: store the round's tiles, zero the accumulators, fetch the
    // row ids of the round after next
    {
      x3_sfor<0, RT>([&](auto rtc) {
        constexpr int rt = decltype(rtc)::value;
        const int t = t_lo + RT * rd + rt;
        if constexpr (!EPI) {
          // acc[rt][ct][v] = C[16 t + i][n0 + 16 ct + 4 q + v]
          const int64_t row = (int64_t)t * 16 + i;
          if (t < t_hi && row < M) {
#pragma unroll
            for (int ct = 0; ct < 8; ++ct) {
              const int col = n0 + 16 * ct + 4 * q;
              if (col < N) *reinterpret_cast<x3f4*>(C + (uint64_t)row * ldc + col) = acc[rt][ct];
            }
          }
        } else if (t < t_hi) {
          // acc[rt][ct][v] = C[16 t + 4 q + v][n0 + 16 ct + i], relu + dropout
          // (compile-time indices throughout: a runtime-indexed accumulator
          // array goes to scratch)
          const int64_t r4 = (int64_t)t * 16 + 4 * q;
          x3_sfor<0, 8>([&](auto ctc) {
            constexpr int ct = decltype(ctc)::value;
            const uint32_t col = (uint32_t)(n0 + 16 * ct + i);
            if ((int)col < N) {
              const uint4 rnd = dropout_words((uint64_t)r4, col, ep.seed, ep.offset);
              const uint32_t wd[4] = {rnd.x, rnd.y, rnd.z, rnd.w};
              x3_sfor<0, 4>([&](auto vc) {
                constexpr int v = decltype(vc)::value;
                const float o = acc[rt][ct][v];
                if (r4 + v < M)
                  C[(uint64_t)(r4 + v) * ldc + col] =
                      (dropout_bits(wd[v], col) >= ep.keep_threshold && o > 0.f) ? o * ep.scale : 0.f;
              });
            }
          });
        }
#pragma unroll
        for (int ct = 0; ct < 8; ++ct) acc[rt][ct] = x3f4{0.f, 0.f, 0.f, 0.f};
      });
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) nid[rt] = row_id(rd + 2, rt);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS DMA outlives the block
}

// ---------------------------------------------------------------------------
// launchers (gemm3.hip's gemm3_tn / gemm3_nn try these first)

// whole rows of at most 608 floats (Kp), 16-byte aligned, read as Kp floats
// (so the table's row pitch must cover Kp); 128-column blocks
bool x3_tn_ok(int M, int N, int K, const float* A, uint64_t lda, const float* B, uint64_t ldb,
              const float* Xm, uint64_t ldxm) {
  const int Kp = (M + 31) / 32 * 32;
  // the X stages, dH stages (+ the mask rows) and planes leave room for >= 256
  // row ids (Kp <= 608)
  const int lds = 3 * 16 * 4 * Kp + 2 * kX3BRaw + 6 * kX3BPl + (Xm ? 2 * kX3BRaw : 0) + 4 * 16 * 3 +
                  4 * 256;
  return M >= 32 && lds <= 160 * 1024 && N % 128 == 0 && K >= 256 && lda >= (uint64_t)Kp && lda % 4 == 0 &&
         (uintptr_t)A % 16 == 0 && ldb % 4 == 0 && (uintptr_t)B % 16 == 0 &&
         (!Xm || (ldxm % 4 == 0 && (uintptr_t)Xm % 16 == 0));
}

int x3_tn(nts_hip_ctx* ctx, int M, int N, int K, const float* A, uint64_t lda, const uint32_t* amap,
          const float* B, uint64_t ldb, float* C, uint64_t ldc, const float* Xm, uint64_t ldxm,
          float bscale) {
  const int Kp = (M + 31) / 32 * 32, RB = 4 * Kp;
  const int nnb = N / 128;
  const int ksteps = (K + 15) / 16;
  int splits = std::max(1, std::min(256 / nnb, ksteps / 8));
  int kchunk = ((ksteps + splits - 1) / splits) * 16;
  const int fixed = 3 * 16 * RB + 2 * kX3BRaw + 6 * kX3BPl + (Xm ? 2 * kX3BRaw : 0) + 4 * 16 * 3;
  kchunk = std::min(kchunk, (160 * 1024 - fixed) / 4 / 16 * 16);
  splits = (K + kchunk - 1) / kchunk;
  const int lds = fixed + 4 * kchunk;
  const uint64_t stride = (uint64_t)M * N;
  float* out = C;
  uint64_t ldo = ldc;
  if (splits > 1) {
    NTS_RET(ensure_scratch(ctx, stride * splits * sizeof(float) + 256));
    out = (float*)ctx->scratch;
    ldo = N;
  }
  const int pr = (RB + 1023) / 1024;
  // tiles a wave: the 32-row tiles of M over 4 row groups (5 for C2's 602;
  // 1 for C3 / C4's 100 — tiles past a wave's own repeat its last one, so a
  // TPW above its count is pure waste)
  const int tpw = ((M + 31) / 32 + 3) / 4;
#define NTS_X3TN(T, P, D, BMK)                                                                   \
  do {                                                                                           \
    NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_x3_tn<T, P, D, BMK>),      \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds));           \
    hipLaunchKernelGGL((k_x3_tn<T, P, D, BMK>), dim3(nnb * splits), dim3(kX3Threads), lds,      \
                       ctx->stream, M, K, A, lda, amap, B, ldb, out, ldo, kchunk,                \
                       splits > 1 ? stride : (uint64_t)0, nnb, Xm, ldxm, bscale);                \
  } while (0)
#ifdef NTS_PROBE_BUILD
  static const int diag = [] {
    const char* e = getenv("NTS_X3_DIAG");
    return e ? atoi(e) : 0;
  }();
  if (pr == 3 && diag && !Xm) {
    switch (diag) {
      case 1: NTS_X3TN(5, 3, 1, false); break;
      case 2: NTS_X3TN(5, 3, 2, false); break;
      case 4: NTS_X3TN(5, 3, 4, false); break;
      case 5: NTS_X3TN(5, 3, 5, false); break;
      case 6: NTS_X3TN(5, 3, 6, false); break;
      case 8: NTS_X3TN(5, 3, 8, false); break;
      case 10: NTS_X3TN(5, 3, 10, false); break;
      case 12: NTS_X3TN(5, 3, 12, false); break;
      case 14: NTS_X3TN(5, 3, 14, false); break;
      case 16: NTS_X3TN(5, 3, 16, false); break;
      case 32: NTS_X3TN(5, 3, 32, false); break;
      case 36: NTS_X3TN(5, 3, 36, false); break;
      default: NTS_X3TN(5, 3, 15, false); break;
    }
  } else
#endif
  // (the one-tile form for the masked short shapes; unmasked shapes keep TPW 5)
  if (Xm && tpw <= 1 && pr == 1) {
    NTS_X3TN(1, 1, 0, true);
  } else if (Xm) {
    return NTS_ERR_INVALID;  // (x3_tn_bm_ok keeps masked calls to one-tile shapes)
  } else if (pr == 1) NTS_X3TN(5, 1, 0, false);
  else if (pr == 2) NTS_X3TN(5, 2, 0, false);
  else NTS_X3TN(5, 3, 0, false);
#undef NTS_X3TN
  NTS_LAUNCH_CHECK();
  if (splits == 1) return NTS_OK;
  return sum_splits(ctx->stream, out, splits, stride, M, N, C, ldc);
}

// the masked (BM) form is instantiated for one-tile shapes only: M <= 128
bool x3_tn_bm_ok(int M, int N, int K, const float* A, uint64_t lda, const float* B, uint64_t ldb,
                 const float* Xm, uint64_t ldxm) {
  return M <= 128 && x3_tn_ok(M, N, K, A, lda, B, ldb, Xm, ldxm);
}

// NN over gathered rows (or dense, amap null): rows read as Kp = 32 ceil(K /
// 32) floats (the row pitch must cover them), 16-byte aligned
bool x3_nn_ok(int M, int N, int K, const float* A, uint64_t lda) {
  const int Kp = (K + 31) / 32 * 32;
  return M >= 256 && K >= 1 && N % 16 == 0 && lda >= (uint64_t)Kp && lda % 4 == 0 &&
         (uintptr_t)A % 16 == 0;
}
// k_x3_nn7's shapes: >= 4 k-steps (its rounds chain the next round's loads
// over the last two) and enough rows for its 4-wave blocks to fill the chip
// (2,048 16-row tiles: one round of 7 per wave over 256 blocks... and more)
bool x3_nn7_ok(int M, int N, int K, const float* A, uint64_t lda) {
  return x3_nn_ok(M, N, K, A, lda) && (K + 31) / 32 >= 4 && M >= 32768;
}

int x3_nn(nts_hip_ctx* ctx, bool epi, int M, int N, int K, const float* A, uint64_t lda,
          const uint32_t* amap, const char* bimg, float* C, uint64_t ldc, uint32_t keep_threshold,
          float scale, uint64_t seed, uint64_t offset) {
  X3Epi ep;
  ep.keep_threshold = keep_threshold;
  ep.scale = scale;
  ep.seed = seed;
  ep.offset = offset;
  // one 8-wave block per CU over all column blocks (row blocks a multiple of
  // 8: the column blocks of the same rows share an XCD), no more blocks than
  // 16-tile rounds (gemm3.hip's grid)
  const int ncb = (N + 127) / 128;
  const int T = (M + 15) / 16;
  int gx = std::max(8, (256 / ncb) / 8 * 8);
  gx = std::min(gx, std::max(8, ((T + 15) / 16 + 7) / 8 * 8));
  const int64_t Wn = (int64_t)gx * 8;
  const int max_tiles = (int)((T + Wn - 1) / Wn);
  const int rounds = (max_tiles + 1) / 2;
  const dim3 grid(gx, ncb);
#define NTS_X3NN(E, D)                                                                            \
  do {                                                                                            \
    NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_x3_nn<E, D>),                \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kX3NnLds));       \
    hipLaunchKernelGGL((k_x3_nn<E, D>), grid, dim3(kX3Threads), kX3NnLds, ctx->stream, M, N, K, A, \
                       lda, amap, bimg, C, ldc, rounds, ep);                                      \
  } while (0)
#ifndef NTS_X3_NN_V1  // (A/B builds: -DNTS_X3_NN_V1 keeps k_x3_nn for every call)
  if (x3_nn7_ok(M, N, K, A, lda)) {
    // k_x3_nn7: 4-wave blocks, at most one per CU and column block, each wave
    // kX3N7RT tiles a round
    const int T7 = (M + 15) / 16;
    const int gx7 = std::max(1, std::min(std::max(1, 256 / ncb), (T7 + 4 * kX3N7RT - 1) / (4 * kX3N7RT)));
    const int64_t W7 = (int64_t)gx7 * 4;
    const int tiles7 = (int)((T7 + W7 - 1) / W7);
    const int rounds7 = (tiles7 + kX3N7RT - 1) / kX3N7RT;
#define NTS_X3N7E(D, E)                                                                          \
  do {                                                                                           \
    NTS_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_x3_nn7<kX3N7RT, D, E>),     \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kX3N7Lds));      \
    hipLaunchKernelGGL((k_x3_nn7<kX3N7RT, D, E>), dim3(gx7, ncb), dim3(kX3N7Threads), kX3N7Lds,  \
                       ctx->stream, M, N, K, A, lda, amap, bimg, C, ldc, rounds7, ep);           \
  } while (0)
#define NTS_X3N7(D) NTS_X3N7E(D, false)
#ifdef NTS_PROBE_BUILD
    static const int diag7 = [] {
      const char* e = getenv("NTS_X3_DIAG");
      return e ? atoi(e) : 0;
    }();
    if (epi) NTS_X3N7E(0, true);
    else switch (diag7) {
      case 0: NTS_X3N7(0); break;
      case 1: NTS_X3N7(1); break;
      case 2: NTS_X3N7(2); break;
      case 4: NTS_X3N7(4); break;
      case 8: NTS_X3N7(8); break;
      case 16: NTS_X3N7(16); break;
      case 32: NTS_X3N7(32); break;
      case 6: NTS_X3N7(6); break;
      case 14: NTS_X3N7(14); break;
      case 62: NTS_X3N7(62); break;
      case 64: NTS_X3N7(64); break;
      case 68: NTS_X3N7(68); break;
      default: NTS_X3N7(63); break;
    }
#else
    if (epi) NTS_X3N7E(0, true);
    else NTS_X3N7(0);
#endif
#undef NTS_X3N7
#undef NTS_X3N7E
    NTS_LAUNCH_CHECK();
    return NTS_OK;
  }
#endif
#ifdef NTS_PROBE_BUILD
  static const int diag = [] {
    const char* e = getenv("NTS_X3_DIAG");
    return e ? atoi(e) : 0;
  }();
  if (!epi && diag) {
    switch (diag) {
      case 1: NTS_X3NN(false, 1); break;
      case 2: NTS_X3NN(false, 2); break;
      case 4: NTS_X3NN(false, 4); break;
      case 6: NTS_X3NN(false, 6); break;
      case 8: NTS_X3NN(false, 8); break;
      case 12: NTS_X3NN(false, 12); break;
      case 14: NTS_X3NN(false, 14); break;
      default: NTS_X3NN(false, 5); break;
    }
  } else
#endif
  if (epi) NTS_X3NN(true, 0);
  else NTS_X3NN(false, 0);
#undef NTS_X3NN
  NTS_LAUNCH_CHECK();
  return NTS_OK;
}

}  // namespace nts_hip
