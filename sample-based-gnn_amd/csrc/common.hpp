// Internal helpers shared by the HIP translation units of libnts_hip.so.
// Not part of the C-ABI (see include/nts_hip.h).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "nts_hip.h"

namespace nts_hip {

// ---- error plumbing (thread-local message, status codes) -----------------
void set_error(const char* fmt, ...);
// NTS_LAUNCH_TRACE=1 (debugging a hang): every launch check prints its site,
// waits for the device and prints it again
bool launch_trace();
void launch_trace_sync(const char* file, int line);

#define NTS_HIP_TRY(expr)                                                        \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    if (_e != hipSuccess) {                                                      \
      ::nts_hip::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #expr,    \
                           hipGetErrorString(_e));                               \
      return NTS_ERR_HIP;                                                        \
    }                                                                            \
  } while (0)

#define NTS_CHECK_ARG(cond, msg)                                                 \
  do {                                                                           \
    if (!(cond)) {                                                               \
      ::nts_hip::set_error("%s: invalid argument: %s", __func__, msg);          \
      return NTS_ERR_INVALID;                                                    \
    }                                                                            \
  } while (0)

#define NTS_LAUNCH_CHECK()                                                       \
  do {                                                                           \
    hipError_t _e = hipGetLastError();                                           \
    if (_e != hipSuccess) {                                                      \
      ::nts_hip::set_error("%s:%d: kernel launch failed: %s", __FILE__, __LINE__, \
                           hipGetErrorString(_e));                               \
      return NTS_ERR_HIP;                                                        \
    }                                                                            \
    if (::nts_hip::launch_trace()) ::nts_hip::launch_trace_sync(__FILE__, __LINE__); \
  } while (0)

#define NTS_RET(expr)                                                            \
  do {                                                                           \
    int _r = (expr);                                                             \
    if (_r != NTS_OK) return _r;                                                 \
  } while (0)

constexpr int kWave = 64;  // CDNA wavefront

// Philox4x32-10 (Salmon et al., SC'11): the counter-based generator behind the
// PHILOX sampling streams and the fused dropout masks.
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += W0;
    k.y += W1;
  }
  return c;
}

// Dropout keep bits shared by every fused relu/dropout epilogue: element
// (row, col) takes 16 bits of Philox4x32-10 at counter {row/4, col/2,
// offset_lo, offset_hi} under key `seed` — word row % 4, its low half for an
// even col and its high half for an odd col — and is kept iff those bits are
// >= floor(p * 65536).  One generator call covers a 4 x 2 element block.
__device__ __forceinline__ uint4 dropout_words(uint64_t row, uint32_t col, uint64_t seed,
                                               uint64_t offset) {
  return philox4x32_10(
      make_uint4((uint32_t)(row >> 2), col >> 1, (uint32_t)offset, (uint32_t)(offset >> 32)),
      make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
}
__device__ __forceinline__ uint32_t dropout_bits(uint32_t word, uint32_t col) {
  return (col & 1u) ? (word >> 16) : (word & 0xFFFFu);
}
inline uint32_t dropout_threshold(double p) {
  return p >= 1.0 ? 65536u : (uint32_t)std::min(p * 65536.0, 65536.0);
}

inline uint32_t ceil_div(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }
inline uint32_t ceil_log2(uint64_t x) {
  uint32_t b = 0;
  while ((uint64_t(1) << b) < x) ++b;
  return b;
}

// Memory-bound grid cap: 256 CUs x 8 blocks of 256 threads (guide G11).
constexpr uint32_t kMaxGrid = 2048;

}  // namespace nts_hip

// ---- context ---------------------------------------------------------------
struct nts_hip_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  uint64_t seed = 2000;
  // Scratch arena (grown by nts_hip_ctx_reserve / on demand).
  uint8_t* marks = nullptr;        // [V] frontier byte map
  uint32_t* src_index = nullptr;   // [V] global -> local id of the current layer
  uint64_t v_cap = 0;
  void* scratch = nullptr;         // scans / radix sort temporaries
  size_t scratch_bytes = 0;
  uint32_t* mt_state = nullptr;    // 624 words + position (device)
  uint64_t* scan_state = nullptr;  // single-pass scan tile states (epoch-tagged)
  uint64_t scan_state_elems = 0;
  uint32_t scan_epoch = 0;
  int gemm_mode = NTS_GEMM_F32;    // layer GEMM arithmetic (nts_hip_ctx_set_gemm_mode)
  // MT19937 modes: the generator's stream as tempered words in a device ring,
  // generated ahead of the layers that read it on a side stream (sampler.hip,
  // mt_ring_prepare).  Stream word a (0 = the first word after seeding) lives
  // at mt_ring[a % kMtRingWords]; mt_done = {position after the last MT layer
  // (40 bits) | that layer's sequence number (24 bits)}.
  uint32_t* mt_ring = nullptr;
  uint32_t* mt_gen_raw = nullptr;      // [624] the raw block the generator continues from
  uint64_t* mt_done = nullptr;         // device word, and its pinned host copy:
  uint64_t* mt_done_host = nullptr;
  uint64_t mt_gen_blocks = 0;          // 624-word blocks generated (issued)
  uint32_t mt_seq = 0;                 // MT layers issued since seeding
  uint64_t mt_pos_done = 0;            // host: last position read back, and its layer
  uint32_t mt_seq_done = 0;
  hipStream_t mt_gen_stream = nullptr;
  std::vector<std::pair<uint32_t, uint64_t>> mt_pending;    // (layer seq, word bound) not yet read back
  std::vector<std::pair<uint64_t, hipEvent_t>> mt_gen_evs;  // (blocks after, event) of generation launches
  std::vector<hipEvent_t> mt_ev_pool;
  double mt_budget_scale = 1.0;        // x every layer's word bound (nts_hip_mt_budget_scale)
};

namespace nts_hip {
// Ensure scratch capacity (may allocate: call nts_hip_ctx_reserve up front
// to keep the hot loop allocation-free).
int ensure_vertices(nts_hip_ctx* ctx, uint64_t n_vertices);
int ensure_scratch(nts_hip_ctx* ctx, size_t bytes);

// Exclusive scan of n items (n = *n_dev, or n_cap when n_dev == nullptr):
// out[i] = sum(in[0..i)) for i in [0, n]; out must hold n_cap+1 entries.
// In-place (in == out) is allowed.  tmp must hold scan_tmp_elems(n_cap).
template <typename T>
int scan_exclusive(const T* in, T* out, const uint32_t* n_dev, uint64_t n_cap, T* tmp,
                   hipStream_t stream);
template <typename T>
size_t scan_tmp_elems(uint64_t n_cap);

// Single-pass exclusive scan (u32, decoupled look-back; primitives.hip):
// out[i] = sum(in[0..i)) for i in [0, n], n = *n_dev (or n_cap).  One kernel.
int scan1_exclusive(nts_hip_ctx* ctx, const uint32_t* in, uint32_t* out, const uint32_t* n_dev,
                    uint64_t n_cap, hipStream_t stream);
int ensure_scan_state(nts_hip_ctx* ctx, uint64_t elems);
size_t scan1_state_elems(uint64_t n_cap);
// the next per-call epoch of the look-back tile states (never 0)
uint32_t scan_next_epoch(nts_hip_ctx* ctx);
// MT19937 stream ring (sampler.hip): forget the generated stream (seeding)
int mt_ring_reset(nts_hip_ctx* ctx);
int mt_ring_rebase(nts_hip_ctx* ctx);
void mt_ring_free(nts_hip_ctx* ctx);

// The tile a look-back workgroup works on: its ticket in dispatch order, not
// blockIdx.x.  Workgroups are not placed in index order across the XCDs, so
// once a grid exceeds what is resident at once (about 2K workgroups) a tile
// could wait on a lower-indexed one that never gets a slot: the frontier
// compaction of a 111 M-vertex graph (27 K tiles) hung that way.  With tickets
// every lower tile already runs.  The workgroup that draws the last ticket
// resets the counter (no other draw is left in the launch) for the stream's
// next one.  Every thread of the workgroup calls it.
__device__ __forceinline__ uint32_t lb_ticket(uint32_t* ctr, uint32_t nblk) {
  __shared__ uint32_t s_tile;
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == nblk - 1) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_tile = t;
  }
  __syncthreads();
  return s_tile;
}
// the ticket counter: the last word of the zeroed state array (past every
// tile's word)
inline uint32_t* scan_ticket(nts_hip_ctx* ctx) {
  return reinterpret_cast<uint32_t*>(ctx->scan_state + ctx->scan_state_elems - 1);
}

// Decoupled look-back (one wave, every lane calls): tile `tile` publishes its
// aggregate, sums its predecessors' states (RELAXED agent-scope atomics: each
// 64-bit word {epoch:30 | kind:2 | value:32} carries its own value) up to the
// first inclusive one, publishes its inclusive prefix and returns the
// exclusive one.  Tiles only wait on lower tiles, which already run when
// tiles are tickets (lb_ticket), so the chain completes.
__device__ __forceinline__ uint64_t lb_word(uint32_t epoch, uint64_t kind, uint32_t v) {
  return ((uint64_t)(epoch & 0x3FFFFFFFu) << 34) | (kind << 32) | v;
}
__device__ __forceinline__ uint32_t lookback_exclusive(uint64_t* state, uint32_t tile,
                                                       uint32_t epoch, uint32_t agg) {
  constexpr uint64_t kAgg = 1, kIncl = 2;
  const int lane = threadIdx.x & 63;
  if (tile == 0) {
    if (lane == 0)
      __hip_atomic_store(state, lb_word(epoch, kIncl, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0u;
  }
  if (lane == 0)
    __hip_atomic_store(state + tile, lb_word(epoch, kAgg, agg), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  uint32_t prefix = 0;
  int64_t top = (int64_t)tile - 1;
  for (;;) {
    const int64_t p = top - lane;
    uint64_t wd = 0;
    uint32_t kind = 0;
    if (p >= 0) {
      for (;;) {
        wd = __hip_atomic_load(state + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(wd >> 34) == (epoch & 0x3FFFFFFFu)) break;
        __builtin_amdgcn_s_sleep(1);
      }
      kind = (uint32_t)((wd >> 32) & 3u);
    }
    const uint64_t inc = __ballot(p >= 0 && kind == kIncl);
    const int stop = inc ? __ffsll((long long)inc) - 1 : 64;
    uint32_t add = (lane <= stop && p >= 0) ? (uint32_t)wd : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) add += __shfl_xor(add, o, 64);
    prefix += add;
    if (inc || top - 64 < 0) break;
    top -= 64;
  }
  if (lane == 0)
    __hip_atomic_store(state + tile, lb_word(epoch, kIncl, prefix + agg), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  return prefix;
}

// The sampler's per-dst counts fused into that scan: co[i] = min(deg(dst[i]),
// fanout) (0 for an omitted dst), exclusive-scanned; sizes[0] = v,
// sizes[1] = min(co[v], e_cap), overflow flags in sizes[3].
struct CountArgs {
  const uint64_t* goff;
  const uint32_t* dst;
  const uint32_t* v_in;
  uint32_t v_cap;
  int fanout;
  uint32_t* sizes;
  uint32_t e_cap;
  const uint32_t* omit_map;
  uint32_t omit_key;
  const uint32_t* omit_loc;
  uint32_t* omit_row;
};
// tmp: count_scan_tmp_elems(v_cap) words for the two-kernel form
// (NTS_SCAN1=0; the default and tmp == nullptr: the single-pass kernel)
int count_scan(nts_hip_ctx* ctx, const CountArgs& ca, uint32_t* co, hipStream_t stream,
               uint32_t* tmp);
size_t count_scan_tmp_elems(uint64_t v_cap);
bool scan1_enabled();

// Stable LSD radix sort of (key, value) pairs on the low `bits` key bits.
// n = *n_dev (or n_cap).  vals_in == nullptr means values = 0..n-1.
// Result lands in keys_out/vals_out.  tmp: radix_tmp_bytes(n_cap).
int radix_sort_pairs(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* keys_out,
                     uint32_t* vals_out, const uint32_t* n_dev, uint64_t n_cap,
                     uint32_t bits, void* tmp, hipStream_t stream, nts_hip_ctx* ctx = nullptr);
size_t radix_tmp_bytes(uint64_t n_cap);
// One stable pass of that sort on digit (key >> shift) & (2^dbits - 1), dbits
// <= 9: keys_in/vals_in -> keys_out/vals_out.  *totals (in tmp) receives the
// per-digit item counts (2^dbits words), valid on the stream after the pass.
// Tiles of 1,024 items (the generic sort: 4,096); tmp: radix_pass_tmp_bytes.
// vals_out may be NULL (keys and payloads only).
// Payloads (optional, vals_in NULL only): pN_out[pos] = pN_in[i] for the
// item i that lands at pos.
struct RadixPayload {
  const uint32_t* p1_in = nullptr;
  uint32_t* p1_out = nullptr;
  const uint32_t* p2_in = nullptr;
  uint32_t* p2_out = nullptr;
};
int radix_pass_pairs(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* keys_out,
                     uint32_t* vals_out, const uint32_t* n_dev, uint64_t n_cap, uint32_t shift,
                     uint32_t dbits, void* tmp, hipStream_t stream, const uint32_t** totals,
                     const RadixPayload& pl = RadixPayload{});
size_t radix_pass_tmp_bytes(uint64_t n_cap);

// C[M x N] = sum of `splits` partial slabs [M x N] (ld N, `stride` floats
// apart) in a fixed order (deterministic; gemm.hip).
int sum_splits(hipStream_t st, const float* part, int splits, uint64_t stride, int M, int N,
               float* C, uint64_t ldc);

// fp32-accurate GEMMs on the bf16 matrix cores (gemm3.hip, NTS_GEMM_SPLIT3)
bool gemm3_nn_ok(int M, int N, int K, const float* A, uint64_t lda);
bool gemm3_tn_ok(int M, int N, int K);
int gemm3_nn(nts_hip_ctx* ctx, bool epi, int M, int N, int K, const float* A, uint64_t lda,
             const uint32_t* amap, const float* B, uint64_t ldb, float* C, uint64_t ldc,
             uint32_t keep_threshold, float scale, uint64_t seed, uint64_t offset);
int gemm3_tn(nts_hip_ctx* ctx, int M, int N, int K, const float* A, uint64_t lda,
             const uint32_t* amap, const float* B, uint64_t ldb, const float* X, uint64_t ldx,
             float bscale, float* C, uint64_t ldc);
// the same arithmetic over whole gathered feature rows streamed into LDS
// (gemmx3.hip): the transform-first bottom layer's GEMMs
bool x3_tn_ok(int M, int N, int K, const float* A, uint64_t lda, const float* B, uint64_t ldb,
              const float* Xm = nullptr, uint64_t ldxm = 0);
bool x3_tn_bm_ok(int M, int N, int K, const float* A, uint64_t lda, const float* B, uint64_t ldb,
                 const float* Xm, uint64_t ldxm);
// Xm != NULL: B = B ⊙ [Xm > 0] · bscale (dense rows, M <= 128)
int x3_tn(nts_hip_ctx* ctx, int M, int N, int K, const float* A, uint64_t lda, const uint32_t* amap,
          const float* B, uint64_t ldb, float* C, uint64_t ldc, const float* Xm = nullptr,
          uint64_t ldxm = 0, float bscale = 1.f);
bool x3_nn_ok(int M, int N, int K, const float* A, uint64_t lda);
bool x3_nn7_ok(int M, int N, int K, const float* A, uint64_t lda);
bool x3_nnk_ok(int M, int N, int K, const float* A, uint64_t lda);  // gemm3.hip: K <= 128, dense
int x3_nn(nts_hip_ctx* ctx, bool epi, int M, int N, int K, const float* A, uint64_t lda,
          const uint32_t* amap, const char* bimg, float* C, uint64_t ldc, uint32_t keep_threshold,
          float scale, uint64_t seed, uint64_t offset);
}  // namespace nts_hip
