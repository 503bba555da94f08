// Context, error plumbing and scratch arena of libnts_hip.so.
// Replaces the reference's Cuda_Stream object lifetime (cuda/ntsCUDAGraphOP.cu:201-212)
// and its per-subgraph GPU arena (core/FullyRepGraph.hpp:113-121).
#include <cstdarg>
#include <vector>

#include "common.hpp"

namespace nts_hip {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int ensure_vertices(nts_hip_ctx* ctx, uint64_t n_vertices) {
  if (n_vertices <= ctx->v_cap) return NTS_OK;
  NTS_HIP_TRY(hipStreamSynchronize(ctx->stream));
  if (ctx->marks) NTS_HIP_TRY(hipFree(ctx->marks));
  if (ctx->src_index) NTS_HIP_TRY(hipFree(ctx->src_index));
  ctx->marks = nullptr;
  ctx->src_index = nullptr;
  // marks are scanned 16 bytes per lane: pad to a multiple of 4096.
  uint64_t padded = (n_vertices + 4095) / 4096 * 4096;
  NTS_HIP_TRY(hipMalloc(&ctx->marks, padded));
  // zeroed on the context's stream (a plain hipMemset goes to the NULL
  // stream, which a non-blocking stream does not wait for) and waited for
  NTS_HIP_TRY(hipMemsetAsync(ctx->marks, 0, padded, ctx->stream));
  NTS_HIP_TRY(hipStreamSynchronize(ctx->stream));
  NTS_HIP_TRY(hipMalloc(&ctx->src_index, n_vertices * sizeof(uint32_t)));
  ctx->v_cap = n_vertices;
  return NTS_OK;
}

int ensure_scratch(nts_hip_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->scratch_bytes) return NTS_OK;
  // Growing the arena must not race with in-flight kernels using it.
  NTS_HIP_TRY(hipStreamSynchronize(ctx->stream));
  if (ctx->scratch) NTS_HIP_TRY(hipFree(ctx->scratch));
  ctx->scratch = nullptr;
  size_t b = bytes + bytes / 4;
  NTS_HIP_TRY(hipMalloc(&ctx->scratch, b));
  ctx->scratch_bytes = b;
  return NTS_OK;
}

bool launch_trace() {
  static const bool on = [] {
    const char* e = getenv("NTS_LAUNCH_TRACE");
    return e && e[0] == '1';
  }();
  return on;
}
void launch_trace_sync(const char* file, int line) {
  fprintf(stderr, "[launch] %s:%d\n", file, line);
  fflush(stderr);
  (void)hipDeviceSynchronize();
  fprintf(stderr, "[done] %s:%d\n", file, line);
  fflush(stderr);
}

// Tile states of the single-pass scan: zeroed once (epoch 0 is never issued).
int ensure_scan_state(nts_hip_ctx* ctx, uint64_t elems) {
  if (elems < ctx->scan_state_elems) return NTS_OK;  // the last word: the ticket counter
  NTS_HIP_TRY(hipStreamSynchronize(ctx->stream));
  if (ctx->scan_state) NTS_HIP_TRY(hipFree(ctx->scan_state));
  ctx->scan_state = nullptr;
  const uint64_t n = elems + elems / 4 + 64;
  NTS_HIP_TRY(hipMalloc(&ctx->scan_state, n * sizeof(uint64_t)));
  // zeroed on the context's stream and waited for: the NULL stream's
  // hipMemset is not ordered before the next kernel on a non-blocking stream,
  // and a tile word or the ticket counter still holding the old allocation's
  // bytes when the first look-back kernel runs hangs it (a stale ticket count
  // sends tiles past the grid)
  NTS_HIP_TRY(hipMemsetAsync(ctx->scan_state, 0, n * sizeof(uint64_t), ctx->stream));
  NTS_HIP_TRY(hipStreamSynchronize(ctx->stream));
  ctx->scan_state_elems = n;
  return NTS_OK;
}

// std::mt19937 seeding (init_genrand): sequential, done on the host.
static void mt_seed_host(uint64_t seed, uint32_t* st) {
  st[0] = (uint32_t)seed;
  for (int i = 1; i < 624; ++i)
    st[i] = 1812433253u * (st[i - 1] ^ (st[i - 1] >> 30)) + (uint32_t)i;
  st[624] = 624;  // position: next call twists
}

}  // namespace nts_hip

using namespace nts_hip;

extern "C" {

int nts_hip_abi_version(void) { return NTS_HIP_ABI_VERSION; }

const char* nts_hip_last_error(void) { return g_err; }

int nts_hip_ctx_create(nts_hip_ctx** out, int device, void* stream, uint64_t seed) {
  NTS_CHECK_ARG(out != nullptr, "out is NULL");
  *out = nullptr;
  NTS_HIP_TRY(hipSetDevice(device));
  nts_hip_ctx* ctx = new nts_hip_ctx();
  ctx->device = device;
  ctx->seed = seed;
  // NULL is HIP's legacy default stream, used as-is (ordered with every other
  // blocking stream of the device, like torch's default stream).
  ctx->stream = (hipStream_t)stream;
  hipError_t e = hipMalloc(&ctx->mt_state, 625 * sizeof(uint32_t));
  if (e != hipSuccess) {
    set_error("hipMalloc(mt_state): %s", hipGetErrorString(e));
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return NTS_ERR_HIP;
  }
  *out = ctx;
  return nts_hip_rng_seed(ctx, seed);
}

int nts_hip_ctx_destroy(nts_hip_ctx* ctx) {
  if (!ctx) return NTS_OK;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  if (ctx->marks) (void)hipFree(ctx->marks);
  if (ctx->src_index) (void)hipFree(ctx->src_index);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->mt_state) (void)hipFree(ctx->mt_state);
  mt_ring_free(ctx);
  if (ctx->scan_state) (void)hipFree(ctx->scan_state);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return NTS_OK;
}

int nts_hip_ctx_set_stream(nts_hip_ctx* ctx, void* stream) {
  NTS_CHECK_ARG(ctx && stream, "ctx/stream is NULL");
  if (ctx->own_stream) {
    NTS_HIP_TRY(hipStreamSynchronize(ctx->stream));
    NTS_HIP_TRY(hipStreamDestroy(ctx->stream));
    ctx->own_stream = false;
  }
  ctx->stream = (hipStream_t)stream;
  return NTS_OK;
}

void* nts_hip_ctx_get_stream(nts_hip_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int nts_hip_ctx_set_gemm_mode(nts_hip_ctx* ctx, int mode) {
  NTS_CHECK_ARG(ctx, "ctx is NULL");
  NTS_CHECK_ARG(mode == NTS_GEMM_F32 || mode == NTS_GEMM_SPLIT3 || mode == NTS_GEMM_SPLIT3_ALL,
                "unknown GEMM mode");
  ctx->gemm_mode = mode;
  return NTS_OK;
}

int nts_hip_ctx_get_gemm_mode(nts_hip_ctx* ctx) { return ctx ? ctx->gemm_mode : NTS_GEMM_F32; }

int nts_hip_ctx_reserve(nts_hip_ctx* ctx, uint64_t n_vertices, uint64_t max_items) {
  NTS_CHECK_ARG(ctx, "ctx is NULL");
  NTS_HIP_TRY(hipSetDevice(ctx->device));
  NTS_RET(ensure_vertices(ctx, n_vertices));
  uint64_t items = max_items > n_vertices ? max_items : n_vertices;
  size_t need = radix_tmp_bytes(items);
  size_t s64 = scan_tmp_elems<uint64_t>(items + 1) * sizeof(uint64_t) + 256;
  if (s64 > need) need = s64;
  // look-back state: the largest single-pass scan is the count scan (1,024-item
  // tiles over a layer's dsts, count_scan); the frontier compaction uses at
  // most 256 tiles and scan1_exclusive 4,096-item tiles (the
  // radix sort's digit scans need no state since round 5)
  NTS_RET(ensure_scan_state(ctx, (items / 1024 + 2 + 63) / 64 * 64));
  return ensure_scratch(ctx, need);
}

int nts_hip_rng_seed(nts_hip_ctx* ctx, uint64_t seed) {
  NTS_CHECK_ARG(ctx, "ctx is NULL");
  std::vector<uint32_t> st(625);
  mt_seed_host(seed, st.data());
  ctx->seed = seed;
  // Synchronous copy from pageable memory is safe w.r.t. the host vector's
  // lifetime; order it after prior work on the stream first.
  NTS_HIP_TRY(hipStreamSynchronize(ctx->stream));
  NTS_HIP_TRY(hipMemcpy(ctx->mt_state, st.data(), 625 * sizeof(uint32_t),
                        hipMemcpyHostToDevice));
  return mt_ring_reset(ctx);
}

int nts_hip_rng_state(nts_hip_ctx* ctx, uint32_t* host_state625) {
  NTS_CHECK_ARG(ctx && host_state625, "NULL argument");
  NTS_HIP_TRY(hipStreamSynchronize(ctx->stream));
  NTS_HIP_TRY(hipMemcpy(host_state625, ctx->mt_state, 625 * sizeof(uint32_t),
                        hipMemcpyDeviceToHost));
  return NTS_OK;
}

}  // extern "C"
