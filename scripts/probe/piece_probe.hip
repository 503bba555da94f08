// Piece-size probe (not part of the library): a pass over the C2 feature
// table (fp32 rows, 2,560-B pitch, 228,616 sorted row ids out of 232,965, one
// contiguous id range per block, one 512-thread block per CU) read by LDS DMA
// in k-chunks: a block takes G rows at a time and, for each P-byte slice of
// those rows (P = 2,560: whole rows), streams G x P bytes as 1-KiB
// wave-instructions into an LDS ring, DEPTH pieces in flight per wave, no
// consumer.  Question answered: how much of the whole-row streaming rate do
// row pieces of 128 / 256 / 512 / 1,280 B keep (the k-sliced GEMM tilings).
// Build: hipcc -O3 --offload-arch=gfx950 scripts/probe/piece_probe.hip -o scripts/probe/piece_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));      \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int kPitch = 2560;
constexpr int kThreads = 512;

__device__ __forceinline__ void glds16(const void* src, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}

template <int G, int P, int DEPTH>
__global__ __launch_bounds__(kThreads, 1) void k_piece(const char* __restrict__ Q, const uint32_t* ids,
                                                       uint32_t M, uint32_t chunk, uint32_t* sink) {
  extern __shared__ __attribute__((aligned(16))) char ring[];
  uint32_t* sid = reinterpret_cast<uint32_t*>(ring + 131072);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t r0 = blockIdx.x * chunk, r1 = min(M, r0 + chunk);
  for (uint32_t r = r0 + threadIdx.x; r < r1; r += kThreads) sid[r - r0] = ids[r];
  __syncthreads();
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)ring + w * 16384;
  constexpr int kPieces = G * P / 1024;  // 1-KiB wave-instructions per (group, slice)
  constexpr int kSlices = kPitch / P;
  int slot = 0;
  for (uint32_t g0 = r0; g0 < r1; g0 += G) {
    for (int c = 0; c < kSlices; ++c) {
      for (int p = w; p < kPieces; p += 8) {
        const int o = 1024 * p + 16 * lane;
        const int row = o / P, col = o - row * P;
        const uint32_t r = min(g0 + row, r1 - 1);
        const char* src = Q + (uint64_t)sid[r - r0] * kPitch + c * P + col;
        const uint32_t dst = __builtin_amdgcn_readfirstlane(base + 1024 * (slot & 15));
        glds16(src, dst);
        ++slot;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH) : "memory");
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (reinterpret_cast<uint32_t*>(ring)[threadIdx.x] == 0x12345678u) sink[0] = 1;
}

int main(int argc, char** argv) {
  const uint32_t V = 232965, M = 228616;
  const int iters = argc > 1 ? atoi(argv[1]) : 10;
  char* Q;
  CK(hipMalloc(&Q, (size_t)V * kPitch));
  CK(hipMemset(Q, 1, (size_t)V * kPitch));
  std::vector<uint32_t> h(V);
  for (uint32_t i = 0; i < V; ++i) h[i] = i;
  std::mt19937 g(1);
  std::shuffle(h.begin(), h.end(), g);
  h.resize(M);
  std::sort(h.begin(), h.end());
  uint32_t *ids, *sink;
  CK(hipMalloc(&ids, M * 4));
  CK(hipMalloc(&sink, 4));
  CK(hipMemcpy(ids, h.data(), M * 4, hipMemcpyHostToDevice));
  const uint32_t blocks = 256, chunk = (M + blocks - 1) / blocks;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double bytes = (double)M * kPitch;
  auto run = [&](const char* name, auto kern) {
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 131072 + 4096));
    auto launch = [&] {
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(kThreads), 131072 + 4096, 0, Q, ids, M, chunk, sink);
    };
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / iters;
    printf("{\"probe\": \"%s\", \"us\": %.1f, \"TBps\": %.2f}\n", name, us, bytes / us / 1e6);
    fflush(stdout);
  };
  run("G16_P2560", k_piece<16, 2560, 12>);
  run("G32_P1280", k_piece<32, 1280, 12>);
  run("G64_P512", k_piece<64, 512, 12>);
  run("G128_P512", k_piece<128, 512, 12>);
  run("G64_P256", k_piece<64, 256, 12>);
  run("G128_P256", k_piece<128, 256, 12>);
  run("G128_P128", k_piece<128, 128, 12>);
  run("G256_P128", k_piece<256, 128, 12>);
  run("G64_P512_d15", k_piece<64, 512, 15>);
  run("G16_P2560_d15", k_piece<16, 2560, 15>);
  CK(hipGetLastError());
  return 0;
}
