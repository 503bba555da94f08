// Streaming probe (not part of the library): how fast can one pass over the
// transform-first bottom layer's planar pair table move, with the access
// pattern of k_h2_nn3 / k_h2_tn4 (sorted row ids covering ~98 % of V, 2560-B
// rows, one contiguous chunk of ids per block, one block per CU), without
// their MFMA and barrier structure:
//   reg   each wave loads whole rows into registers (global_load_dwordx4)
//   lds   LDS DMA (global_load_lds_dwordx4), 1 KiB pieces cut at rows, into an
//         LDS ring, `depth` pieces in flight per wave, no consumer
//   dense the same LDS-DMA loop over contiguous rows (no ids)
// Build: hipcc -O3 --offload-arch=gfx950 scripts/probe/stream_probe.hip -o scripts/probe/stream_probe
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

// wave w of the block takes rows w, w + 8, ... of the block's chunk
__global__ __launch_bounds__(kThreads, 1) void k_reg(const char* __restrict__ Q, const uint32_t* ids,
                                                     uint32_t M, uint32_t chunk, uint32_t* sink) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t r0 = blockIdx.x * chunk, r1 = min(M, r0 + chunk);
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint32_t r = r0 + w; r < r1; r += 16) {
    const uint32_t ida = ids[r];
    const uint32_t idb = r + 8 < r1 ? ids[r + 8] : ida;
    uint4 v[5];
#pragma unroll
    for (int q = 0; q < 2; ++q) v[q] = reinterpret_cast<const uint4*>(Q + (uint64_t)ida * kPitch + 1024 * q)[lane];
    v[2] = lane < 32 ? reinterpret_cast<const uint4*>(Q + (uint64_t)ida * kPitch + 2048)[lane] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 2; ++q) v[3 + q] = reinterpret_cast<const uint4*>(Q + (uint64_t)idb * kPitch + 1024 * q)[lane];
    uint4 t = lane < 32 ? reinterpret_cast<const uint4*>(Q + (uint64_t)idb * kPitch + 2048)[lane] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      acc.x ^= v[q].x; acc.y ^= v[q].y; acc.z ^= v[q].z; acc.w ^= v[q].w;
    }
    acc.x ^= t.x;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

// LDS DMA: wave w streams rows w, w + 8, ... (3 pieces per row) into its own
// ring of 16 KiB; at most DEPTH pieces in flight (counted vmcnt)
template <int DEPTH, bool DENSE>
__global__ __launch_bounds__(kThreads, 1) void k_lds(const char* __restrict__ Q, const uint32_t* ids,
                                                     uint32_t M, uint32_t chunk, uint32_t* sink) {
  extern __shared__ __attribute__((aligned(16))) char ring[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t r0 = blockIdx.x * chunk, r1 = min(M, r0 + chunk);
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)ring + w * 16384;
  int slot = 0;
  for (uint32_t r = r0 + w; r < r1; r += 8) {
    const uint32_t id = DENSE ? r : ids[r];
    const char* row = Q + (uint64_t)id * kPitch;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const uint32_t dst = __builtin_amdgcn_readfirstlane(base + 1024 * (slot & 15));
      if (q < 2 || lane < 32) glds16(row + 1024 * q + 16 * lane, dst);
      ++slot;
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH) : "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (reinterpret_cast<uint32_t*>(ring)[threadIdx.x] == 0x12345678u) sink[0] = 1;
}

// as k_lds, the block's row ids staged in LDS first (as k_h2_nn3 / k_h2_tn4
// do), so no row's DMA waits on a global id load
template <int DEPTH>
__global__ __launch_bounds__(kThreads, 1) void k_lds_ids(const char* __restrict__ Q, const uint32_t* ids,
                                                         uint32_t M, uint32_t chunk, uint32_t* sink) {
  extern __shared__ __attribute__((aligned(16))) char ring[];
  uint32_t* sid = reinterpret_cast<uint32_t*>(ring + 131072);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t r0 = blockIdx.x * chunk, r1 = min(M, r0 + chunk);
  for (uint32_t r = r0 + threadIdx.x; r < r1; r += kThreads) sid[r - r0] = ids[r];
  __syncthreads();
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)ring + w * 16384;
  int slot = 0;
  for (uint32_t r = r0 + w; r < r1; r += 8) {
    const uint32_t id = sid[r - r0];
    const char* row = Q + (uint64_t)id * kPitch;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const uint32_t dst = __builtin_amdgcn_readfirstlane(base + 1024 * (slot & 15));
      if (q < 2 || lane < 32) glds16(row + 1024 * q + 16 * lane, dst);
      ++slot;
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH) : "memory");
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
  auto run = [&](const char* name, auto launch) {
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
  };
  CK(hipFuncSetAttribute((const void*)k_lds<8, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)k_lds<12, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)k_lds<15, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)k_lds<12, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  run("reg", [&] { hipLaunchKernelGGL(k_reg, dim3(blocks), dim3(kThreads), 0, 0, Q, ids, M, chunk, sink); });
  run("lds_d8", [&] { hipLaunchKernelGGL((k_lds<8, false>), dim3(blocks), dim3(kThreads), 131072, 0, Q, ids, M, chunk, sink); });
  run("lds_d12", [&] { hipLaunchKernelGGL((k_lds<12, false>), dim3(blocks), dim3(kThreads), 131072, 0, Q, ids, M, chunk, sink); });
  run("lds_d15", [&] { hipLaunchKernelGGL((k_lds<15, false>), dim3(blocks), dim3(kThreads), 131072, 0, Q, ids, M, chunk, sink); });
  CK(hipFuncSetAttribute((const void*)k_lds_ids<12>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072 + 4096));
  CK(hipFuncSetAttribute((const void*)k_lds_ids<15>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072 + 4096));
  run("lds_ids_d12", [&] { hipLaunchKernelGGL((k_lds_ids<12>), dim3(blocks), dim3(kThreads), 131072 + 4096, 0, Q, ids, M, chunk, sink); });
  run("lds_ids_d15", [&] { hipLaunchKernelGGL((k_lds_ids<15>), dim3(blocks), dim3(kThreads), 131072 + 4096, 0, Q, ids, M, chunk, sink); });
  run("dense_d12", [&] { hipLaunchKernelGGL((k_lds<12, true>), dim3(blocks), dim3(kThreads), 131072, 0, Q, ids, M, chunk, sink); });
  CK(hipGetLastError());
  return 0;
}
