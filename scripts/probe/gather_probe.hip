// Row-gather probe (not part of the library): the ceiling of the transform-
// first bottom aggregation's access pattern — 1.36 M random 512-byte rows
// (128 floats) read from a 117 MB table (228,616 rows: H = X[src] W at C2),
// each row summed into a per-destination accumulator (25 rows per dst in CSC
// order, the sampled hop-1 layer), no weights, no stores beyond one row per
// dst.  Forms:
//   reg_u<U>  one 32-lane half-wave per dst (16 B per lane = one row per
//             load), U rows in flight per half-wave (the library's
//             k_spmm_gather shape: LPD 32, float4)
//   lds       LDS DMA of whole rows (global_load_lds_dwordx4, one 512-byte
//             piece per half-wave instruction) into a per-wave ring, DEPTH
//             pieces in flight, summed from LDS
// Build: hipcc -O3 --offload-arch=gfx950 scripts/probe/gather_probe.hip -o scripts/probe/gather_probe
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

constexpr int kF = 128;  // floats per row

template <int U>
__global__ __launch_bounds__(256) void k_reg(const float4* __restrict__ H, const uint32_t* __restrict__ idx,
                                             uint32_t ndst, uint32_t fan, float4* __restrict__ out) {
  const int lane = threadIdx.x & 31;
  const uint32_t d = blockIdx.x * 8 + (threadIdx.x >> 5);
  if (d >= ndst) return;
  const uint32_t* ix = idx + (uint64_t)d * fan;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (uint32_t e = 0; e < fan; e += U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t r = ix[min(e + u, fan - 1)];
      v[u] = H[(uint64_t)r * (kF / 4) + lane];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (e + u < fan) {
        acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
      }
  }
  out[(uint64_t)d * (kF / 4) + lane] = acc;
}

__device__ __forceinline__ void glds16(const void* src, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}

// one wave per dst pair (half-waves: one dst each), rows by LDS DMA: two rows
// (one per half) per 1 KiB wave-instruction, DEPTH instructions in flight
template <int DEPTH>
__global__ __launch_bounds__(256) void k_lds(const float* __restrict__ H, const uint32_t* __restrict__ idx,
                                             uint32_t ndst, uint32_t fan, float4* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char ring[];  // [4 waves][16][1024]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, half = lane >> 5, l32 = lane & 31;
  const uint32_t d = (blockIdx.x * 4 + w) * 2 + half;
  const bool ok = d < ndst;
  const uint32_t* ix = idx + (uint64_t)min(d, ndst - 1) * fan;
  const uint32_t myix = l32 < (int)fan ? ix[l32] : 0u;  // (fan <= 32: the dst's ids, one per lane)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)ring + w * 16384;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (uint32_t e = 0; e < fan + DEPTH; ++e) {
    if (e < fan) {
      const uint32_t r = __shfl(myix, (int)e, 32);
      glds16(H + (uint64_t)r * kF + 4 * l32, __builtin_amdgcn_readfirstlane(base + 1024 * (e & 15)));
    }
    if (e >= DEPTH) {
      if (e < fan) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const float4 v = *reinterpret_cast<const float4*>(ring + w * 16384 + 1024 * ((e - DEPTH) & 15) + 16 * lane);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  if (ok) out[(uint64_t)d * (kF / 4) + l32] = acc;
}

int main(int argc, char** argv) {
  const uint32_t S = 228616, ndst = 54400, fan = 25;  // ~1.36 M edges
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  float* H;
  float4* out;
  uint32_t* idx;
  CK(hipMalloc(&H, (size_t)S * kF * 4));
  CK(hipMemset(H, 0, (size_t)S * kF * 4));
  CK(hipMalloc(&out, (size_t)ndst * kF * 4));
  std::vector<uint32_t> h((size_t)ndst * fan);
  std::mt19937 g(3);
  for (auto& x : h) x = g() % S;
  CK(hipMalloc(&idx, h.size() * 4));
  CK(hipMemcpy(idx, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double rows_bytes = (double)h.size() * kF * 4;
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
    printf("{\"probe\": \"%s\", \"us\": %.1f, \"rows_TBps\": %.2f}\n", name, us, rows_bytes / us / 1e6);
    fflush(stdout);
  };
  const uint32_t greg = (ndst + 7) / 8, glds = (ndst + 7) / 8;
  run("reg_u4", [&] { hipLaunchKernelGGL(k_reg<4>, dim3(greg), dim3(256), 0, 0, (const float4*)H, idx, ndst, fan, out); });
  run("reg_u8", [&] { hipLaunchKernelGGL(k_reg<8>, dim3(greg), dim3(256), 0, 0, (const float4*)H, idx, ndst, fan, out); });
  run("reg_u13", [&] { hipLaunchKernelGGL(k_reg<13>, dim3(greg), dim3(256), 0, 0, (const float4*)H, idx, ndst, fan, out); });
  run("reg_u25", [&] { hipLaunchKernelGGL(k_reg<25>, dim3(greg), dim3(256), 0, 0, (const float4*)H, idx, ndst, fan, out); });
  run("lds_d8", [&] { hipLaunchKernelGGL(k_lds<8>, dim3(glds), dim3(256), 65536, 0, (const float*)H, idx, ndst, fan, out); });
  run("lds_d12", [&] { hipLaunchKernelGGL(k_lds<12>, dim3(glds), dim3(256), 65536, 0, (const float*)H, idx, ndst, fan, out); });
  CK(hipGetLastError());
  return 0;
}
