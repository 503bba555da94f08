// Row-access-order probe (not part of the library): the A stream of the
// row-gathered NN GEMM (k_x3_nn7) without MFMAs — 256 blocks x 4 waves, each
// wave 7 tiles x 16 sorted rows of the C2 feature table (2,560-B pitch) per
// round, every float of the first 608 of each row read once into registers —
// in four orders:
//   KB = 1  : k-step outer (19 steps of 128 B per row), tile inner: each row
//             is revisited once per k-step (k_x3_nn7's order);
//   KB = 2/4: blocks of KB k-steps outer, tile inner, each tile's rows read
//             KB x 128 contiguous bytes at once;
//   KB = 19 : tile outer, whole rows (608 floats) per tile.
// Loads are plain global_load_dwordx4 (the kernel's form), DEPTH tiles in
// flight per wave.  Question: does the DRAM row-buffer locality of the
// k-outer order cost the NN its A stream?
// Build: hipcc -O3 --offload-arch=gfx950 scripts/probe/rowpat_probe.hip -o scripts/probe/rowpat_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int kPitch = 640;  // floats
constexpr int kSteps = 19;   // 32-float k-steps of a 602 (608) float row
constexpr int RT = 7;

template <int KB>
__global__ __launch_bounds__(256, 1) void k_rowpat(const float* __restrict__ X, const uint32_t* __restrict__ ids,
                                                 int M, int rounds, float* sink) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int T = (M + 15) / 16;
  const int64_t Wn = (int64_t)gridDim.x * 4, gw = (int64_t)blockIdx.x * 4 + wv;
  const int t_lo = (int)(gw * T / Wn), t_hi = (int)((gw + 1) * T / Wn);
  float acc = 0.f;
  for (int rd = 0; rd < rounds; ++rd) {
    const float* ptr[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      int t = min(t_lo + RT * rd + rt, max(t_hi, t_lo + 1) - 1);
      t = min(t, T - 1);
      int r = min(t * 16 + i, M - 1);
      ptr[rt] = X + (uint64_t)ids[r] * kPitch + 8 * q;
    }
    if constexpr (KB < kSteps) {
      // one KB-block of every tile in flight (the kernel keeps a step's 7)
      for (int s0 = 0; s0 < kSteps; s0 += KB) {
        float4 v[RT][2 * KB];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int k = 0; k < KB; ++k) {
            const int s = min(s0 + k, kSteps - 1);
            v[rt][2 * k] = *reinterpret_cast<const float4*>(ptr[rt] + 32 * s);
            v[rt][2 * k + 1] = *reinterpret_cast<const float4*>(ptr[rt] + 32 * s + 4);
          }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int k = 0; k < 2 * KB; ++k) acc += v[rt][k].x + v[rt][k].y + v[rt][k].z + v[rt][k].w;
      }
    } else {
      // whole rows, two tiles in flight
#pragma unroll
      for (int r0 = 0; r0 < RT; r0 += 2) {
        float4 v[2][2 * kSteps];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int s = 0; s < kSteps; ++s) {
            const float* p = ptr[min(r0 + u, RT - 1)];
            v[u][2 * s] = *reinterpret_cast<const float4*>(p + 32 * s);
            v[u][2 * s + 1] = *reinterpret_cast<const float4*>(p + 32 * s + 4);
          }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int k = 0; k < 2 * kSteps; ++k) acc += v[u][k].x + v[u][k].y + v[u][k].z + v[u][k].w;
      }
    }
  }
  if (acc == 1234.5f) sink[0] = acc;
}

int main(int argc, char** argv) {
  const int V = 232965, M = 228616;
  std::vector<uint32_t> ids(V);
  for (int v = 0; v < V; ++v) ids[v] = v;
  std::mt19937 gen(1);
  std::shuffle(ids.begin(), ids.end(), gen);
  ids.resize(M);
  std::sort(ids.begin(), ids.end());
  float* X;
  uint32_t* dids;
  float* sink;
  CK(hipMalloc(&X, (size_t)V * kPitch * 4));
  CK(hipMalloc(&dids, (size_t)M * 4));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(X, 0, (size_t)V * kPitch * 4));
  CK(hipMemcpy(dids, ids.data(), (size_t)M * 4, hipMemcpyHostToDevice));
  const int T = (M + 15) / 16, W = 1024;
  const int rounds = ((T + W - 1) / W + RT - 1) / RT;
  const double bytes = (double)M * 608 * 4;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](auto kern, const char* name) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, X, dids, M, rounds, sink);
    CK(hipDeviceSynchronize());
    const int it = 20;
    CK(hipEventRecord(a));
    for (int w = 0; w < it; ++w) hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, X, dids, M, rounds, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = 1e3 * ms / it;
    printf("{\"pattern\": \"%s\", \"us\": %.1f, \"TBps\": %.3f}\n", name, us, bytes / us / 1e6);
    fflush(stdout);
  };
  for (int r = 0; r < 2; ++r) {
    run(k_rowpat<1>, "kstep-outer KB=1 (128 B / row / visit)");
    run(k_rowpat<2>, "KB=2 (256 B)");
    run(k_rowpat<4>, "KB=4 (512 B)");
    run(k_rowpat<19>, "tile-outer whole rows");
  }
  return 0;
}
