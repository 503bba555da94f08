// Calibration probe: fp32 MFMA issue rate with NACC independent accumulators
// per wave, operands in registers (no memory in the loop).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
template <int NACC>
__global__ __launch_bounds__(256) void k_probe(float* out, int iters, float x) {
  f32x16 acc[NACC];
  for (int t = 0; t < NACC; ++t)
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  float a = x * threadIdx.x, b = x + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 16; ++s)
#pragma unroll
      for (int t = 0; t < NACC; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[t], 0, 0, 0);
  }
  float s = 0.f;
  for (int t = 0; t < NACC; ++t)
    for (int i = 0; i < 16; ++i) s += acc[t][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
typedef float f32x4v __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ __launch_bounds__(256) void k_probe16(float* out, int iters, float x) {
  f32x4v acc[NACC];
  for (int t = 0; t < NACC; ++t)
    for (int i = 0; i < 4; ++i) acc[t][i] = 0.f;
  float a = x * threadIdx.x, b = x + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 16; ++s)
#pragma unroll
      for (int t = 0; t < NACC; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
  }
  float s = 0.f;
  for (int t = 0; t < NACC; ++t)
    for (int i = 0; i < 4; ++i) s += acc[t][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int NACC>
void run16(int blocks, float* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 800;
  hipLaunchKernelGGL(k_probe16<NACC>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_probe16<NACC>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double flops = (double)blocks * 4 * iters * 16 * NACC * 16 * 16 * 4 * 2;
  printf("16x16x4 NACC=%d blocks=%d: %.1f us  %.1f TF\n", NACC, blocks, ms * 1e3, flops / ms / 1e9);
}
template <int NACC>
void run(int blocks, float* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 200;
  hipLaunchKernelGGL(k_probe<NACC>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_probe<NACC>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double flops = (double)blocks * 4 * iters * 16 * NACC * 32 * 32 * 2 * 2;
  printf("NACC=%d blocks=%d: %.1f us  %.1f TF\n", NACC, blocks, ms * 1e3, flops / ms / 1e9);
}
int main() {
  float* out; hipMalloc(&out, 1 << 26);
  for (int b : {256, 512, 1024}) { run<1>(b, out); run<2>(b, out); run<4>(b, out); }
  for (int b : {256, 512, 1024}) { run16<2>(b, out); run16<4>(b, out); run16<8>(b, out); }
  return 0;
}
