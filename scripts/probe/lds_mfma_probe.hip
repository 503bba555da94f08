// Calibration probe: the k_gemm_wres inner loop in isolation.
//  mode 0: 16x16x4 MFMAs, A operands in registers, B operands by ds_read_b128 from LDS
//  mode 1: mode 0 + per-k-block global loads of A (2 row tiles x 32 B per lane, one block ahead)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { if ((x) != hipSuccess) { printf("err %s\n", #x); return 1; } } while (0)
template <int MODE>
__global__ __launch_bounds__(1024) void k(float* out, const float* A, int nkb, int lda) {
  __shared__ __attribute__((aligned(16))) float sB[608 * 64];
  for (int e = threadIdx.x; e < 608 * 64; e += 1024) sB[e] = (float)(e & 7);
  __syncthreads();
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4, wv = threadIdx.x >> 6;
  f32x4 acc[2][4];
  for (int r = 0; r < 2; ++r) for (int j = 0; j < 4; ++j) acc[r][j] = f32x4{0, 0, 0, 0};
  float a[2][8], an[2][8];
  const float* arow[2];
  for (int r = 0; r < 2; ++r) {
    arow[r] = A + (size_t)((blockIdx.x * 16 + wv) * 32 + 16 * r + i) * lda + 8 * g;
    for (int e = 0; e < 8; ++e) a[r][e] = arow[r][e];
  }
  for (int rep = 0; rep < 3; ++rep)
  for (int kb = 0; kb < nkb; ++kb) {
    if (MODE == 1) {
      const int kn = (kb + 1) % nkb;
      for (int r = 0; r < 2; ++r)
        for (int q = 0; q < 4; ++q) {
          const float2 x = reinterpret_cast<const float2*>(arow[r] + 32 * kn)[q];
          an[r][2 * q] = x.x; an[r][2 * q + 1] = x.y;
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    const float* bb = sB + (32 * (kb % 19) + 8 * g) * 64 + 4 * i;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(bb + t * 64);
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          acc[r][jj] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[r][t], b[jj], acc[r][jj], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (MODE == 1)
      for (int r = 0; r < 2; ++r) for (int e = 0; e < 8; ++e) a[r][e] = an[r][e];
  }
  float s = 0;
  for (int r = 0; r < 2; ++r) for (int j = 0; j < 4; ++j) for (int v = 0; v < 4; ++v) s += acc[r][j][v];
  out[blockIdx.x * 1024 + threadIdx.x] = s;
}
template <int MODE>
int run(const float* A, float* out) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int nkb = 19, blocks = 256;
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(1024), 0, 0, out, A, nkb, 608);
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(1024), 0, 0, out, A, nkb, 608);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  const double mf = 3.0 * blocks * 16 * nkb * 8 * 8;  // MFMAs
  printf("mode %d: %.1f us  %.1f TF\n", MODE, ms * 1e3, mf * 16 * 16 * 4 * 2 / ms / 1e9);
  return 0;
}
int main() {
  float *A, *out;
  CK(hipMalloc(&A, (size_t)256 * 16 * 32 * 608 * 4));
  CK(hipMemset(A, 0, (size_t)256 * 16 * 32 * 608 * 4));
  CK(hipMalloc(&out, 1 << 24));
  if (run<0>(A, out) || run<1>(A, out) || run<0>(A, out) || run<1>(A, out)) return 1;
  return 0;
}
