// Calibration probe for the GEMM main loop: the k-step structure of
// csrc/gemm.hip (LDS A/B tiles, 2 accumulators per wave) with parts switched
// off, to see which part keeps the MFMA pipe idle.  Results are NOT a GEMM.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kAP = 36, kBM = 64, kBN = 128, kBK = 32;
template <bool GLOBAL, bool BARRIER, bool LDSREAD, bool STORE>
__global__ __launch_bounds__(256, 3) void k_probe(const float* __restrict__ A, const float* __restrict__ B,
                                                  float* out, int steps, int lda) {
  __shared__ float sa[2][kBM * kAP];
  __shared__ float sb[2][kBK * kBN];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int wr = 32 * (w & 1), wc = w >> 1;
  f32x16 acc[2];
  for (int t = 0; t < 2; ++t)
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  const int tid = threadIdx.x;
  const float* abase = A + ((size_t)blockIdx.x * 64 + tid / 16) * lda + (tid % 16) * 2;
  const float* bbase = B + (tid & 31);
  float av[8], bv[16];
  for (int i = 0; i < 8; ++i) av[i] = 0.f;
  for (int i = 0; i < 16; ++i) bv[i] = 0.f;
  for (int j = 0; j < steps; ++j) {
    const int cur = j & 1;
    if (GLOBAL) {
      const int k0 = (j % 18) * kBK;
      for (int p = 0; p < 4; ++p) {
        const float2 x = *reinterpret_cast<const float2*>(abase + (size_t)16 * p * lda + k0);
        av[2 * p] = x.x; av[2 * p + 1] = x.y;
      }
      for (int p = 0; p < 4; ++p)
        for (int t = 0; t < 4; ++t) bv[4 * p + t] = bbase[(size_t)(k0 + (tid >> 5) + 8 * p) * 128 + 32 * t];
    }
    __builtin_amdgcn_sched_barrier(0);
    float a[16];
    if (LDSREAD) {
      const float4* ap = reinterpret_cast<const float4*>(sa[cur] + (wr + r) * kAP + 16 * h);
      for (int q = 0; q < 4; ++q) {
        const float4 x = ap[q];
        a[4 * q] = x.x; a[4 * q + 1] = x.y; a[4 * q + 2] = x.z; a[4 * q + 3] = x.w;
      }
      const float2* bp = reinterpret_cast<const float2*>(sb[cur] + (16 * h) * kBN + 64 * wc) + r;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const float2 b = bp[s * (kBN / 2)];
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b.x, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b.y, acc[1], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32((float)s, 1.f, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32((float)s, 2.f, acc[1], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (STORE) {
      for (int p = 0; p < 4; ++p)
        *reinterpret_cast<float2*>(sa[cur ^ 1] + (tid / 16 + 16 * p) * kAP + (tid % 16) * 2) =
            make_float2(av[2 * p], av[2 * p + 1]);
      for (int p = 0; p < 4; ++p) {
        float* row = sb[cur ^ 1] + ((tid >> 5) + 8 * p) * kBN;
        *reinterpret_cast<float2*>(row + 2 * r) = make_float2(bv[4 * p], bv[4 * p + 1]);
        *reinterpret_cast<float2*>(row + 64 + 2 * r) = make_float2(bv[4 * p + 2], bv[4 * p + 3]);
      }
    }
    if (BARRIER) __syncthreads();
  }
  float s = 0.f;
  for (int t = 0; t < 2; ++t)
    for (int i = 0; i < 16; ++i) s += acc[t][i];
  out[blockIdx.x * 256 + tid] = s;
}
template <bool G, bool Bar, bool L, bool S>
void run(const char* name, const float* A, const float* B, float* out, int blocks, int steps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((k_probe<G, Bar, L, S>), dim3(blocks), dim3(256), 0, 0, A, B, out, steps, 602);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((k_probe<G, Bar, L, S>), dim3(blocks), dim3(256), 0, 0, A, B, out, steps, 602);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  double flops = (double)blocks * 64 * 128 * 32 * 2 * steps;
  printf("%-34s blocks=%d: %8.1f us %6.1f TF\n", name, blocks, ms * 1e3, flops / ms / 1e9);
}
int main() {
  float *A, *B, *out;
  (void)hipMalloc(&A, (size_t)2048 * 64 * 602 * 4);
  (void)hipMalloc(&B, (size_t)602 * 128 * 4);
  (void)hipMalloc(&out, (size_t)4096 * 256 * 4);
  (void)hipMemset(A, 0, (size_t)2048 * 64 * 602 * 4);
  (void)hipMemset(B, 0, (size_t)602 * 128 * 4);
  for (int blocks : {768, 1536}) {
    run<false, false, false, false>("mfma only", A, B, out, blocks, 180);
    run<false, false, true, false>("+lds reads", A, B, out, blocks, 180);
    run<false, true, true, false>("+lds reads +barrier", A, B, out, blocks, 180);
    run<false, true, true, true>("+lds reads +barrier +stores", A, B, out, blocks, 180);
    run<true, true, true, true>("full (global loads)", A, B, out, blocks, 180);
    run<true, false, true, true>("full minus barrier", A, B, out, blocks, 180);
  }
  return 0;
}
