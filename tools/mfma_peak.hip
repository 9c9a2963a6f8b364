// mfma_peak.hip — sustained fp32-MFMA ceiling on this box: every wave runs
// independent v_mfma_f32_32x32x2_f32 chains with no memory traffic (operands
// in registers), grid = 8 waves per CU x 256 CUs.  Prices the dense mix
// (dense_mix_mfma_kernel) against what the matrix cores actually sustain,
// as copy_kernel prices the streaming kernels against HBM.
//   hipcc --offload-arch=gfx950 -O3 -o mfma_peak mfma_peak.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <int CHAINS>
__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters, float a, float b) {
  f32x16 acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  float x = a + threadIdx.x * 1e-7f, y = b;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc[c], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;  // keeps the chains live
}

int main() {
  int dev = 0, ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int blocks = ncu * 2, iters = 20000;  // 2 x 256 threads = 8 waves per CU
  float* out;
  CHECK(hipMalloc(&out, size_t(blocks) * 256 * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(256), 0, 0, out, 100, 1.0f, 1e-3f);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f, 1e-3f);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double flops = double(blocks) * 4 /*waves*/ * iters * 4 /*chains*/ * 2.0 * 32 * 32 * 2;
  printf("CUs %d  sustained fp32 MFMA (v_mfma_f32_32x32x2_f32): %.1f TFLOP/s  (%.3f ms)\n", ncu, flops / (ms / 1e3) / 1e12, ms);
  return 0;
}
