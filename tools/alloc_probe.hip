// alloc_probe.hip — does HOW the bank's memory is allocated change the ring
// round's HBM rate?  The r03 "slow allocation" (the same kernel 4-8 % slower
// in some processes) points at the physical placement of the buffers.  This
// times dol_mix_ring_f32 at 8192 x 2^20 (ld = 2^20 + 1024, the bench's
// geometry) on X / Y allocated three ways, alternating A/B/C blocks:
//   0 hipMalloc (what torch's caching allocator does for a 32 GiB block)
//   1 hipExtMallocWithFlags(hipDeviceMallocContiguous)
//   2 virtual memory: one hipMemCreate physical allocation per buffer, mapped
//     with hipMemMap (one chunk = the driver's largest fragments)
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/alloc_probe tools/alloc_probe.hip \
//          -I include -L distributed-optimization-and-learning_amd/dolhip -ldol_hip \
//          -Wl,-rpath,'$ORIGIN/../distributed-optimization-and-learning_amd/dolhip'
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "dol_hip.h"

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                        \
    }                                                                                 \
  } while (0)

__global__ void fill_kernel(float* p, size_t n, float v) {
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    p[i] = v + float(i & 1023) * 1e-3f;
}

struct Buf {
  float* p = nullptr;
  int mode = 0;
  size_t bytes = 0;
  hipMemGenericAllocationHandle_t h{};
};

static bool alloc(Buf& b, size_t bytes, int mode) {
  b.mode = mode;
  b.bytes = bytes;
  if (mode == 0) return hipMalloc(reinterpret_cast<void**>(&b.p), bytes) == hipSuccess;
  if (mode == 1) return hipExtMallocWithFlags(reinterpret_cast<void**>(&b.p), bytes, hipDeviceMallocContiguous) == hipSuccess;
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gran = 0;
  if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended) != hipSuccess) return false;
  b.bytes = (bytes + gran - 1) / gran * gran;
  if (hipMemCreate(&b.h, b.bytes, &prop, 0) != hipSuccess) return false;
  void* va = nullptr;
  if (hipMemAddressReserve(&va, b.bytes, 0, nullptr, 0) != hipSuccess) return false;
  if (hipMemMap(va, b.bytes, 0, b.h, 0) != hipSuccess) return false;
  hipMemAccessDesc acc{};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  if (hipMemSetAccess(va, b.bytes, &acc, 1) != hipSuccess) return false;
  b.p = static_cast<float*>(va);
  return true;
}

static void release(Buf& b) {
  if (!b.p) return;
  if (b.mode < 2) {
    CHECK(hipFree(b.p));
  } else {
    CHECK(hipMemUnmap(b.p, b.bytes));
    CHECK(hipMemAddressFree(b.p, b.bytes));
    CHECK(hipMemRelease(b.h));
  }
  b.p = nullptr;
}

int main(int argc, char** argv) {
  const int N = 8192;
  const int64_t P = 1 << 20, ld = P + 1024;
  const size_t bytes = size_t(N) * ld * 4;
  const int reps = 20, blocks = argc > 1 ? atoi(argv[1]) : 2;
  float *wp, *wn;
  CHECK(hipMalloc(&wp, N * 4));
  CHECK(hipMalloc(&wn, N * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(64), dim3(256), 0, 0, wp, size_t(N), 0.5f);
  hipLaunchKernelGGL(fill_kernel, dim3(64), dim3(256), 0, 0, wn, size_t(N), 0.25f);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* names[] = {"hipMalloc", "hipExtMallocWithFlags(Contiguous)", "hipMemCreate+hipMemMap"};
  for (int blk = 0; blk < blocks; ++blk) {
    for (int mode = 0; mode < 3; ++mode) {
      Buf X, Y;
      if (!alloc(X, bytes, mode) || !alloc(Y, bytes, mode)) {
        printf("{\"block\": %d, \"mode\": \"%s\", \"error\": \"allocation failed\"}\n", blk, names[mode]);
        (void)hipGetLastError();
        release(X);
        release(Y);
        continue;
      }
      hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, X.p, bytes / 4, 1.0f);
      hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, Y.p, bytes / 4, 0.0f);
      for (int w = 0; w < 3; ++w)
        if (dol_mix_ring_f32(X.p, ld, Y.p, ld, N, P, nullptr, nullptr, wp, wn, 0)) {
          fprintf(stderr, "dol_mix_ring_f32: %s\n", dol_last_error());
          return 2;
        }
      std::vector<float> ms(reps);
      for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(e0, 0));
        (void)dol_mix_ring_f32(X.p, ld, Y.p, ld, N, P, nullptr, nullptr, wp, wn, 0);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms[r], e0, e1));
      }
      double mean = 0, best = 1e30;
      for (float m : ms) {
        mean += m / reps;
        best = m < best ? m : best;
      }
      printf("{\"block\": %d, \"mode\": \"%s\", \"ring_ms_mean\": %.4f, \"ring_ms_best\": %.4f, \"TBps_mean\": %.3f, "
             "\"x\": \"%p\", \"y\": \"%p\"}\n",
             blk, names[mode], mean, best, 2.0 * N * P * 4 / (mean * 1e-3) / 1e12, (void*)X.p, (void*)Y.p);
      fflush(stdout);
      release(X);
      release(Y);
    }
  }
  return 0;
}
