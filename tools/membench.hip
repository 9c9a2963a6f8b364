// membench.hip — exploration harness for HBM-streaming structure on gfx950.
// Times copy and ring-stencil variants on 2 x 32 GiB buffers (8192 x 2^20 fp32)
// with HIP events, variants interleaved over rounds in one process.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o membench membench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <string>
#include <algorithm>
#include <functional>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

template <bool NT>
__device__ __forceinline__ f4 ldf(const f4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p); else return *p;
}
template <bool NT>
__device__ __forceinline__ void stf(f4* p, f4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v;
}

// grid-stride copy, U loads in flight per lane
template <bool NTL, bool NTS, int U>
__global__ __launch_bounds__(256) void copy_gs(const f4* __restrict__ s, f4* __restrict__ d, int64_t n) {
  const int64_t stride = int64_t(gridDim.x) * 256;
  int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ldf<NTL>(s + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) stf<NTS>(d + i + u * stride, v[u]);
  }
  for (; i < n; i += stride) stf<NTS>(d + i, ldf<NTL>(s + i));
}

// one block = 256*U contiguous f4, no grid-stride
template <bool NTL, bool NTS, int U>
__global__ __launch_bounds__(256) void copy_blk(const f4* __restrict__ s, f4* __restrict__ d, int64_t n) {
  const int64_t base = int64_t(blockIdx.x) * 256 * U + threadIdx.x;
  f4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) if (base + u * 256 < n) v[u] = ldf<NTL>(s + base + u * 256);
#pragma unroll
  for (int u = 0; u < U; ++u) if (base + u * 256 < n) stf<NTS>(d + base + u * 256, v[u]);
}

__device__ __forceinline__ f4 mix2(float a, f4 x, float b, f4 y) {
  f4 z = {0.f, 0.f, 0.f, 0.f};
  z = z + a * x;
  z = z + b * y;
  return z;
}

// ring: CPT f4 columns per lane (at c, c+256, ...), R rows per block, PF prefetch
template <int PF, int CPT, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void ring(const float* __restrict__ X, float* __restrict__ Y, int64_t ld,
                                            int n, int64_t ncols4, int64_t ntiles, int R,
                                            const float* __restrict__ wp, const float* __restrict__ wn) {
  const int64_t b = blockIdx.x;
  const int64_t ct = b % ntiles;
  const int rg = int(b / ntiles);
  const int64_t c0 = ct * 256 * CPT + threadIdx.x;
  const int r0 = rg * R, r1 = min(r0 + R, n);
  auto rowp = [&](int r) -> const f4* {
    int rr = r < 0 ? n - 1 : (r >= n ? 0 : r);
    return reinterpret_cast<const f4*>(X + int64_t(rr) * ld) + c0;
  };
  f4 q[PF + 2][CPT];
#pragma unroll
  for (int j = 0; j < CPT; ++j) { q[0][j] = ldf<NTL>(rowp(r0 - 1) + 256 * j); q[1][j] = ldf<NTL>(rowp(r0) + 256 * j); }
#pragma unroll
  for (int k = 0; k < PF; ++k)
#pragma unroll
    for (int j = 0; j < CPT; ++j) q[2 + k][j] = ldf<NTL>(rowp(min(r0 + 1 + k, r1)) + 256 * j);
  for (int i = r0; i < r1; i += PF) {
    f4 nx[PF][CPT];
#pragma unroll
    for (int k = 0; k < PF; ++k)
#pragma unroll
      for (int j = 0; j < CPT; ++j) nx[k][j] = ldf<NTL>(rowp(min(i + PF + 1 + k, r1)) + 256 * j);
#pragma unroll
    for (int k = 0; k < PF; ++k) {
      const int r = i + k;
      if (r < r1) {
        f4* yp = reinterpret_cast<f4*>(Y + int64_t(r) * ld) + c0;
#pragma unroll
        for (int j = 0; j < CPT; ++j) stf<NTS>(yp + 256 * j, mix2(wp[r], q[k][j], wn[r], q[k + 2][j]));
      }
    }
#pragma unroll
    for (int j = 0; j < CPT; ++j) { q[0][j] = q[PF][j]; q[1][j] = q[PF + 1][j]; }
#pragma unroll
    for (int k = 0; k < PF; ++k)
#pragma unroll
      for (int j = 0; j < CPT; ++j) q[2 + k][j] = nx[k][j];
  }
}

struct Variant {
  std::string name;
  double bytes;
  std::function<void()> launch;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 8192;
  const int64_t P = argc > 2 ? atoll(argv[2]) : (1 << 20);
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  const int64_t nel = int64_t(N) * P;
  float *X, *Y, *wp, *wn;
  CHECK(hipMalloc(&X, nel * 4));
  CHECK(hipMalloc(&Y, nel * 4));
  CHECK(hipMalloc(&wp, N * 4));
  CHECK(hipMalloc(&wn, N * 4));
  CHECK(hipMemset(X, 0x3f, nel * 4));
  CHECK(hipMemset(Y, 0, nel * 4));
  std::vector<float> hw(N, 0.5f);
  CHECK(hipMemcpy(wp, hw.data(), N * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(wn, hw.data(), N * 4, hipMemcpyHostToDevice));
  const int64_t n4 = nel / 4;
  const double cbytes = 2.0 * nel * 4;
  std::vector<Variant> vs;
  auto addc = [&](std::string nm, std::function<void()> f) { vs.push_back({nm, cbytes, f, {}}); };
  const f4* s4 = reinterpret_cast<const f4*>(X);
  f4* d4 = reinterpret_cast<f4*>(Y);
  for (int g : {2048, 4096, 8192}) {
    addc("copy_gs nt/nt U1 g" + std::to_string(g), [=] { copy_gs<true, true, 1><<<g, 256>>>(s4, d4, n4); });
    addc("copy_gs pl/pl U4 g" + std::to_string(g), [=] { copy_gs<false, false, 4><<<g, 256>>>(s4, d4, n4); });
    addc("copy_gs pl/nt U4 g" + std::to_string(g), [=] { copy_gs<false, true, 4><<<g, 256>>>(s4, d4, n4); });
    addc("copy_gs nt/nt U4 g" + std::to_string(g), [=] { copy_gs<true, true, 4><<<g, 256>>>(s4, d4, n4); });
  }
  addc("copy_blk pl/pl U4", [=] { copy_blk<false, false, 4><<<unsigned(n4 / 1024), 256>>>(s4, d4, n4); });
  addc("copy_blk pl/nt U4", [=] { copy_blk<false, true, 4><<<unsigned(n4 / 1024), 256>>>(s4, d4, n4); });
  addc("copy_blk nt/nt U4", [=] { copy_blk<true, true, 4><<<unsigned(n4 / 1024), 256>>>(s4, d4, n4); });
  addc("copy_blk pl/pl U8", [=] { copy_blk<false, false, 8><<<unsigned(n4 / 2048), 256>>>(s4, d4, n4); });
  addc("copy_blk pl/nt U8", [=] { copy_blk<false, true, 8><<<unsigned(n4 / 2048), 256>>>(s4, d4, n4); });
  addc("copy_blk pl/pl U2", [=] { copy_blk<false, false, 2><<<unsigned(n4 / 512), 256>>>(s4, d4, n4); });
  addc("hipMemcpyDtoD", [=] { CHECK(hipMemcpyAsync(Y, X, nel * 4, hipMemcpyDeviceToDevice, 0)); });

  const double rbytes = 2.0 * nel * 4;
  auto addr = [&](std::string nm, int cpt, std::function<void(int64_t, int64_t)> f, int R) {
    const int64_t ncols4 = P / 4;
    const int64_t ntiles = ncols4 / (256 * cpt);
    const int64_t grid = ntiles * ((N + R - 1) / R);
    vs.push_back({nm + " R" + std::to_string(R), rbytes, [=] { f(grid, ntiles); }, {}});
  };
  for (int R : {32, 64, 128, 256}) {
    addr("ring PF4 C1 pl/nt", 1, [=](int64_t g, int64_t t) { ring<4, 1, false, true><<<unsigned(g), 256>>>(X, Y, P, N, P / 4, t, R, wp, wn); }, R);
    addr("ring PF4 C1 pl/pl", 1, [=](int64_t g, int64_t t) { ring<4, 1, false, false><<<unsigned(g), 256>>>(X, Y, P, N, P / 4, t, R, wp, wn); }, R);
    addr("ring PF2 C2 pl/nt", 2, [=](int64_t g, int64_t t) { ring<2, 2, false, true><<<unsigned(g), 256>>>(X, Y, P, N, P / 4, t, R, wp, wn); }, R);
    addr("ring PF4 C2 pl/nt", 2, [=](int64_t g, int64_t t) { ring<4, 2, false, true><<<unsigned(g), 256>>>(X, Y, P, N, P / 4, t, R, wp, wn); }, R);
    addr("ring PF8 C1 pl/nt", 1, [=](int64_t g, int64_t t) { ring<8, 1, false, true><<<unsigned(g), 256>>>(X, Y, P, N, P / 4, t, R, wp, wn); }, R);
    addr("ring PF2 C1 pl/nt", 1, [=](int64_t g, int64_t t) { ring<2, 1, false, true><<<unsigned(g), 256>>>(X, Y, P, N, P / 4, t, R, wp, wn); }, R);
    addr("ring PF4 C1 nt/nt", 1, [=](int64_t g, int64_t t) { ring<4, 1, true, true><<<unsigned(g), 256>>>(X, Y, P, N, P / 4, t, R, wp, wn); }, R);
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (auto& v : vs) { v.launch(); }
  CHECK(hipDeviceSynchronize());
  for (int round = 0; round < 3; ++round) {
    for (auto& v : vs) {
      v.launch();
      CHECK(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; ++r) v.launch();
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / reps);
      CHECK(hipGetLastError());
    }
    fprintf(stderr, "round %d done\n", round);
  }
  printf("%-34s %10s %10s %10s\n", "variant", "ms(med)", "GB/s(med)", "GB/s(best)");
  for (auto& v : vs) {
    std::vector<float> m = v.ms;
    std::sort(m.begin(), m.end());
    printf("%-34s %10.3f %10.1f %10.1f\n", v.name.c_str(), m[m.size() / 2], v.bytes / (m[m.size() / 2] * 1e-3) / 1e9,
           v.bytes / (m[0] * 1e-3) / 1e9);
  }
  return 0;
}
