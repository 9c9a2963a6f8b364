// membench7.hip — what bounds the copy-like streams on gfx950: read-only,
// write-only, register vs LDS-DMA (global_load_lds ... nt) loads, and the ring
// stencil with LDS-DMA loads.  8192 x (2^20 + 1024) fp32 buffers.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o membench7 membench7.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <string>
#include <algorithm>
#include <functional>

typedef float f4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
#define GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define LPTR(p) ((__attribute__((address_space(3))) void*)(p))

__device__ __forceinline__ f4 mix2(float a, f4 x, float b, f4 y) {
  f4 z = {0.f, 0.f, 0.f, 0.f};
  z = z + a * x;
  z = z + b * y;
  return z;
}

template <bool NT, int U>
__global__ __launch_bounds__(256) void read_reg(const f4* __restrict__ s, float* __restrict__ sink, int64_t n) {
  const int64_t base = int64_t(blockIdx.x) * 256 * U + threadIdx.x;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < U; ++u) acc += NT ? __builtin_nontemporal_load(s + base + u * 256) : s[base + u * 256];
  if (acc.x == 1234.5f) sink[threadIdx.x] = acc.y;
}

template <int U, int AUX>
__global__ __launch_bounds__(256) void read_dma(const float* __restrict__ s, float* __restrict__ sink, int64_t n) {
  __shared__ __attribute__((aligned(16))) float lds[4][U][256];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float* g = s + int64_t(blockIdx.x) * 1024 * U + wave * 256 + lane * 4;
#pragma unroll
  for (int u = 0; u < U; ++u) __builtin_amdgcn_global_load_lds(GPTR(g + u * 1024), LPTR(&lds[wave][u][0]), 16, 0, AUX);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const f4 v = *reinterpret_cast<const f4*>(&lds[wave][0][lane * 4]);
  if (v.x == 1234.5f) sink[threadIdx.x] = v.y;
}

template <int U>
__global__ __launch_bounds__(256) void write_reg(f4* __restrict__ d, int64_t n, float val) {
  const int64_t base = int64_t(blockIdx.x) * 256 * U + threadIdx.x;
#pragma unroll
  for (int u = 0; u < U; ++u) __builtin_nontemporal_store(f4{val, val, val, val}, d + base + u * 256);
}

template <int U>
__global__ __launch_bounds__(256) void copy_reg(const f4* __restrict__ s, f4* __restrict__ d, int64_t n) {
  const int64_t base = int64_t(blockIdx.x) * 256 * U + threadIdx.x;
  f4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(s + base + u * 256);
#pragma unroll
  for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], d + base + u * 256);
}

// copy with LDS-DMA loads: wave w moves U pieces of 1 KiB
template <int U, int AUX>
__global__ __launch_bounds__(256) void copy_dma(const float* __restrict__ s, float* __restrict__ d, int64_t n) {
  __shared__ __attribute__((aligned(16))) float lds[4][U][256];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t off = int64_t(blockIdx.x) * 1024 * U + wave * 256 + lane * 4;
#pragma unroll
  for (int u = 0; u < U; ++u) __builtin_amdgcn_global_load_lds(GPTR(s + off + u * 1024), LPTR(&lds[wave][u][0]), 16, 0, AUX);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int u = 0; u < U; ++u)
    __builtin_nontemporal_store(*reinterpret_cast<const f4*>(&lds[wave][u][lane * 4]), reinterpret_cast<f4*>(d + off + u * 1024));
}

// register ring (library kernel shape): R=4 rows, 6 loads up front
__global__ __launch_bounds__(256) void ring_reg(const float* __restrict__ X, float* __restrict__ Y, int64_t ld, int n,
                                                uint32_t ntiles, const float* __restrict__ wp, const float* __restrict__ wn) {
  const uint32_t b = blockIdx.x;
  const uint32_t ct = b % ntiles;
  const int r0 = int(b / ntiles) * 4;
  const int64_t c = int64_t(ct) * 256 + threadIdx.x;
  f4 v[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    int r = r0 - 1 + k;
    r = r < 0 ? r + n : (r >= n ? r - n : r);
    v[k] = reinterpret_cast<const f4*>(X + int64_t(r) * ld)[c];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    __builtin_nontemporal_store(mix2(wp[r0 + k], v[k], wn[r0 + k], v[k + 2]), reinterpret_cast<f4*>(Y + int64_t(r0 + k) * ld) + c);
}

// LDS-DMA ring: each wave DMAs its 1 KiB quarter of the 6 rows, then reads back its lanes
template <int AUX>
__global__ __launch_bounds__(256) void ring_dma(const float* __restrict__ X, float* __restrict__ Y, int64_t ld, int n,
                                                uint32_t ntiles, const float* __restrict__ wp, const float* __restrict__ wn) {
  __shared__ __attribute__((aligned(16))) float lds[4][6][256];
  const uint32_t b = blockIdx.x;
  const uint32_t ct = b % ntiles;
  const int r0 = int(b / ntiles) * 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t c = int64_t(ct) * 1024 + wave * 256 + lane * 4;  // float column
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    int r = r0 - 1 + k;
    r = r < 0 ? r + n : (r >= n ? r - n : r);
    __builtin_amdgcn_global_load_lds(GPTR(X + int64_t(r) * ld + c), LPTR(&lds[wave][k][0]), 16, 0, AUX);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  f4 v[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) v[k] = *reinterpret_cast<const f4*>(&lds[wave][k][lane * 4]);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    __builtin_nontemporal_store(mix2(wp[r0 + k], v[k], wn[r0 + k], v[k + 2]), reinterpret_cast<f4*>(Y + int64_t(r0 + k) * ld + c));
}

// buffer stores with explicit cache-policy bits: aux 0 plain, 2 nt, 16 sc1, 17 sc0|sc1, 18 nt|sc1
template <int U, int AUX>
__global__ __launch_bounds__(256) void write_buf(float* __restrict__ d, float val) {
  float* base = d + int64_t(blockIdx.x) * 1024 * U;
  auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, 0, 1024 * U * 4, 0x00020000);
  const f4 v = {val, val, val, val};
#pragma unroll
  for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, (u * 256 + threadIdx.x) * 16, 0, AUX);
}

template <int AUX>
__global__ __launch_bounds__(256) void ring_dma_st(const float* __restrict__ X, float* __restrict__ Y, int64_t ld, int n,
                                                   uint32_t ntiles, const float* __restrict__ wp, const float* __restrict__ wn) {
  __shared__ __attribute__((aligned(16))) float lds[4][6][256];
  const uint32_t b = blockIdx.x;
  const uint32_t ct = b % ntiles;
  const int r0 = int(b / ntiles) * 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t c = int64_t(ct) * 1024 + wave * 256 + lane * 4;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    int r = r0 - 1 + k;
    r = r < 0 ? r + n : (r >= n ? r - n : r);
    __builtin_amdgcn_global_load_lds(GPTR(X + int64_t(r) * ld + c), LPTR(&lds[wave][k][0]), 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  f4 v[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) v[k] = *reinterpret_cast<const f4*>(&lds[wave][k][lane * 4]);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float* rowbase = Y + int64_t(r0 + k) * ld + int64_t(ct) * 1024;
    auto rsrc = __builtin_amdgcn_make_buffer_rsrc(rowbase, 0, 4096, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(mix2(wp[r0 + k], v[k], wn[r0 + k], v[k + 2]), rsrc, (wave * 256 + lane * 4) * 4, 0, AUX);
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
  const int reps = argc > 3 ? atoi(argv[3]) : 4;
  const int64_t ld = P + 1024;
  const int64_t nel = int64_t(N) * ld;
  float *X, *Y, *wp, *wn, *sink;
  CHECK(hipMalloc(&X, nel * 4));
  CHECK(hipMalloc(&Y, nel * 4));
  CHECK(hipMalloc(&wp, N * 4));
  CHECK(hipMalloc(&wn, N * 4));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMemset(X, 0x3f, nel * 4));
  std::vector<float> hw(N, 0.5f);
  CHECK(hipMemcpy(wp, hw.data(), N * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(wn, hw.data(), N * 4, hipMemcpyHostToDevice));
  const int64_t n4 = int64_t(N) * P / 4;  // stream the first N*P floats
  const double one = double(N) * P * 4;
  std::vector<Variant> vs;
  const f4* s4 = (const f4*)X;
  f4* d4 = (f4*)Y;
  vs.push_back({"write reg nt U4 (global)", one, [=] { write_reg<4><<<unsigned(n4 / 1024), 256>>>(d4, n4, 1.0f); }, {}});
  vs.push_back({"write buf plain U4", one, [=] { write_buf<4, 0><<<unsigned(n4 / 1024), 256>>>(Y, 1.0f); }, {}});
  vs.push_back({"write buf nt U4", one, [=] { write_buf<4, 2><<<unsigned(n4 / 1024), 256>>>(Y, 1.0f); }, {}});
  vs.push_back({"write buf sc1 U4", one, [=] { write_buf<4, 16><<<unsigned(n4 / 1024), 256>>>(Y, 1.0f); }, {}});
  vs.push_back({"write buf sc0sc1 U4", one, [=] { write_buf<4, 17><<<unsigned(n4 / 1024), 256>>>(Y, 1.0f); }, {}});
  vs.push_back({"write buf nt|sc1 U4", one, [=] { write_buf<4, 18><<<unsigned(n4 / 1024), 256>>>(Y, 1.0f); }, {}});
  vs.push_back({"write buf nt U8", one, [=] { write_buf<8, 2><<<unsigned(n4 / 2048), 256>>>(Y, 1.0f); }, {}});
  vs.push_back({"copy  dma nt + st nt U2", 2 * one, [=] { copy_dma<2, 2><<<unsigned(n4 / 512), 256>>>(X, Y, n4); }, {}});
  const uint32_t nt = uint32_t(P / 1024);
  const unsigned rg = unsigned(int64_t(nt) * (N / 4));
  vs.push_back({"ring  reg R4 (library)", 2 * one, [=] { ring_reg<<<rg, 256>>>(X, Y, ld, N, nt, wp, wn); }, {}});
  vs.push_back({"ring  dma pl R4 (global st nt)", 2 * one, [=] { ring_dma<0><<<rg, 256>>>(X, Y, ld, N, nt, wp, wn); }, {}});
  vs.push_back({"ring  dma pl R4 buf st plain", 2 * one, [=] { ring_dma_st<0><<<rg, 256>>>(X, Y, ld, N, nt, wp, wn); }, {}});
  vs.push_back({"ring  dma pl R4 buf st nt", 2 * one, [=] { ring_dma_st<2><<<rg, 256>>>(X, Y, ld, N, nt, wp, wn); }, {}});
  vs.push_back({"ring  dma pl R4 buf st sc1", 2 * one, [=] { ring_dma_st<16><<<rg, 256>>>(X, Y, ld, N, nt, wp, wn); }, {}});
  vs.push_back({"ring  dma pl R4 buf st nt|sc1", 2 * one, [=] { ring_dma_st<18><<<rg, 256>>>(X, Y, ld, N, nt, wp, wn); }, {}});
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (auto& v : vs) v.launch();
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
