// membench6.hip — CSR mixing on a random 4-regular graph (8192 x 2^20 fp32):
// tile width, rows per block, block order and XCD pinning.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o membench6 membench6.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <string>
#include <algorithm>
#include <functional>
#include <random>

typedef float f4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

__device__ __forceinline__ f4 fmac(f4 acc, float a, f4 x) { return acc + a * x; }

// (a) library-style: block = RPB rows x 256 f4 (4 KiB), row-group fastest
template <int RPB>
__global__ __launch_bounds__(256) void csr_rowfast(const float* __restrict__ X, int64_t ld, float* __restrict__ Y, int n,
                                                   int64_t nrg, const int* __restrict__ rp, const int* __restrict__ col,
                                                   const float* __restrict__ val) {
  const uint32_t b = blockIdx.x;
  const int rg = int(b % uint32_t(nrg));
  const int64_t ct = b / uint32_t(nrg);
  const int64_t c = ct * 256 + threadIdx.x;
  const f4* xb = reinterpret_cast<const f4*>(X) + c;
  const int64_t ldv = ld / 4;
  for (int r = rg * RPB; r < min(rg * RPB + RPB, n); ++r) {
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    const int e0 = rp[r], e1 = rp[r + 1];
    int e = e0;
    for (; e + 4 <= e1; e += 4) {
      f4 x0 = xb[col[e] * ldv], x1 = xb[col[e + 1] * ldv], x2 = xb[col[e + 2] * ldv], x3 = xb[col[e + 3] * ldv];
      acc = fmac(acc, val[e], x0); acc = fmac(acc, val[e + 1], x1); acc = fmac(acc, val[e + 2], x2); acc = fmac(acc, val[e + 3], x3);
    }
    for (; e < e1; ++e) acc = fmac(acc, val[e], xb[col[e] * ldv]);
    __builtin_nontemporal_store(acc, reinterpret_cast<f4*>(Y + int64_t(r) * ld) + c);
  }
}

// (b) XCD-pinned narrow tiles: a block covers RB rows x W f4 columns (W lanes per row,
// 256/W rows per pass); all blocks of one column tile share b % 8, so its X slab
// (n rows x W*16 B) is fetched into ONE XCD's L2 and re-read from there.
template <int W, int PASSES>
__global__ __launch_bounds__(256) void csr_xcd(const float* __restrict__ X, int64_t ld, float* __restrict__ Y, int n,
                                               int64_t nrb, int64_t ntiles, const int* __restrict__ rp,
                                               const int* __restrict__ col, const float* __restrict__ val) {
  constexpr int ROWS = 256 / W;            // rows per pass
  constexpr int RB = ROWS * PASSES;        // rows per block
  const uint32_t b = blockIdx.x;
  const uint32_t xcd = b & 7u;
  const uint32_t local = b >> 3;
  const uint32_t tiles_per_xcd = uint32_t((ntiles + 7) / 8);
  const uint32_t tloc = local / uint32_t(nrb);
  const uint32_t rb = local % uint32_t(nrb);
  const uint32_t ct = tloc * 8 + xcd;
  if (tloc >= tiles_per_xcd || ct >= ntiles) return;
  const int lane_c = threadIdx.x % W;
  const int lane_r = threadIdx.x / W;
  const int64_t c = int64_t(ct) * W + lane_c;
  const f4* xb = reinterpret_cast<const f4*>(X) + c;
  const int64_t ldv = ld / 4;
#pragma unroll
  for (int p = 0; p < PASSES; ++p) {
    const int r = int(rb) * RB + p * ROWS + lane_r;
    if (r < n) {
      f4 acc = {0.f, 0.f, 0.f, 0.f};
      const int e0 = rp[r], e1 = rp[r + 1];
      int e = e0;
      for (; e + 4 <= e1; e += 4) {
        f4 x0 = xb[col[e] * ldv], x1 = xb[col[e + 1] * ldv], x2 = xb[col[e + 2] * ldv], x3 = xb[col[e + 3] * ldv];
        acc = fmac(acc, val[e], x0); acc = fmac(acc, val[e + 1], x1); acc = fmac(acc, val[e + 2], x2); acc = fmac(acc, val[e + 3], x3);
      }
      for (; e < e1; ++e) acc = fmac(acc, val[e], xb[col[e] * ldv]);
      __builtin_nontemporal_store(acc, reinterpret_cast<f4*>(Y + int64_t(r) * ld) + c);
    }
  }
}

template <bool NTL, bool NTS, int U>
__global__ __launch_bounds__(256) void copy_blk(const f4* __restrict__ s, f4* __restrict__ d, int64_t n) {
  const int64_t base = int64_t(blockIdx.x) * 256 * U + threadIdx.x;
  f4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) if (base + u * 256 < n) v[u] = NTL ? __builtin_nontemporal_load(s + base + u * 256) : s[base + u * 256];
#pragma unroll
  for (int u = 0; u < U; ++u) if (base + u * 256 < n) __builtin_nontemporal_store(v[u], d + base + u * 256);
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
  const int deg = 4;
  const int64_t ld = P + 1024;
  // circulant C_n(1,2) under a random relabelling: 4-regular, non-local neighbours
  std::mt19937 rng(2028);
  std::vector<int> perm(N);
  for (int i = 0; i < N; ++i) perm[i] = i;
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<std::vector<int>> nb(N);
  for (int k = 1; k <= deg / 2; ++k)
    for (int i = 0; i < N; ++i) {
      int a = perm[i], b = perm[(i + k) % N];
      nb[a].push_back(b);
      nb[b].push_back(a);
    }
  std::vector<int> rp(N + 1, 0), col;
  std::vector<float> val;
  for (int i = 0; i < N; ++i) {
    std::sort(nb[i].begin(), nb[i].end());
    for (int j : nb[i]) { col.push_back(j); val.push_back(0.25f); }
    rp[i + 1] = int(col.size());
  }
  float *X, *Y, *dval;
  int *drp, *dcol;
  CHECK(hipMalloc(&X, int64_t(N) * ld * 4));
  CHECK(hipMalloc(&Y, int64_t(N) * ld * 4));
  CHECK(hipMalloc(&drp, (N + 1) * 4));
  CHECK(hipMalloc(&dcol, col.size() * 4));
  CHECK(hipMalloc(&dval, val.size() * 4));
  CHECK(hipMemcpy(drp, rp.data(), (N + 1) * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dcol, col.data(), col.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dval, val.data(), val.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemset(X, 0x3f, int64_t(N) * ld * 4));
  const double bytes = 2.0 * N * P * 4;
  std::vector<Variant> vs;
  const int64_t n4 = int64_t(N) * ld / 4;
  vs.push_back({"copy_blk nt/nt U4 (same bytes)", 2.0 * n4 * 16, [=] { copy_blk<true, true, 4><<<unsigned(n4 / 1024), 256>>>((const f4*)X, (f4*)Y, n4); }, {}});
  const int64_t nct = P / 4 / 256;
#define ROWF(R) vs.push_back({"rowfast 4KiB R" #R, bytes, [=] { const int64_t nrg = (N + R - 1) / R; csr_rowfast<R><<<unsigned(nct * nrg), 256>>>(X, ld, Y, N, nrg, drp, dcol, dval); }, {}});
  ROWF(4) ROWF(8) ROWF(16) ROWF(32)
#define XCD(W, PS)                                                                                                     \
  vs.push_back({"xcd W" #W " (" + std::to_string(W * 16) + "B) passes" #PS, bytes, [=] {                              \
    constexpr int RB = (256 / W) * PS;                                                                                  \
    const int64_t ntiles = P / 4 / W;                                                                                   \
    const int64_t nrb = (N + RB - 1) / RB;                                                                              \
    const int64_t tiles_per_xcd = (ntiles + 7) / 8;                                                                     \
    csr_xcd<W, PS><<<unsigned(tiles_per_xcd * nrb * 8), 256>>>(X, ld, Y, N, nrb, ntiles, drp, dcol, dval);              \
  }, {}});
  XCD(16, 1) XCD(16, 2) XCD(16, 4) XCD(32, 1) XCD(32, 2) XCD(64, 1) XCD(64, 2) XCD(8, 1) XCD(8, 2)
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
  printf("%-40s %10s %10s %10s\n", "variant", "ms(med)", "GB/s(med)", "GB/s(best)");
  for (auto& v : vs) {
    std::vector<float> m = v.ms;
    std::sort(m.begin(), m.end());
    printf("%-40s %10.3f %10.1f %10.1f\n", v.name.c_str(), m[m.size() / 2], v.bytes / (m[m.size() / 2] * 1e-3) / 1e9,
           v.bytes / (m[0] * 1e-3) / 1e9);
  }
  return 0;
}
