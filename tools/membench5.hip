// membench2.hip — ring-stencil tile shapes, block order and row-stride padding
// on gfx950 (8192 x 2^20 fp32).  hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <string>
#include <algorithm>
#include <functional>

typedef float f4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

template <bool NT> __device__ __forceinline__ f4 ldf(const f4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p); else return *p;
}
template <bool NT> __device__ __forceinline__ void stf(f4* p, f4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v;
}
__device__ __forceinline__ f4 mix2(float a, f4 x, float b, f4 y) {
  f4 z = {0.f, 0.f, 0.f, 0.f};
  z = z + a * x;
  z = z + b * y;
  return z;
}

template <bool NTL, bool NTS, int U>
__global__ __launch_bounds__(256) void copy_blk(const f4* __restrict__ s, f4* __restrict__ d, int64_t n) {
  const int64_t base = int64_t(blockIdx.x) * 256 * U + threadIdx.x;
  f4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) if (base + u * 256 < n) v[u] = ldf<NTL>(s + base + u * 256);
#pragma unroll
  for (int u = 0; u < U; ++u) if (base + u * 256 < n) stf<NTS>(d + base + u * 256, v[u]);
}

// short-lived tile: R output rows x (256*CPT) f4 columns; loads all R+2 rows first
template <int R, int CPT, bool NTL, bool NTS, bool ROWFAST>
__global__ __launch_bounds__(256) void ring_tile(const float* __restrict__ X, float* __restrict__ Y, int64_t ld, int n,
                                                 int64_t ntiles, int64_t nrg, const float* __restrict__ wp,
                                                 const float* __restrict__ wn) {
  const int64_t b = blockIdx.x;
  int64_t ct, rg;
  if constexpr (ROWFAST) { rg = b % nrg; ct = b / nrg; } else { ct = b % ntiles; rg = b / ntiles; }
  const int64_t c0 = ct * 256 * CPT + threadIdx.x;
  const int r0 = int(rg) * R;
  f4 v[R + 2][CPT];
#pragma unroll
  for (int k = 0; k < R + 2; ++k) {
    int r = r0 - 1 + k;
    r = r < 0 ? r + n : (r >= n ? r - n : r);
    const f4* p = reinterpret_cast<const f4*>(X + int64_t(r) * ld) + c0;
#pragma unroll
    for (int j = 0; j < CPT; ++j) v[k][j] = ldf<NTL>(p + 256 * j);
  }
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int r = r0 + k;
    if (r < n) {
      f4* p = reinterpret_cast<f4*>(Y + int64_t(r) * ld) + c0;
#pragma unroll
      for (int j = 0; j < CPT; ++j) stf<NTS>(p + 256 * j, mix2(wp[r], v[k][j], wn[r], v[k + 2][j]));
    }
  }
}

// the library's long-lived sliding-window kernel (PF prefetch)
template <int PF, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void ring_slide(const float* __restrict__ X, float* __restrict__ Y, int64_t ld, int n,
                                                  int64_t ntiles, int R, const float* __restrict__ wp,
                                                  const float* __restrict__ wn) {
  const int64_t b = blockIdx.x;
  const int64_t ct = b % ntiles;
  const int rg = int(b / ntiles);
  const int64_t c0 = ct * 256 + threadIdx.x;
  const int r0 = rg * R, r1 = min(r0 + R, n);
  auto rowp = [&](int r) -> const f4* {
    int rr = r < 0 ? n - 1 : (r >= n ? 0 : r);
    return reinterpret_cast<const f4*>(X + int64_t(rr) * ld) + c0;
  };
  f4 q[PF + 2];
  q[0] = ldf<NTL>(rowp(r0 - 1));
  q[1] = ldf<NTL>(rowp(r0));
#pragma unroll
  for (int k = 0; k < PF; ++k) q[2 + k] = ldf<NTL>(rowp(min(r0 + 1 + k, r1)));
  for (int i = r0; i < r1; i += PF) {
    f4 nx[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) nx[k] = ldf<NTL>(rowp(min(i + PF + 1 + k, r1)));
#pragma unroll
    for (int k = 0; k < PF; ++k) {
      const int r = i + k;
      if (r < r1) stf<NTS>(reinterpret_cast<f4*>(Y + int64_t(r) * ld) + c0, mix2(wp[r], q[k], wn[r], q[k + 2]));
    }
    q[0] = q[PF];
    q[1] = q[PF + 1];
#pragma unroll
    for (int k = 0; k < PF; ++k) q[2 + k] = nx[k];
  }
}

// geometry control: same tile walk as ring_slide but Y[r] = X[r] (one read stream)
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void tile_copy(const float* __restrict__ X, float* __restrict__ Y, int64_t ld, int n,
                                                 int64_t ntiles, int R) {
  const int64_t b = blockIdx.x;
  const int64_t ct = b % ntiles;
  const int rg = int(b / ntiles);
  const int64_t c0 = ct * 256 + threadIdx.x;
  const int r0 = rg * R, r1 = min(r0 + R, n);
  for (int i = r0; i < r1; i += 4) {
    f4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = ldf<NTL>(reinterpret_cast<const f4*>(X + int64_t(min(i + k, r1 - 1)) * ld) + c0);
#pragma unroll
    for (int k = 0; k < 4; ++k) if (i + k < r1) stf<NTS>(reinterpret_cast<f4*>(Y + int64_t(i + k) * ld) + c0, v[k]);
  }
}

template <int PF, int CPT, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void ring_slideC(const float* __restrict__ X, float* __restrict__ Y, int64_t ld, int n,
                                                   int64_t ntiles, int R, const float* __restrict__ wp,
                                                   const float* __restrict__ wn) {
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

// blocked layout [P/B][N][B]: column block k of row r at ((k*N)+r)*B; CPT = B/1024 f4 per lane
template <int R, int CPT, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void ring_blk(const float* __restrict__ X, float* __restrict__ Y, int n,
                                                int64_t nkb, int64_t nrg, const float* __restrict__ wp,
                                                const float* __restrict__ wn) {
  constexpr int B = 1024 * CPT;
  const int64_t b = blockIdx.x;
  const int64_t k = b % nkb;   // column block fastest
  const int64_t rg = b / nkb;
  const int r0 = int(rg) * R;
  const float* xb = X + k * int64_t(n) * B;
  float* yb = Y + k * int64_t(n) * B;
  f4 v[R + 2][CPT];
#pragma unroll
  for (int q = 0; q < R + 2; ++q) {
    int r = r0 - 1 + q;
    r = r < 0 ? r + n : (r >= n ? r - n : r);
    const f4* p = reinterpret_cast<const f4*>(xb + int64_t(r) * B) + threadIdx.x;
#pragma unroll
    for (int j = 0; j < CPT; ++j) v[q][j] = ldf<NTL>(p + 256 * j);
  }
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int r = r0 + q;
    if (r < n) {
      f4* p = reinterpret_cast<f4*>(yb + int64_t(r) * B) + threadIdx.x;
#pragma unroll
      for (int j = 0; j < CPT; ++j) stf<NTS>(p + 256 * j, mix2(wp[r], v[q][j], wn[r], v[q + 2][j]));
    }
  }
}
// blocked layout, row-group fastest (all rows of one column block back to back = contiguous stream)
template <int R, int CPT, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void ring_blk_rf(const float* __restrict__ X, float* __restrict__ Y, int n,
                                                   int64_t nkb, int64_t nrg, const float* __restrict__ wp,
                                                   const float* __restrict__ wn) {
  constexpr int B = 1024 * CPT;
  const int64_t b = blockIdx.x;
  const int64_t rg = b % nrg;
  const int64_t k = b / nrg;
  const int r0 = int(rg) * R;
  const float* xb = X + k * int64_t(n) * B;
  float* yb = Y + k * int64_t(n) * B;
  f4 v[R + 2][CPT];
#pragma unroll
  for (int q = 0; q < R + 2; ++q) {
    int r = r0 - 1 + q;
    r = r < 0 ? r + n : (r >= n ? r - n : r);
    const f4* p = reinterpret_cast<const f4*>(xb + int64_t(r) * B) + threadIdx.x;
#pragma unroll
    for (int j = 0; j < CPT; ++j) v[q][j] = ldf<NTL>(p + 256 * j);
  }
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int r = r0 + q;
    if (r < n) {
      f4* p = reinterpret_cast<f4*>(yb + int64_t(r) * B) + threadIdx.x;
#pragma unroll
      for (int j = 0; j < CPT; ++j) stf<NTS>(p + 256 * j, mix2(wp[r], v[q][j], wn[r], v[q + 2][j]));
    }
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
  const int64_t maxpad = 4096;
  const int64_t nel = int64_t(N) * (P + maxpad);
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
  const double bytes = 2.0 * N * P * 4;
  std::vector<Variant> vs;
  const int64_t n4 = int64_t(N) * P / 4;
  vs.push_back({"copy_blk nt/nt U4", bytes, [=] { copy_blk<true, true, 4><<<unsigned(n4 / 1024), 256>>>((const f4*)X, (f4*)Y, n4); }, {}});
  vs.push_back({"copy_blk nt/nt U2", bytes, [=] { copy_blk<true, true, 2><<<unsigned(n4 / 512), 256>>>((const f4*)X, (f4*)Y, n4); }, {}});
  vs.push_back({"copy_blk nt/nt U4 +4K", bytes, [=] { copy_blk<true, true, 4><<<unsigned(n4 / 1024), 256>>>((const f4*)X, (f4*)(Y + 1024), n4); }, {}});

  {
    const int64_t nt1 = P / 4 / 256;
    { const int64_t ld = P + 0; const int64_t g1 = nt1 * ((N + 2 - 1) / 2);
      vs.push_back({"slide PF2 pl/nt R2 pad0", bytes, [=] { ring_slideC<2, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 2, wp, wn); }, {}}); }
    { const int64_t ld = P + 0; const int64_t g1 = nt1 * ((N + 2 - 1) / 2);
      vs.push_back({"slide PF4 pl/nt R2 pad0", bytes, [=] { ring_slideC<4, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 2, wp, wn); }, {}}); }
    { const int64_t ld = P + 0; const int64_t g1 = nt1 * ((N + 3 - 1) / 3);
      vs.push_back({"slide PF4 pl/nt R3 pad0", bytes, [=] { ring_slideC<4, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 3, wp, wn); }, {}}); }
    { const int64_t ld = P + 0; const int64_t g1 = nt1 * ((N + 4 - 1) / 4);
      vs.push_back({"slide PF4 pl/nt R4 pad0", bytes, [=] { ring_slideC<4, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}}); }
    { const int64_t ld = P + 0; const int64_t g1 = nt1 * ((N + 4 - 1) / 4);
      vs.push_back({"slide PF8 pl/nt R4 pad0", bytes, [=] { ring_slideC<8, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}}); }
    { const int64_t ld = P + 0; const int64_t g1 = nt1 * ((N + 6 - 1) / 6);
      vs.push_back({"slide PF6 pl/nt R6 pad0", bytes, [=] { ring_slideC<6, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 6, wp, wn); }, {}}); }
    { const int64_t ld = P + 0; const int64_t g1 = nt1 * ((N + 6 - 1) / 6);
      vs.push_back({"slide PF8 pl/nt R6 pad0", bytes, [=] { ring_slideC<8, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 6, wp, wn); }, {}}); }
    { const int64_t ld = P + 0; const int64_t g1 = nt1 * ((N + 8 - 1) / 8);
      vs.push_back({"slide PF8 pl/nt R8 pad0", bytes, [=] { ring_slideC<8, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 8, wp, wn); }, {}}); }
    { const int64_t ld = P + 0; const int64_t g1 = nt1 * ((N + 4 - 1) / 4);
      vs.push_back({"slide PF4 nt/nt R4 pad0", bytes, [=] { ring_slideC<4, 1, true, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}});
      vs.push_back({"slide PF4 pl/pl R4 pad0", bytes, [=] { ring_slideC<4, 1, false, false><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}});
      vs.push_back({"tilecopy R4 pad0", bytes, [=] { tile_copy<true, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4); }, {}}); }
    { const int64_t ld = P + 64; const int64_t g1 = nt1 * ((N + 2 - 1) / 2);
      vs.push_back({"slide PF2 pl/nt R2 pad64", bytes, [=] { ring_slideC<2, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 2, wp, wn); }, {}}); }
    { const int64_t ld = P + 64; const int64_t g1 = nt1 * ((N + 2 - 1) / 2);
      vs.push_back({"slide PF4 pl/nt R2 pad64", bytes, [=] { ring_slideC<4, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 2, wp, wn); }, {}}); }
    { const int64_t ld = P + 64; const int64_t g1 = nt1 * ((N + 3 - 1) / 3);
      vs.push_back({"slide PF4 pl/nt R3 pad64", bytes, [=] { ring_slideC<4, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 3, wp, wn); }, {}}); }
    { const int64_t ld = P + 64; const int64_t g1 = nt1 * ((N + 4 - 1) / 4);
      vs.push_back({"slide PF4 pl/nt R4 pad64", bytes, [=] { ring_slideC<4, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}}); }
    { const int64_t ld = P + 64; const int64_t g1 = nt1 * ((N + 4 - 1) / 4);
      vs.push_back({"slide PF8 pl/nt R4 pad64", bytes, [=] { ring_slideC<8, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}}); }
    { const int64_t ld = P + 64; const int64_t g1 = nt1 * ((N + 6 - 1) / 6);
      vs.push_back({"slide PF6 pl/nt R6 pad64", bytes, [=] { ring_slideC<6, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 6, wp, wn); }, {}}); }
    { const int64_t ld = P + 64; const int64_t g1 = nt1 * ((N + 6 - 1) / 6);
      vs.push_back({"slide PF8 pl/nt R6 pad64", bytes, [=] { ring_slideC<8, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 6, wp, wn); }, {}}); }
    { const int64_t ld = P + 64; const int64_t g1 = nt1 * ((N + 8 - 1) / 8);
      vs.push_back({"slide PF8 pl/nt R8 pad64", bytes, [=] { ring_slideC<8, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 8, wp, wn); }, {}}); }
    { const int64_t ld = P + 64; const int64_t g1 = nt1 * ((N + 4 - 1) / 4);
      vs.push_back({"slide PF4 nt/nt R4 pad64", bytes, [=] { ring_slideC<4, 1, true, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}});
      vs.push_back({"slide PF4 pl/pl R4 pad64", bytes, [=] { ring_slideC<4, 1, false, false><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}});
      vs.push_back({"tilecopy R4 pad64", bytes, [=] { tile_copy<true, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4); }, {}}); }
    { const int64_t ld = P + 256; const int64_t g1 = nt1 * ((N + 2 - 1) / 2);
      vs.push_back({"slide PF2 pl/nt R2 pad256", bytes, [=] { ring_slideC<2, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 2, wp, wn); }, {}}); }
    { const int64_t ld = P + 256; const int64_t g1 = nt1 * ((N + 2 - 1) / 2);
      vs.push_back({"slide PF4 pl/nt R2 pad256", bytes, [=] { ring_slideC<4, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 2, wp, wn); }, {}}); }
    { const int64_t ld = P + 256; const int64_t g1 = nt1 * ((N + 3 - 1) / 3);
      vs.push_back({"slide PF4 pl/nt R3 pad256", bytes, [=] { ring_slideC<4, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 3, wp, wn); }, {}}); }
    { const int64_t ld = P + 256; const int64_t g1 = nt1 * ((N + 4 - 1) / 4);
      vs.push_back({"slide PF4 pl/nt R4 pad256", bytes, [=] { ring_slideC<4, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}}); }
    { const int64_t ld = P + 256; const int64_t g1 = nt1 * ((N + 4 - 1) / 4);
      vs.push_back({"slide PF8 pl/nt R4 pad256", bytes, [=] { ring_slideC<8, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}}); }
    { const int64_t ld = P + 256; const int64_t g1 = nt1 * ((N + 6 - 1) / 6);
      vs.push_back({"slide PF6 pl/nt R6 pad256", bytes, [=] { ring_slideC<6, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 6, wp, wn); }, {}}); }
    { const int64_t ld = P + 256; const int64_t g1 = nt1 * ((N + 6 - 1) / 6);
      vs.push_back({"slide PF8 pl/nt R6 pad256", bytes, [=] { ring_slideC<8, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 6, wp, wn); }, {}}); }
    { const int64_t ld = P + 256; const int64_t g1 = nt1 * ((N + 8 - 1) / 8);
      vs.push_back({"slide PF8 pl/nt R8 pad256", bytes, [=] { ring_slideC<8, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 8, wp, wn); }, {}}); }
    { const int64_t ld = P + 256; const int64_t g1 = nt1 * ((N + 4 - 1) / 4);
      vs.push_back({"slide PF4 nt/nt R4 pad256", bytes, [=] { ring_slideC<4, 1, true, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}});
      vs.push_back({"slide PF4 pl/pl R4 pad256", bytes, [=] { ring_slideC<4, 1, false, false><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}});
      vs.push_back({"tilecopy R4 pad256", bytes, [=] { tile_copy<true, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4); }, {}}); }
    { const int64_t ld = P + 1024; const int64_t g1 = nt1 * ((N + 2 - 1) / 2);
      vs.push_back({"slide PF2 pl/nt R2 pad1024", bytes, [=] { ring_slideC<2, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 2, wp, wn); }, {}}); }
    { const int64_t ld = P + 1024; const int64_t g1 = nt1 * ((N + 2 - 1) / 2);
      vs.push_back({"slide PF4 pl/nt R2 pad1024", bytes, [=] { ring_slideC<4, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 2, wp, wn); }, {}}); }
    { const int64_t ld = P + 1024; const int64_t g1 = nt1 * ((N + 3 - 1) / 3);
      vs.push_back({"slide PF4 pl/nt R3 pad1024", bytes, [=] { ring_slideC<4, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 3, wp, wn); }, {}}); }
    { const int64_t ld = P + 1024; const int64_t g1 = nt1 * ((N + 4 - 1) / 4);
      vs.push_back({"slide PF4 pl/nt R4 pad1024", bytes, [=] { ring_slideC<4, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}}); }
    { const int64_t ld = P + 1024; const int64_t g1 = nt1 * ((N + 4 - 1) / 4);
      vs.push_back({"slide PF8 pl/nt R4 pad1024", bytes, [=] { ring_slideC<8, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}}); }
    { const int64_t ld = P + 1024; const int64_t g1 = nt1 * ((N + 6 - 1) / 6);
      vs.push_back({"slide PF6 pl/nt R6 pad1024", bytes, [=] { ring_slideC<6, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 6, wp, wn); }, {}}); }
    { const int64_t ld = P + 1024; const int64_t g1 = nt1 * ((N + 6 - 1) / 6);
      vs.push_back({"slide PF8 pl/nt R6 pad1024", bytes, [=] { ring_slideC<8, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 6, wp, wn); }, {}}); }
    { const int64_t ld = P + 1024; const int64_t g1 = nt1 * ((N + 8 - 1) / 8);
      vs.push_back({"slide PF8 pl/nt R8 pad1024", bytes, [=] { ring_slideC<8, 1, false, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 8, wp, wn); }, {}}); }
    { const int64_t ld = P + 1024; const int64_t g1 = nt1 * ((N + 4 - 1) / 4);
      vs.push_back({"slide PF4 nt/nt R4 pad1024", bytes, [=] { ring_slideC<4, 1, true, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}});
      vs.push_back({"slide PF4 pl/pl R4 pad1024", bytes, [=] { ring_slideC<4, 1, false, false><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4, wp, wn); }, {}});
      vs.push_back({"tilecopy R4 pad1024", bytes, [=] { tile_copy<true, true><<<unsigned(g1), 256>>>(X, Y, ld, N, nt1, 4); }, {}}); }
  }
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
