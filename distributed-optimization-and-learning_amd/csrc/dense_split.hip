// dense_split.hip — dense mix Y = W X on the bf16 matrix cores at fp32 accuracy.
//
// Dense mixing matrices (communication_graph("compelete", "stochastic", n),
// Erdos-Renyi and time-varying W; DIST/simulators.py:54-58, :65-70) make the
// round a GEMM: Y[M,P] = W[M,K] X[K,P], 2 M K P flop.  gfx950 has no
// reduced-precision f32 MFMA (no xf32) and its exact f32 MFMA runs at 1/16 of
// the bf16 rate, so this path splits every fp32 operand into three bf16
// pieces, x = x0 + x1 + x2 exactly (x0 = bf16_rne(x), x1 = bf16_rne(x - x0),
// x2 = bf16_rne(x - x0 - x1): |x1| <= 2^-8 |x|, |x2| <= 2^-16 |x| and the
// remainder is 0), and sums the six piece products of scale >= 2^-16 |w x|
// on v_mfma_f32_32x32x16_bf16:
//     w x ~= w0 x0 + w0 x1 + w1 x0 + w1 x1 + w0 x2 + w2 x0
// Each bf16 x bf16 product is exact in fp32 and the MFMA accumulates in fp32,
// so the result is an fp32-accurate GEMM: the dropped terms (w1 x2, w2 x1,
// w2 x2) sum to at most 2^-23 |w x|, about one fp32 rounding of the product.  Six bf16 MFMAs
// cost 6 x 32 = 192 cycles per 32x32x16 block where the f32 MFMA needs
// 8 x 64 = 512: 2.67x the f32 matrix peak.  Error bound and the tests:
// tests/test_kernels_gpu.py (test_mix_dense_split3_*).
//
// Layout.  A split pass writes both operands in the MFMA's own k-grouping:
// WA[kg][m][piece][8 bf16] and XB[kg][p][piece][8 bf16] (kg = k / 8, rows
// m / columns p padded to the 256-tile, k padded to 16, zero filled), so one
// (row, k-group) record is 48 contiguous bytes holding a lane's three
// fragments, and a 256-row tile of one k-group is 12 KiB contiguous: the GEMM
// stages it with 12 LDS-DMA instructions (global_load_lds_dwordx4, no
// register round trip, no bounds checks) and reads fragments conflict-free
// (48-B lane stride).
//
// GEMM.  256 x 256 output tile per workgroup, 8 waves in 2 x 4, each wave
// 128 x 64 = 4 x 2 accumulators of 32 x 32 (128 accumulator registers, two
// waves per SIMD; the r01 form, 4 waves of 128 x 128 with 256 accumulator
// registers, remains for the narrow tail tiles and DOL_SPLIT3_WAVES=4).
// K advances 16 per stage (= one MFMA k-step); three stages of 48 KiB in LDS,
// two in flight while one feeds 48 MFMAs per wave.  Tile
// order is XCD-aware: workgroup b runs on XCD b % 8, each XCD walks a
// contiguous range of tiles in groups of 8 row tiles, so the 32 tiles an XCD
// holds at once share 8 W panels and 4 X panels in its L2.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/dol_hip.h"
#include "dol_common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kTile = 256;                            // BM = BN
constexpr int kRec = 48;                              // bytes per (row, k-group): 3 pieces x 8 bf16
constexpr int kOpStage = 2 * kTile * kRec;            // 24 KiB: one operand, two k-groups
constexpr int kStageBytes = 2 * kOpStage;             // 48 KiB
constexpr int kStages = 3;
constexpr int kLds = kStages * kStageBytes;           // 144 KiB
constexpr int kGroupM = 8;                            // row tiles per XCD group
constexpr int kDmaPerWave = kStageBytes / 1024 / 4;   // 12 LDS-DMA instructions per wave per stage
// fused-X variant: B staged as fp32 rows (16 k x 256 p, 1040-B pitch so the two
// lane halves' rows 8 apart fall on different banks) and split in registers
constexpr int kBPitch = 1040;
constexpr int kStageFX = kOpStage + 16 * kBPitch;     // 41216 B
constexpr int kDmaFX = (24 + 16) / 4;                  // 10 per wave per stage

#define DOL_GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define DOL_LPTR(p) ((__attribute__((address_space(3))) void*)(p))

__device__ __forceinline__ bool finite_bits(uint32_t u) { return (u & 0x7f800000u) != 0x7f800000u; }

// fp32 -> bf16 bits, round to nearest even; NaN stays NaN (quiet), Inf stays Inf
__device__ __forceinline__ uint32_t bf16_rne(float x) {
  const uint32_t u = __float_as_uint(x);
  if (!finite_bits(u)) return (u >> 16) | ((u & 0x7fffffu) ? 0x40u : 0u);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// x = p0 + p1 + p2 exactly (finite x); non-finite x -> (x, 0, 0)
__device__ __forceinline__ void split3(float x, uint32_t& p0, uint32_t& p1, uint32_t& p2) {
  const uint32_t u = __float_as_uint(x);
  uint32_t h0 = bf16_rne(x);
  if (finite_bits(u) && (h0 & 0x7f80u) == 0x7f80u) h0 = u >> 16;  // |x| rounds past bf16 max: truncate
  const float r1 = finite_bits(u) ? x - __uint_as_float(h0 << 16) : 0.f;
  const uint32_t h1 = bf16_rne(r1);
  const float r2 = r1 - __uint_as_float(h1 << 16);
  p0 = h0;
  p1 = h1;
  p2 = bf16_rne(r2);
}

// Split 8 consecutive-k values into one 48-B record (3 x 16 B).
__device__ __forceinline__ void write_record(const float (&v)[8], uint8_t* dst) {
  u32x4 q[3];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t a0, a1, a2, b0, b1, b2;
    split3(v[2 * j], a0, a1, a2);
    split3(v[2 * j + 1], b0, b1, b2);
    q[0][j] = a0 | (b0 << 16);
    q[1][j] = a1 | (b1 << 16);
    q[2][j] = a2 | (b2 << 16);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) *reinterpret_cast<u32x4*>(dst + 16 * i) = q[i];
}

// W [M][K] (row stride ldw) -> WA[kg][Mp][48 B]; one thread per (m, kg), m fastest
__global__ __launch_bounds__(256) void split3_rows_kernel(const float* __restrict__ W, int64_t ldw, int M, int K,
                                                          int Mp, int Kg, uint8_t* __restrict__ out) {
  const int64_t idx = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (idx >= int64_t(Mp) * Kg) return;
  const int m = int(idx % Mp), kg = int(idx / Mp);
  float v[8];
  const float* row = W + int64_t(m < M ? m : 0) * ldw;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * kg + j;
    v[j] = (m < M && k < K) ? row[k] : 0.f;
  }
  write_record(v, out + idx * kRec);
}

// X [K][P] (row stride ldx) -> XB[kg][Pp][48 B]; one thread per (p, kg), p fastest
// (the r01 pass, DOL_SPLIT3_XPASS1=1; split3_cols4_kernel below is the default:
// 196 vs 224 us at 1024 x 101,770, profiles/r02_split3_xpass.txt)
__global__ __launch_bounds__(256) void split3_cols_kernel(const float* __restrict__ X, int64_t ldx, int K, int64_t P,
                                                          int64_t Pp, int Kg, uint8_t* __restrict__ out) {
  const int64_t idx = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (idx >= Pp * Kg) return;
  const int64_t p = idx % Pp;
  const int kg = int(idx / Pp);
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * kg + j;
    v[j] = (p < P && k < K) ? X[int64_t(k) * ldx + p] : 0.f;
  }
  write_record(v, out + idx * kRec);
}

// The same records, one thread per (4 columns, kg): eight 16-B row loads and
// four whole records.  Thread idx's records are bytes [192 idx, 192 idx + 192)
// of XB (idx = kg Pp/4 + p/4), so a wave's output is 12 KiB contiguous: the
// records go through LDS (208-B thread pitch against bank conflicts) and leave
// as twelve fully coalesced 1-KiB stores per wave.  VEC: X rows 16-B aligned
// (ldx % 4 == 0); the last, partial column group and unaligned X read per
// element.
constexpr int kX4Pitch = 208;
template <bool VEC>
__global__ __launch_bounds__(256) void split3_cols4_kernel(const float* __restrict__ X, int64_t ldx, int K, int64_t P,
                                                           int64_t Pp, int Kg, uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t st[256 * kX4Pitch];
  const int64_t idx = int64_t(blockIdx.x) * 256 + threadIdx.x;
  const int64_t nq = Pp / 4, total = nq * Kg;
  if (idx < total) {
    const int64_t p0 = 4 * (idx % nq);
    const int kg = int(idx / nq);
    float v[4][8];
    const bool whole = VEC && p0 + 4 <= P;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * kg + j;
      const float* row = X + int64_t(k < K ? k : 0) * ldx + p0;
      if (whole) {
        const f4v q = k < K ? *reinterpret_cast<const f4v*>(row) : f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c][j] = q[c];
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c][j] = (k < K && p0 + c < P) ? row[c] : 0.f;
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) write_record(v[c], st + threadIdx.x * kX4Pitch + c * kRec);
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t wbase = (int64_t(blockIdx.x) * 256 + wave * 64) * (4 * kRec);  // first output byte of the wave
  const int64_t end = total * (4 * kRec);
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int o = 1024 * i + 16 * lane;  // byte within the wave's 12 KiB
    const int t = o / (4 * kRec), w = o - t * (4 * kRec);
    if (wbase + o < end)
      *reinterpret_cast<u32x4*>(out + wbase + o) =
          *reinterpret_cast<const u32x4*>(st + (wave * 64 + t) * kX4Pitch + w);
  }
}

// wait until at most N of this wave's vector-memory operations are in flight
template <int N>
__device__ __forceinline__ void wait_vmcnt_le(bool more) {
  if (!more) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
static_assert(kDmaPerWave == 12 && kDmaFX == 10, "stage sizes changed: recheck the DMA counts per wave");

typedef float f2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));

// split3() of 8 values into three bf16x8 fragments with v_cvt_pk_bf16_f32 (RNE,
// the same rounding as bf16_rne), bit-identical to the split pass; a wave with
// any non-finite or |x| >= 0x7f7f8000 value takes split3() itself
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& p0, bf16x8& p1, bf16x8& p2) {
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 8; ++j) bad |= !(__builtin_fabsf(v[j]) < __uint_as_float(0x7f7f8000u));
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(bad) != 0, 0)) {
    u32x4 q[3];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t a0, a1, a2, b0, b1, b2;
      split3(v[2 * j], a0, a1, a2);
      split3(v[2 * j + 1], b0, b1, b2);
      q[0][j] = a0 | (b0 << 16);
      q[1][j] = a1 | (b1 << 16);
      q[2][j] = a2 | (b2 << 16);
    }
    p0 = __builtin_bit_cast(bf16x8, q[0]);
    p1 = __builtin_bit_cast(bf16x8, q[1]);
    p2 = __builtin_bit_cast(bf16x8, q[2]);
    return;
  }
  bf2 a[4], b[4], c[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f2 x = {v[2 * j], v[2 * j + 1]};
    a[j] = __builtin_convertvector(x, bf2);
    const f2 r1 = x - __builtin_convertvector(a[j], f2);
    b[j] = __builtin_convertvector(r1, bf2);
    const f2 r2 = r1 - __builtin_convertvector(b[j], f2);
    c[j] = __builtin_convertvector(r2, bf2);
  }
  auto cat = [](const bf2 (&w)[4]) {
    const bf4 lo = __builtin_shufflevector(w[0], w[1], 0, 1, 2, 3);
    const bf4 hi = __builtin_shufflevector(w[2], w[3], 0, 1, 2, 3);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  p0 = cat(a);
  p1 = cat(b);
  p2 = cat(c);
}

// PROBE (tools only, DOL_SPLIT3_PROBE): 1 = no operand staging (MFMA ceiling of
// the loop), 2 = staging only (no fragment reads / MFMAs), 3 = as 1 without
// the output stores, 4 = full kernel without the output stores (5 / 6 / 7: 1 / 2 /
// 4 on the 8-wave tiles).  Measured at 8192 x
// 101770 (profiles/r01c_dense_split3_probe.txt): full 53 ms, MFMA-only 45 ms,
// staging-only 20 ms.  Tried and dropped (same box, no gain): fragments
// double-buffered in registers with the DMA three stages ahead; the
// v_mfma_f32_16x16x32_bf16 shape with (k-group, piece pair) k slots (same
// speed, and mixing piece scales inside one MFMA loses exactness of x0+x1+x2);
// the DMA issue sliced between the row blocks' MFMA clusters (sched_barrier
// fenced; 53.5-54.1 vs 53.6-53.7 ms).  The full kernel's gap to the MFMA-only
// probe is not an issue-order effect.  128-row tiles (2 stages, two
// workgroups per CU; or 3 stages): 1.27 / 1.40 vs 1.30 ms at 1024 agents,
// 69-70 vs 58 ms at 8192 (profiles/r01c_dense_split3_tiles.txt): kept 256.
// FX: B operand straight from fp32 X (split in registers) instead of the split
// pass's XB records; X rows readable up to `pread` floats (>= P, % 4 == 0).
// NB: 32-column blocks per wave along P.  NB = 4 is the 256 x 256 tile; NB = 1
// / 2 (256 x 64 / 256 x 128 tiles, quarters / halves of a 256 x 256 tile) run
// the last, partial wave of tiles on four / two times as many CUs.  Every output
// element sees the same k-steps and the same six MFMAs in the same order
// under either width, so the two are bit-identical.
// WN: waves along P (2 x WN waves).  WN = 2: 4 waves, one per SIMD, 128 x 32 NB
// each (DOL_SPLIT3_WAVES=4, and the narrow tail tiles); WN = 4 (with NB = 2, the
// default for 256 x 256 tiles): 8 waves, two per SIMD, 128 x 64 each, so one
// wave's LDS-DMA issue and fragment reads overlap the other's MFMAs.
template <int PROBE, bool FX, int NB = 4, int WN = 2>
__global__ __launch_bounds__(128 * WN) __attribute__((amdgpu_waves_per_eu(WN / 2, WN / 2)))
void dense_split3_kernel(const uint8_t* __restrict__ WA, const uint8_t* __restrict__ XB, float* __restrict__ Y,
                         int64_t ldy, int M, int64_t P, int64_t Mp, int64_t Pp, int n_stages, int n_mt,
                         int64_t n_pt, int64_t tiles_per_xcd, int group_m, const float* __restrict__ X,
                         int64_t ldx, int K, int64_t pread, int64_t t_base, int64_t t_end) {
  static_assert((WN == 2 && (NB == 4 || ((NB == 1 || NB == 2) && !FX && PROBE == 0))) ||
                    (WN == 4 && NB == 2 && !FX),
                "tiles: 256 x 256 (4 or 8 waves) or narrow split-pass tiles");
  constexpr int kWaves = 2 * WN;
  constexpr int BN = 32 * NB * WN;                         // tile width along P
  constexpr int kParts = kTile / BN;                       // narrow tiles per 256-wide tile
  constexpr int kStage = FX ? kStageFX : kOpStage + 2 * BN * kRec;
  constexpr int kDmaTot = FX ? 4 * kDmaFX : 24 + 3 * BN / 32;  // 1-KiB DMA pieces per stage
  constexpr int kDma = (kDmaTot + kWaves - 1) / kWaves;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  int64_t t;
  int quarter = 0;
  if constexpr (kParts == 1) {
    const int64_t j = blockIdx.x >> 3;
    t = (blockIdx.x & 7) * tiles_per_xcd + j;
    if (j >= tiles_per_xcd || t >= t_end) return;
  } else {
    t = t_base + blockIdx.x / kParts;
    quarter = blockIdx.x % kParts;
    if (t >= t_end) return;
  }
  const int64_t per_group = int64_t(group_m) * n_pt;
  const int g = int(t / per_group);
  const int first_m = g * group_m;
  const int gs = min(n_mt - first_m, group_m);
  const int64_t r = t - int64_t(g) * per_group;
  const int mt = first_m + int(r % gs);
  const int64_t pt = r / gs;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int h = lane >> 5, li = lane & 31;

  // stage s holds k-groups 2s, 2s+1 of both operands: [A kg0 | A kg1 | B kg0 | B kg1], 12 KiB each
  const uint8_t* srcA = WA + int64_t(mt) * kTile * kRec + lane * 16;
  const int64_t col0 = pt * kTile + quarter * BN;          // first P column of the tile
  const uint8_t* srcB = XB + col0 * kRec + lane * 16;
  const int64_t pitchA = Mp * kRec, pitchB = Pp * kRec;  // bytes per k-group
  auto issue = [&](int s) {
    if constexpr (PROBE == 1 || PROBE == 3) return;
    uint8_t* st = lds + (s % kStages) * kStage;
#pragma unroll
    for (int i = 0; i < kDma; ++i) {
      const int q = wave + kWaves * i;  // 1 KiB each (A records) / one fp32 row of 256 p (FX B)
      if (kDmaTot % kWaves && q >= kDmaTot) continue;
      if (!FX && kParts != 1 && q >= 24) {  // narrow B: 3 * NB pieces per k-group
        const int qb = q - 24, kgl = qb / (3 * NB), chunk = qb % (3 * NB);
        const uint8_t* src = srcB + (2 * int64_t(s) + kgl) * pitchB + chunk * 1024;
        __builtin_amdgcn_global_load_lds(DOL_GPTR(src), DOL_LPTR(st + q * 1024), 16, 0, 0);
        continue;
      }
      if (FX && q >= 24) {
        const int k = min(16 * s + (q - 24), K - 1);     // rows past K: masked after the read
        int64_t c = pt * kTile + lane * 4;
        if (c + 4 > pread) c = pread - 4;                // columns past P: masked after the read
        __builtin_amdgcn_global_load_lds(DOL_GPTR(X + int64_t(k) * ldx + c), DOL_LPTR(st + kOpStage + (q - 24) * kBPitch),
                                         16, 0, 0);
        continue;
      }
      const int op = q / 24, qq = q % 24, kgl = qq / 12, chunk = qq % 12;
      const int64_t kg = 2 * int64_t(s) + kgl;
      const uint8_t* src = (op == 0 ? srcA + kg * pitchA : srcB + kg * pitchB) + chunk * 1024;
      __builtin_amdgcn_global_load_lds(DOL_GPTR(src), DOL_LPTR(st + q * 1024), 16, 0, 0);
    }
  };

  f32x16 acc[4][NB];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  auto read_frags = [&](int s, bf16x8 (&fa)[4][3], bf16x8 (&fb)[NB][3]) {
    const uint8_t* st = lds + (s % kStages) * kStage;
    const uint8_t* sa = st + h * (kTile * kRec) + (wm * 128 + li) * kRec;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int p = 0; p < 3; ++p) fa[i][p] = *reinterpret_cast<const bf16x8*>(sa + i * 32 * kRec + 16 * p);
    if constexpr (FX) {
      const float* bs = reinterpret_cast<const float*>(st + kOpStage) + 8 * h * (kBPitch / 4);
      const bool edge = (pt == n_pt - 1) || (16 * s + 16 > K);  // wave-uniform
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pl = wn * 128 + i * 32 + li;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = bs[j * (kBPitch / 4) + pl];
        if (edge) {
          const bool pin = pt * kTile + pl < P;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (pin && 16 * s + 8 * h + j < K) ? v[j] : 0.f;
        }
        split8(v, fb[i][0], fb[i][1], fb[i][2]);
      }
    } else {
      const uint8_t* sb = st + kOpStage + h * (BN * kRec) + (wn * 32 * NB + li) * kRec;
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int p = 0; p < 3; ++p) fb[i][p] = *reinterpret_cast<const bf16x8*>(sb + i * 32 * kRec + 16 * p);
    }
  };
  // the six piece products of one 32x32x16 block, smallest first
  auto mfmas = [&](const bf16x8 (&fa)[4][3], const bf16x8 (&fb)[NB][3]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        f32x16 c = acc[a][b];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a][2], fb[b][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a][0], fb[b][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a][1], fb[b][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a][1], fb[b][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a][0], fb[b][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a][0], fb[b][0], c, 0, 0, 0);
        acc[a][b] = c;
      }
    __builtin_amdgcn_s_setprio(0);
  };
  auto barrier = [] {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // keep LDS reads below the barrier
  };

  issue(0);
  if (n_stages > 1) issue(1);
  for (int s = 0; s < n_stages; ++s) {
    wait_vmcnt_le<kDmaTot / kWaves>(s + 1 < n_stages);  // my DMA of stage s landed (the fewest any wave issues)
    barrier();                           // ... and every wave's; stage (s + 2) % 3 is free
    if (s + 2 < n_stages) issue(s + 2);
    if constexpr (PROBE == 2) continue;
    bf16x8 fa[4][3], fb[NB][3];
    read_frags(s, fa, fb);
    mfmas(fa, fb);
  }
  // C/D map (gfx950): col = lane & 31, row = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int64_t col = col0 + wn * 32 * NB + b * 32 + li;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = mt * kTile + wm * 128 + a * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (row < M && col < P && (PROBE < 3 || M < 0))  // probes 3/4 drop the stores (M < 0 never holds)
          __builtin_nontemporal_store(acc[a][b][e], Y + int64_t(row) * ldy + col);
      }
    }
}

// FX8 (r05): the in-register X split without redundancy, so the GEMM needs no
// X split pass (at 1024 x 101,770 the pass moved 1.04 GB in 0.18 ms of a
// 1.03 ms round).  Each of the tile's CB waves owns 32 output columns and ALL
// 256 rows (8 row blocks of 32).  Per k-step a wave
//   * stages ITS OWN 32 columns of the 16 X rows by LDS-DMA (2 KiB, two 1-KiB
//     pieces: 8 rows x 128 B each) -- only its own covering vmcnt orders its
//     reads of them, no barrier -- and the A records (the split W) with the
//     other waves (24 KiB per stage, behind the workgroup barrier);
//   * splits its 8 values per lane of the NEXT k-step (split8: the split
//     pass's bits) while this step's MFMAs run, so the split is off the MFMA
//     path (a first build split at the top of each step, behind the barrier:
//     both waves of a SIMD waited on the reads and the split together, 1.011
//     vs 1.045 ms for the split pass + record GEMM, profiles/r05h_split3_ab.jsonl);
//   * runs its 8 row blocks' six MFMAs, A fragments read block by block.
// The r01 FX kernel's 2 x 2 waves split every B value twice and four column
// blocks per wave.  Each output element sees the same k-steps and the same
// six MFMAs in the same order as dense_split3_kernel: bit-identical.
// RW x CW waves, wave (wm, wn) = rows [256 / RW * wm, + 256 / RW) x 32 columns
// at 32 wn: <1, 8> = 256 x 256 tiles, 8 waves (two per SIMD); <4, 2> = the
// 256 x 64 quarter tiles of the last, partial wave of tiles, also 8 waves
// (the four row-waves of a column each stage and split their own copy of
// its X slice, so no wave waits on another's B).
template <int RW, int CW>
struct Fx8Geom {
  static constexpr int kWaves = RW * CW;
  static constexpr int kRB = 8 / RW;                       // 32-row blocks per wave
  static constexpr int kCols = 32 * CW;                    // tile width
  static constexpr int kBWave = 16 * 128;                  // one wave's X slice per stage: 16 rows x 32 floats
  static constexpr int kStage = kOpStage + kWaves * kBWave;
  static constexpr int kDmaA = 24 / kWaves;                // A pieces per wave per stage
  static constexpr int kDma = kDmaA + 2;                   // + the wave's two B pieces
  static_assert(24 % kWaves == 0 && 8 % RW == 0, "A pieces / row blocks must split evenly over the waves");
};

template <int RW, int CW, int BATCH = 1>
__global__ __launch_bounds__(64 * RW * CW)
__attribute__((amdgpu_waves_per_eu(RW * CW >= 8 ? RW * CW / 4 : 1, RW * CW >= 8 ? RW * CW / 4 : 1)))
void dense_split3_fx8_kernel(const uint8_t* __restrict__ WA, float* __restrict__ Y, int64_t ldy, int M, int64_t P,
                             int64_t Mp, int n_stages, int n_mt, int64_t n_pt, int64_t tiles_per_xcd, int group_m,
                             const float* __restrict__ X, int64_t ldx, int K, int64_t pread, int64_t t_base,
                             int64_t t_end) {
  using Gm = Fx8Geom<RW, CW>;
  constexpr int kParts = 8 / CW;  // narrow tiles per 256-wide tile
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  int64_t t;
  int part = 0;
  if constexpr (kParts == 1) {
    const int64_t j = blockIdx.x >> 3;
    t = (blockIdx.x & 7) * tiles_per_xcd + j;
    if (j >= tiles_per_xcd || t >= t_end) return;
  } else {
    t = t_base + blockIdx.x / kParts;
    part = blockIdx.x % kParts;
    if (t >= t_end) return;
  }
  const int64_t per_group = int64_t(group_m) * n_pt;
  const int g = int(t / per_group);
  const int first_m = g * group_m;
  const int gs = min(n_mt - first_m, group_m);
  const int64_t r = t - int64_t(g) * per_group;
  const int mt = first_m + int(r % gs);
  const int64_t pt = r / gs;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / CW, wn = wave % CW;
  const int h = lane >> 5, li = lane & 31;
  const uint8_t* srcA = WA + int64_t(mt) * kTile * kRec + lane * 16;
  const int64_t pitchA = Mp * kRec;
  const int64_t col0 = pt * kTile + part * Gm::kCols + 32 * wn;  // this wave's first P column
  // B DMA: lane -> row (lane >> 3) of 8, 16 B at column 4 (lane & 7); past P: clamped, masked after the read
  int64_t cdma = col0 + 4 * (lane & 7);
  if (cdma + 4 > pread) cdma = pread - 4;
  const int drow = lane >> 3;
  uint8_t* const bwave = lds + kOpStage + wave * Gm::kBWave;  // + stage offset

  auto issue = [&](int s) {
    uint8_t* st = lds + (s % kStages) * Gm::kStage;
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // B first: a wave's wait for its B slice leaves its A pieces in flight
      const int k = min(16 * s + 8 * i + drow, K - 1);  // rows past K: clamped, masked after the read
      __builtin_amdgcn_global_load_lds(DOL_GPTR(X + int64_t(k) * ldx + cdma),
                                       DOL_LPTR(bwave + (s % kStages) * Gm::kStage + i * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < Gm::kDmaA; ++i) {  // A: k-group 2s + q / 12, 1-KiB piece q % 12 of the 256 rows' records
      const int q = wave + Gm::kWaves * i;
      const uint8_t* src = srcA + (2 * int64_t(s) + q / 12) * pitchA + (q % 12) * 1024;
      __builtin_amdgcn_global_load_lds(DOL_GPTR(src), DOL_LPTR(st + q * 1024), 16, 0, 0);
    }
  };
  const bool col_ok = col0 + li < P;
  // the B fragments of step s from this wave's slice (k = 16 s + 8 h + j of column li)
  auto read_b = [&](int s, float (&v)[8]) {
    const float* bs = reinterpret_cast<const float*>(bwave + (s % kStages) * Gm::kStage + 8 * h * 128) + li;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bs[j * 32];
  };
  auto split_b = [&](int s, float (&v)[8], bf16x8 (&fb)[3]) {
    if (!col_ok || 16 * s + 16 > K) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (col_ok && 16 * s + 8 * h + j < K) ? v[j] : 0.f;
    }
    split8(v, fb[0], fb[1], fb[2]);
  };

  f32x16 acc[Gm::kRB];
#pragma unroll
  for (int a = 0; a < Gm::kRB; ++a)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[a][e] = 0.f;

  issue(0);
  if (n_stages > 1) issue(1);
  bf16x8 fb[3];
  // my B slice of step 0 landed (step 0's A pieces and step 1 may still fly)
  if (n_stages > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Gm::kDmaA + Gm::kDma) : "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Gm::kDmaA) : "memory");
  {
    float v0[8];
    read_b(0, v0);
    split_b(0, v0, fb);
  }
  for (int s = 0; s < n_stages; ++s) {
    wait_vmcnt_le<Gm::kDma>(s + 1 < n_stages);  // my DMA of step s landed
    __builtin_amdgcn_s_barrier();               // ... and every wave's A pieces; stage (s + 2) % 3 is free
    asm volatile("" ::: "memory");
    if (s + 2 < n_stages) issue(s + 2);
    const uint8_t* sa = lds + (s % kStages) * Gm::kStage + h * (kTile * kRec) + (wm * 32 * Gm::kRB + li) * kRec;
    bf16x8 fn[3];
    float vn[8];  // the next step's X values: read now, split under this step's MFMAs
    if (s + 1 < n_stages) {
      // my B slice of step s + 1 landed: its A pieces and (if issued) step s + 2 may still fly
      if (s + 2 < n_stages) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Gm::kDmaA + Gm::kDma) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Gm::kDmaA) : "memory");
      read_b(s + 1, vn);
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    // A fragments: BATCH = 1 double-buffers single blocks (block a + 1's reads
    // in flight while block a's MFMAs issue); BATCH > 1 reads BATCH blocks'
    // fragments at once and then runs their MFMAs (one LDS wait per batch).
    // The scheduler otherwise sinks each read to its use and waits
    // lgkmcnt(0) before every block's six MFMAs: sched_barrier keeps the
    // reads where they are written.
    constexpr int NQ = BATCH == 1 ? 2 : BATCH;
    bf16x8 fq[NQ][3];
    auto read_block = [&](int a, bf16x8 (&f)[3]) {
#pragma unroll
      for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const bf16x8*>(sa + a * 32 * kRec + 16 * p);
    };
    if constexpr (BATCH == 1) read_block(0, fq[0]);
#pragma unroll
    for (int a = 0; a < Gm::kRB; ++a) {
      if constexpr (BATCH == 1) {
        if (a + 1 < Gm::kRB) read_block(a + 1, fq[(a + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
      } else if (a % BATCH == 0) {
#pragma unroll
        for (int u = 0; u < BATCH; ++u) read_block(a + u, fq[u]);
        __builtin_amdgcn_sched_barrier(0);
      }
      const bf16x8 (&fa)[3] = fq[BATCH == 1 ? (a & 1) : (a % BATCH)];
      f32x16 c = acc[a];  // the six piece products of one 32x32x16 block, smallest first (as dense_split3_kernel)
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[0], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[2], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[0], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[1], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], c, 0, 0, 0);
      acc[a] = c;
      if (a == (Gm::kRB > 1 ? 1 : 0) && s + 1 < n_stages) split_b(s + 1, vn, fn);  // under this step's MFMAs
    }
    __builtin_amdgcn_s_setprio(0);
    if (s + 1 < n_stages) {
#pragma unroll
      for (int p = 0; p < 3; ++p) fb[p] = fn[p];
    }
  }
  // C/D map (gfx950): col = lane & 31, row = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)
  const int64_t col = col0 + li;
#pragma unroll
  for (int a = 0; a < Gm::kRB; ++a)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = mt * kTile + wm * 32 * Gm::kRB + a * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (row < M && col < P) __builtin_nontemporal_store(acc[a][e], Y + int64_t(row) * ldy + col);
    }
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

struct Split3Geom {
  int64_t Mp, Pp, Kg, bytesA, bytesB;
};

inline Split3Geom geom(int32_t M, int32_t K, int64_t P) {
  Split3Geom g;
  g.Mp = cdiv(M, kTile) * kTile;
  g.Pp = cdiv(P, kTile) * kTile;
  g.Kg = cdiv(K, 16) * 2;
  g.bytesA = g.Kg * g.Mp * kRec;
  g.bytesB = g.Kg * g.Pp * kRec;
  return g;
}

// The in-register X split (FX kernel, opt-in with DOL_SPLIT3_FUSE_X) needs whole
// 16-B pieces of X rows: rows 16-B aligned, ldx % 4 == 0 and readable up to
// round_up(P, 4) floats — always so when P % 4 == 0, and asserted by the caller
// with DOL_SPLIT3_X_ROWS_PADDED.  It needs no X workspace (0.40 vs 5.4 GB at
// 8192 x 101,770) but runs slower: 68.8 vs 54.4 ms there, 1.45 vs 1.43 ms at
// 1024 agents (each B value is split by both row-waves, 32 ds_read_b32 + ~250
// VALU per stage and wave beside the 96 MFMAs) — the split pass is the default.
inline bool fused_x_ok(const float* X, int64_t ldx, int64_t P, int flags) {
  const bool aligned = reinterpret_cast<uintptr_t>(X) % 16 == 0 && ldx % 4 == 0;
  return (flags & DOL_SPLIT3_FUSE_X) && aligned && P >= 4 && (P % 4 == 0 || (flags & DOL_SPLIT3_X_ROWS_PADDED));
}


// FXW (r05): the split-pass kernel's 2 x 4 waves and fragment reads (12 A + 6
// B ds_read_b128 per wave and k-step, the fewest of any layout), with the B
// records made in the kernel instead of by the split pass.  Each of the 512
// lanes owns one (8 k x 1 column) record of a k-step; each wave stages the X
// rows of its own 64 records by LDS-DMA (8 rows x 256 B, two 1-KiB pieces,
// two stages), so after its own vmcnt wait -- no barrier -- it reads its 8
// values (ds_read_b32, conflict-free), splits them under the current step's
// MFMAs (split8: the split pass's bits) and writes the 48-B record into the
// other half of a double-buffered B stage, which every wave reads after the
// next step's barrier.  LDS: 3 x 24 KiB of A + 2 x 16 KiB of X + 2 x 24 KiB
// of B records = 152 KiB.  Same k-steps, same fragments, same six MFMAs per
// block in the same order as dense_split3_kernel: bit-identical.
constexpr int kFxwX = 16 * 1024;                                         // one X stage: 8 waves x 8 rows x 256 B
constexpr int kFxwLds = kStages * kOpStage + 2 * kFxwX + 2 * kOpStage;    // 152 KiB
static_assert(kFxwLds <= 160 * 1024, "LDS budget");

// the split after row block 1's MFMAs: after 0 / 2 / 3 measured 1-2 % slower, before the
// MFMAs (in the barrier bubble, X reads ahead of the fragment reads) 4 % slower
constexpr int kFxwSplitAt = 1;

__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
void dense_split3_fxw_kernel(const uint8_t* __restrict__ WA, float* __restrict__ Y, int64_t ldy, int M, int64_t P,
                             int64_t Mp, int n_stages, int n_mt, int64_t n_pt, int64_t tiles_per_xcd, int group_m,
                             const float* __restrict__ X, int64_t ldx, int K, int64_t pread, int64_t t_base,
                             int64_t t_end) {
  (void)t_base;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int64_t jt = blockIdx.x >> 3;
  const int64_t t = (blockIdx.x & 7) * tiles_per_xcd + jt;
  if (jt >= tiles_per_xcd || t >= t_end) return;
  const int64_t per_group = int64_t(group_m) * n_pt;
  const int g = int(t / per_group);
  const int first_m = g * group_m;
  const int gs = min(n_mt - first_m, group_m);
  const int64_t r = t - int64_t(g) * per_group;
  const int mt = first_m + int(r % gs);
  const int64_t pt = r / gs;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int h = lane >> 5, li = lane & 31;
  const uint8_t* srcA = WA + int64_t(mt) * kTile * kRec + lane * 16;
  const int64_t pitchA = Mp * kRec;
  const int64_t col0 = pt * kTile;
  // X DMA: each wave stages the rows of its own records (k-group rkg, 64 columns), so the
  // split needs only the wave's own vmcnt, no barrier; lane: row lane / 16, 16 B at column 4 (lane % 16)
  int64_t cdma = col0 + ((wave & 3) << 6) + 4 * (lane & 15);  // past P: clamped, masked after the read
  if (cdma + 4 > pread) cdma = pread - 4;
  uint8_t* const ringA = lds;
  uint8_t* const ringX = lds + kStages * kOpStage;
  uint8_t* const ringB = ringX + 2 * kFxwX;
  // this lane's record of every k-step: k-group rkg of the step, tile column rp
  const int rkg = wave >> 2, rp = ((wave & 3) << 6) + lane;
  const bool cok = col0 + rp < P;
  uint8_t* const rec = ringB + rkg * (kTile * kRec) + rp * kRec;

  // step group s, in issue order: X(s) 2 DMAs, A(s) 3 DMAs per wave
  auto issue = [&](int s) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // rows 8 rkg + 4 i .. + 3 of this wave's 64 columns: 4 x 256 B
      const int k = min(16 * s + 8 * rkg + 4 * i + (lane >> 4), K - 1);  // rows past K: clamped, masked after the read
      __builtin_amdgcn_global_load_lds(DOL_GPTR(X + int64_t(k) * ldx + cdma),
                                       DOL_LPTR(ringX + (s & 1) * kFxwX + wave * 2048 + i * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int q = wave + 8 * i;
      const uint8_t* src = srcA + (2 * int64_t(s) + q / 12) * pitchA + (q % 12) * 1024;
      __builtin_amdgcn_global_load_lds(DOL_GPTR(src), DOL_LPTR(ringA + (s % kStages) * kOpStage + q * 1024), 16, 0, 0);
    }
  };
  auto read_x = [&](int s, float (&v)[8]) {  // step s's record of this lane from X stage s % 2 (row j at j * 256 B)
    const float* xs = reinterpret_cast<const float*>(ringX + (s & 1) * kFxwX + wave * 2048) + lane;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = xs[j * 64];
  };
  auto split_x = [&](int s, float (&v)[8]) {  // ... split into B stage s % 2
    if (!cok || 16 * s + 16 > K) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (cok && 16 * s + 8 * rkg + j < K) ? v[j] : 0.f;
    }
    bf16x8 q0, q1, q2;
    split8(v, q0, q1, q2);
    uint8_t* d = rec + (s & 1) * kOpStage;
    *reinterpret_cast<bf16x8*>(d) = q0;
    *reinterpret_cast<bf16x8*>(d + 16) = q1;
    *reinterpret_cast<bf16x8*>(d + 32) = q2;
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  issue(0);
  if (n_stages > 1) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // my X(0) rows landed (A(0) and group 1 may fly)
  } else {
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  }
  {
    float v0[8];
    read_x(0, v0);
    split_x(0, v0);
  }
  for (int s = 0; s < n_stages; ++s) {
    // A(s) landed: after it only group s + 1 may fly.  lgkmcnt(0): this wave's
    // record writes and fragment reads are done before the barrier
    if (s + 1 < n_stages) asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's A(s) and B records of s are in LDS
    asm volatile("" ::: "memory");
    if (s + 2 < n_stages) issue(s + 2);  // X slot s % 2 (my rows, split during s - 1), A slot (s + 2) % 3: free
    const uint8_t* sa = ringA + (s % kStages) * kOpStage + h * (kTile * kRec) + (wm * 128 + li) * kRec;
    const uint8_t* sb = ringB + (s & 1) * kOpStage + h * (kTile * kRec) + (wn * 64 + li) * kRec;
    bf16x8 fa[4][3], fb[2][3];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int p = 0; p < 3; ++p) fa[i][p] = *reinterpret_cast<const bf16x8*>(sa + i * 32 * kRec + 16 * p);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int p = 0; p < 3; ++p) fb[i][p] = *reinterpret_cast<const bf16x8*>(sb + i * 32 * kRec + 16 * p);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < 4; ++a) {
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        f32x16 c = acc[a][b];  // six piece products, smallest first (as dense_split3_kernel)
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a][2], fb[b][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a][0], fb[b][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a][1], fb[b][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a][1], fb[b][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a][0], fb[b][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a][0], fb[b][0], c, 0, 0, 0);
        acc[a][b] = c;
      }
      if (a == kFxwSplitAt && s + 1 < n_stages) {  // step s + 1's record, under this step's MFMAs
        // my X(s + 1) rows landed: after them A(s + 1) and group s + 2 may fly
        if (s + 2 < n_stages) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        float xv[8];
        read_x(s + 1, xv);
        split_x(s + 1, xv);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  }
  // C/D map (gfx950): col = lane & 31, row = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int64_t col = col0 + wn * 64 + b * 32 + li;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = mt * kTile + wm * 128 + a * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (row < M && col < P) __builtin_nontemporal_store(acc[a][b][e], Y + int64_t(row) * ldy + col);
      }
    }
}

}  // namespace

extern "C" int64_t dol_mix_dense_split3_workspace_bytes(int32_t M, int32_t K, int64_t P, int flags) {
  if (M <= 0 || K <= 0 || P <= 0 || P > dol::kMaxDim) return 0;
  const Split3Geom g = geom(M, K, P);
  // FUSE_X + X_ROWS_PADDED promise the fused path (given an aligned X): W pieces only
  const bool fused = (flags & DOL_SPLIT3_FUSE_X) && (flags & DOL_SPLIT3_X_ROWS_PADDED) && P >= 4;
  return fused ? g.bytesA : g.bytesA + g.bytesB;
}

extern "C" int dol_mix_dense_split3_f32(const float* W, int64_t ldw, const float* X, int64_t ldx, float* Y,
                                        int64_t ldy, int32_t M, int32_t K, int64_t P, void* work,
                                        int64_t work_bytes, int flags, hipStream_t s) {
  DOL_DIMS_OK("dol_mix_dense_split3_f32", ldw, ldx, ldy, P, work_bytes);
  using dol::fail;
  if (M < 0 || K < 0 || P < 0) return fail(DOL_EINVAL, "dol_mix_dense_split3_f32: negative size");
  if (M == 0 || P == 0) return DOL_OK;
  if (!Y || (K > 0 && (!W || !X))) return fail(DOL_EINVAL, "dol_mix_dense_split3_f32: null pointer");
  if (ldy < P || (K > 0 && (ldw < K || ldx < P))) return fail(DOL_EINVAL, "dol_mix_dense_split3_f32: ld too small");
  if (X == Y || W == Y) return fail(DOL_EINVAL, "dol_mix_dense_split3_f32: Y aliases an input");
  if (K == 0) return hipMemset2DAsync(Y, ldy * 4, 0, P * 4, M, s) == hipSuccess ? DOL_OK
                     : fail(DOL_EINVAL, "dol_mix_dense_split3_f32: memset failed");
  const Split3Geom g = geom(M, K, P);
  const bool fx = fused_x_ok(X, ldx, P, flags);
  const int64_t need = fx ? g.bytesA : g.bytesA + g.bytesB;
  if (!work || work_bytes < need)
    return fail(DOL_EINVAL, "dol_mix_dense_split3_f32: workspace %lld bytes, need %lld",
                static_cast<long long>(work_bytes), static_cast<long long>(need));
  if (reinterpret_cast<uintptr_t>(work) % 256) return fail(DOL_EINVAL, "dol_mix_dense_split3_f32: workspace not 256-B aligned");
  uint8_t* wa = static_cast<uint8_t*>(work);
  uint8_t* xb = fx ? nullptr : wa + g.bytesA;
  if (!(flags & DOL_SPLIT3_W_READY)) {
    const int64_t n = g.Mp * g.Kg;
    if (cdiv(n, 256) >= (int64_t(1) << 32)) return fail(DOL_EINVAL, "dol_mix_dense_split3_f32: W too large");
    hipLaunchKernelGGL(split3_rows_kernel, dim3(static_cast<unsigned>(cdiv(n, 256))), dim3(256), 0, s, W, ldw, M, K,
                       static_cast<int>(g.Mp), static_cast<int>(g.Kg), wa);
  }
  if (!fx) {
    const int64_t n = g.Pp * g.Kg;
    if (cdiv(n, 256) >= (int64_t(1) << 32)) return fail(DOL_EINVAL, "dol_mix_dense_split3_f32: X too large");
    static const bool per_column = getenv("DOL_SPLIT3_XPASS1") != nullptr;  // diagnostic: the r01 pass
    const bool vec = reinterpret_cast<uintptr_t>(X) % 16 == 0 && ldx % 4 == 0;
    if (per_column)
      hipLaunchKernelGGL(split3_cols_kernel, dim3(static_cast<unsigned>(cdiv(n, 256))), dim3(256), 0, s, X, ldx, K, P,
                         g.Pp, static_cast<int>(g.Kg), xb);
    else if (vec)
      hipLaunchKernelGGL(split3_cols4_kernel<true>, dim3(static_cast<unsigned>(cdiv(n / 4, 256))), dim3(256), 0, s, X,
                         ldx, K, P, g.Pp, static_cast<int>(g.Kg), xb);
    else
      hipLaunchKernelGGL(split3_cols4_kernel<false>, dim3(static_cast<unsigned>(cdiv(n / 4, 256))), dim3(256), 0, s, X,
                         ldx, K, P, g.Pp, static_cast<int>(g.Kg), xb);
  }
  // diagnostics knobs (tools/gpu_dense_probe.sh); read once per process
  static const int probe = [] { const char* e = getenv("DOL_SPLIT3_PROBE"); return e ? atoi(e) : 0; }();
  // 8 waves (two per SIMD) unless DOL_SPLIT3_WAVES=4: 1.07-1.10 vs 1.11-1.12 ms at
  // 1024 x 101,770, 54.4-54.5 vs 56.2 ms at 8192 (profiles/r02_split3_waves.txt);
  // same bits (tests/test_kernels_gpu.py split3 tests under both)
  static const bool waves8 = [] { const char* e = getenv("DOL_SPLIT3_WAVES"); return !(e && atoi(e) == 4); }();
  static const int group_m = [] {
    const char* e = getenv("DOL_SPLIT3_GROUP_M");
    return e && atoi(e) > 0 ? atoi(e) : kGroupM;
  }();
  const int n_mt = static_cast<int>(g.Mp / kTile);
  const int64_t n_pt = g.Pp / kTile;
  const int64_t n_tiles = int64_t(n_mt) * n_pt;
  // Tail: when the last wave of 256 x 256 tiles would fill at most a quarter
  // (a half) of the CUs, those tiles run as 256 x 64 quarters (256 x 128
  // halves) in a second launch: 1024 agents x 101,770 = 1592 tiles = 6 x 256 +
  // 56 -> quarters, 2048 agents = 12 x 256 + 112 -> halves.  DOL_SPLIT3_CUS overrides the
  // CU count (tests force the tail path at small sizes; 0 disables it).
  static const int n_cu = [] {
    int dev = 0, cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cu = 0;
    return cu;
  }();
  const char* cus_env = getenv("DOL_SPLIT3_CUS");
  const int64_t cus = cus_env && *cus_env ? atoi(cus_env) : n_cu;
  const int64_t tail = cus > 0 ? n_tiles % cus : 0;
  // FUSE_X runs dense_split3_fx8_kernel (r05) unless DOL_SPLIT3_FX=1 asks for the r01 in-register kernel
  static const bool fx_old = [] { const char* e = getenv("DOL_SPLIT3_FX"); return e && atoi(e) == 1; }();
  const bool fx8 = fx && !fx_old && probe == 0;
  const bool fx8_tail = fx8 && n_tiles > cus && tail > 0 && 4 * tail <= cus;  // 256 x 64 quarters, one CU each
  const bool narrow_tail = (!fx && probe == 0 && n_tiles > cus && tail > 0 && 2 * tail <= cus) || fx8_tail;
  const int nb_tail = 4 * tail <= cus ? 1 : 2;
  const int64_t t_main = narrow_tail ? n_tiles - tail : n_tiles;
  const int64_t tiles_per_xcd = cdiv(t_main, 8);
  if (8 * tiles_per_xcd >= (int64_t(1) << 32) || 4 * tail >= (int64_t(1) << 32))
    return fail(DOL_EINVAL, "dol_mix_dense_split3_f32: too many tiles");
  const int64_t pread = (P % 4 == 0) ? P : (P + 3) / 4 * 4;
  auto launch = [&](auto kern, int lds, int64_t grid, int64_t t_base, int64_t t_end, int threads = 256) {
    // > 64 KiB of dynamic LDS: set on every call (cheap), so every device of the process gets it
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(grid)), dim3(threads), lds, s, wa, xb, Y, ldy, M,
                       P, g.Mp, g.Pp, static_cast<int>(g.Kg / 2), n_mt, n_pt, tiles_per_xcd, group_m, X, ldx, K,
                       pread, t_base, t_end);
  };
  const int64_t grid = 8 * tiles_per_xcd;
  if (fx8) {
    auto launch8 = [&](auto kern, int lds, int64_t grd, int64_t t_base, int64_t t_end, int threads) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(grd)), dim3(threads), lds, s, wa, Y, ldy, M, P, g.Mp,
                         static_cast<int>(g.Kg / 2), n_mt, n_pt, tiles_per_xcd, group_m, X, ldx, K, pread, t_base,
                         t_end);
    };
    // DOL_SPLIT3_FX8_BATCH (read per call; A fragment batching, same bits): 1 (default), 2 or 4
    const char* be = getenv("DOL_SPLIT3_FX8_BATCH");
    const int batch = be ? atoi(be) : 1;
    // main tiles: dense_split3_fxw_kernel (r05; 864-872 vs 884-887 us for FX8's 1 x 8 layout at
    // 1024 x 101,770, profiles/r05x_split3_fxw_ab.jsonl) unless DOL_SPLIT3_FXW=0 (read per call; same bits)
    const char* we = getenv("DOL_SPLIT3_FXW");
    if (!(we && atoi(we) == 0)) launch8(dense_split3_fxw_kernel, kFxwLds, grid, 0, t_main, 512);
    else if (batch == 4) launch8(dense_split3_fx8_kernel<1, 8, 4>, kStages * Fx8Geom<1, 8>::kStage, grid, 0, t_main, 512);
    else if (batch == 2) launch8(dense_split3_fx8_kernel<1, 8, 2>, kStages * Fx8Geom<1, 8>::kStage, grid, 0, t_main, 512);
    else launch8(dense_split3_fx8_kernel<1, 8>, kStages * Fx8Geom<1, 8>::kStage, grid, 0, t_main, 512);
    // the tail's quarter tiles: DOL_SPLIT3_FX8_TAIL (read per call; same bits) 8 = 4 x 2 waves (default), 4 = 2 x 2
    const char* te = getenv("DOL_SPLIT3_FX8_TAIL");
    if (fx8_tail && te && atoi(te) == 4)
      launch8(dense_split3_fx8_kernel<2, 2>, kStages * Fx8Geom<2, 2>::kStage, 4 * tail, t_main, n_tiles, 256);
    else if (fx8_tail)
      launch8(dense_split3_fx8_kernel<4, 2>, kStages * Fx8Geom<4, 2>::kStage, 4 * tail, t_main, n_tiles, 512);
    return dol::check_launch("dol_mix_dense_split3_f32");
  }
  if (fx) {
    if (probe == 1) launch(dense_split3_kernel<1, true>, kStages * kStageFX, grid, 0, t_main);
    else if (probe == 2) launch(dense_split3_kernel<2, true>, kStages * kStageFX, grid, 0, t_main);
    else launch(dense_split3_kernel<0, true>, kStages * kStageFX, grid, 0, t_main);
  } else {
    if (probe == 1) launch(dense_split3_kernel<1, false>, kLds, grid, 0, t_main);
    else if (probe == 2) launch(dense_split3_kernel<2, false>, kLds, grid, 0, t_main);
    else if (probe == 3) launch(dense_split3_kernel<3, false>, kLds, grid, 0, t_main);
    else if (probe == 4) launch(dense_split3_kernel<4, false>, kLds, grid, 0, t_main);
    else if (waves8 && probe == 0) launch(dense_split3_kernel<0, false, 2, 4>, kLds, grid, 0, t_main, 512);
    else if (waves8 && probe == 5) launch(dense_split3_kernel<1, false, 2, 4>, kLds, grid, 0, t_main, 512);
    else if (waves8 && probe == 6) launch(dense_split3_kernel<2, false, 2, 4>, kLds, grid, 0, t_main, 512);
    else if (waves8 && probe == 7) launch(dense_split3_kernel<4, false, 2, 4>, kLds, grid, 0, t_main, 512);
    else launch(dense_split3_kernel<0, false>, kLds, grid, 0, t_main);
  }
  if (narrow_tail && nb_tail == 1)
    launch(dense_split3_kernel<0, false, 1>, kStages * (kOpStage + 2 * 64 * kRec), 4 * tail, t_main, n_tiles);
  else if (narrow_tail)
    launch(dense_split3_kernel<0, false, 2>, kStages * (kOpStage + 2 * 128 * kRec), 2 * tail, t_main, n_tiles);
  return dol::check_launch("dol_mix_dense_split3_f32");
}
