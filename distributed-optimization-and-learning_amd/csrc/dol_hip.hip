// dol_hip.hip — gfx950 kernels and the C-ABI of include/dol_hip.h.
//
// Build (see csrc/Makefile):  hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared
// -ffp-contract=off is load-bearing: the reference (torch CPU) rounds every
// product and every sum separately in the mixing / dual / prox arithmetic, so
// the only fused multiply-add in this file is the explicit __builtin_fmaf of
// the SGD parameter update (ATen's vectorised add_(d, alpha=-lr) is an FMA).
//
// Layout: agent k's parameter vector is row k of a row-major fp32 matrix
// with leading dimension ld (elements).  Columns are streamed 16 B per lane
// (f4) when every row base is 16-B aligned; otherwise, and for the
// P % 4 tail, the same kernels run on scalar columns.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdarg.h>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <unordered_map>
#include <type_traits>

#include "../../include/dol_hip.h"
#include "dol_common.h"

// ----------------------------------------------------------------------------
// error plumbing (shared with the other translation units via dol_common.h)
// ----------------------------------------------------------------------------
namespace dol {
thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    return fail(-static_cast<int>(e), "%s: launch failed: %s", what, hipGetErrorString(e));
  }
  g_err[0] = '\0';
  return DOL_OK;
}
}  // namespace dol

namespace {
using dol::check_launch;
using dol::fail;
using dol::g_err;

constexpr int kThreads = 256;            // 4 waves of 64
constexpr int64_t kMaxBlocks = int64_t(1) << 24;
constexpr int kRingStepsVariants = 5;  // highest dol_mix_ring_steps_ex_f32 variant

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  return atoi(v);
}

// ----------------------------------------------------------------------------
// vector helpers: the same kernel body runs on float (tail / unaligned) and
// f4 (main stream).  All arithmetic is explicit per lane so that each
// product and sum rounds once, exactly as the reference's torch CPU ops.
// ----------------------------------------------------------------------------
typedef float f4 __attribute__((ext_vector_type(4)));  // native 16-B vector (nontemporal builtins need it)
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

template <typename V> struct Vec;
template <> struct Vec<float> {
  static constexpr int W = 1;
};
template <> struct Vec<f4> {
  static constexpr int W = 4;
};

__device__ __forceinline__ float axpy0(float wp, float a, float wn, float b) {
  // ((+0 + wp*a) + wn*b) with every operation rounded (no contraction)
  float acc = 0.0f;
  acc = acc + wp * a;
  acc = acc + wn * b;
  return acc;
}
__device__ __forceinline__ f4 axpy0(float wp, f4 a, float wn, f4 b) {
  return f4{axpy0(wp, a.x, wn, b.x), axpy0(wp, a.y, wn, b.y),
            axpy0(wp, a.z, wn, b.z), axpy0(wp, a.w, wn, b.w)};
}
// (ring_steps_kernel with 8-B lanes and R = 22-54: 11.25-11.65 ms vs 11.24-11.27
// for f4 / R = 22 at eps = 5, 8192 x 2^20, same box: kept f4)
__device__ __forceinline__ float fmac(float acc, float a, float x) { return acc + a * x; }
__device__ __forceinline__ f4 fmac(f4 acc, float a, f4 x) {
  return f4{acc.x + a * x.x, acc.y + a * x.y, acc.z + a * x.z, acc.w + a * x.w};
}
__device__ __forceinline__ float vzero(float) { return 0.0f; }
__device__ __forceinline__ f4 vzero(f4) { return f4{0.f, 0.f, 0.f, 0.f}; }
__device__ __forceinline__ float vadd(float a, float b) { return a + b; }
__device__ __forceinline__ f4 vadd(f4 a, f4 b) {
  return f4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w};
}
__device__ __forceinline__ float vdiv(float a, float s) { return a / s; }
__device__ __forceinline__ f4 vdiv(f4 a, float s) {
  return f4{a.x / s, a.y / s, a.z / s, a.w / s};
}

// ----------------------------------------------------------------------------
// Mixing epilogues.  NoEpi: Y = W X (the gossip round).  DgdEpi: then `steps`
// local momentum-SGD iterations per agent on a separable synthetic loss —
// BASELINE config 3, decentralised gradient descent in the reference's round
// order (DIST/simulators.py:147-162: consensus, then local_update with the
// optimizer of DIST/clients.py:43-49) — so a round streams X, the targets and
// the momentum once.  Rounding as oracle_dgd_local_f32:
//   OBJ 0 least squares  g = x - t;   OBJ 1 logistic  g = -t / (1 + exp(t x))
//   MODE 0 plain SGD; 1 momentum, first step (buf = g); 2 momentum (buf = buf*mom + g)
//   x = fma(-lr, d, x)
// load() is issued with the mixing loads; apply() runs after the mix.
// ----------------------------------------------------------------------------
struct Empty {};
struct NoEpi {
  template <typename V> __device__ __forceinline__ Empty load(int, int64_t) const { return {}; }
  template <typename V> __device__ __forceinline__ V apply(V y, Empty, int, int64_t) const { return y; }
};

template <typename V> struct DgdState { V t, b; };

template <int OBJ, int MODE>
struct DgdEpi {
  const float* __restrict__ T; int64_t ldt;
  float* __restrict__ M; int64_t ldm;
  float neg_lr, mom;
  int steps;
  // Target / momentum rows are read once: buffer loads with the nontemporal
  // policy (aux 3 = sc0 nt), so they do not push the X halo rows -- re-read by
  // the next row group's tile, 1024 workgroups later -- out of the XCD's L2.
  // With plain loads the ring round read 1.16x its bytes (14.97 vs 12.88 GB
  // at 1024 x 2^20, least squares + momentum) and ran 3.58-3.59 ms; with these
  // 12.90 GB = 1.00x and 3.44-3.45 ms (profiles/r06f_dgd_epi_policy.jsonl; sc0
  // sc1 without nt: no change).  DOL_DGD_EPI_NT=0 restores plain loads, 1 the
  // compiler's nontemporal global loads.
  int nt;

  template <typename V> __device__ __forceinline__ V ld(const float* row, int64_t cf) const {
    const V* p = reinterpret_cast<const V*>(row + cf);
    if constexpr (sizeof(V) == 16) {
      if (nt == 3) {
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(row), 0, 0x7ffffff0, 0x00020000);
        return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(rs, uint32_t(cf) * 4u, 0, 3));
      }
      if (nt == 1) return __builtin_nontemporal_load(p);
    }
    return *p;
  }
  template <typename V> __device__ __forceinline__ DgdState<V> load(int r, int64_t cf) const {
    DgdState<V> st;
    st.t = ld<V>(T + int64_t(r) * ldt, cf);
    if constexpr (MODE == 2) st.b = ld<V>(M + int64_t(r) * ldm, cf);
    else st.b = vzero(V{});
    return st;
  }
  __device__ __forceinline__ float local(float x, float t, float& b) const {
    for (int s = 0; s < steps; ++s) {
      float g;
      if constexpr (OBJ == 0) g = x - t;
      else g = -t / (1.0f + expf(t * x));
      float d = g;
      if constexpr (MODE != 0) {
        if (MODE == 1 && s == 0) b = g;
        else b = b * mom + g;
        d = b;
      }
      x = __builtin_fmaf(neg_lr, d, x);
    }
    return x;
  }
  template <typename V> __device__ __forceinline__ V apply(V y, DgdState<V> st, int r, int64_t cf) const {
    if constexpr (Vec<V>::W == 1) {
      y = local(y, st.t, st.b);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float bj = st.b[j];
        y[j] = local(y[j], st.t[j], bj);
        st.b[j] = bj;
      }
    }
    if constexpr (MODE != 0) __builtin_nontemporal_store(st.b, reinterpret_cast<V*>(M + int64_t(r) * ldm + cf));
    return y;
  }
};

template <typename V, bool NT>
__device__ __forceinline__ V ldv(const V* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <typename V, bool NT>
__device__ __forceinline__ void stv(V* p, V v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// ----------------------------------------------------------------------------
// Ring mix: one workgroup = one column tile (256 lanes x V = 4 KiB of a row)
// x R consecutive agent rows.  The three-point stencil along the agent axis is
// carried in a register window; PF rows are loaded one iteration ahead.
// Measured on MI355X (tools/membench*.hip, 8192 x 2^20): short-lived tiles win
// — R = 4 with all R+2 loads issued up front (PF >= R), plain loads and
// nontemporal stores reach 6.14 TB/s against a 6.26 TB/s flat-copy ceiling,
// while R = 64 long-lived tiles stay near 5.1-5.4.  The halo rows (2 per
// tile) are re-read from L2: vertically adjacent tiles are n_col_tiles
// blocks apart (a multiple of 8 -> same XCD) and co-resident.
// ----------------------------------------------------------------------------
template <typename V, int PF, bool NT_LOAD, bool NT_STORE, class Epi = NoEpi>
__global__ __launch_bounds__(kThreads) void ring_mix_kernel(
    const float* __restrict__ X, int64_t ldx, float* __restrict__ Y, int64_t ldy,
    int n_rows, int64_t c_off, int64_t ncols_v, int64_t n_col_tiles, int rows_per_block,
    const float* __restrict__ halo_prev, const float* __restrict__ halo_next,
    const float* __restrict__ wprev, const float* __restrict__ wnext, Epi epi) {
  // 32-bit block decomposition (grids are < 2^24 blocks); column tile fastest,
  // so co-resident workgroups share rows and the halo re-reads hit L2
  const uint32_t b = blockIdx.x;
  const uint32_t nct = static_cast<uint32_t>(n_col_tiles);
  const uint32_t ct = b % nct;
  const int rg = static_cast<int>(b / nct);
  const int64_t c = int64_t(ct) * kThreads + threadIdx.x;  // column in units of V
  if (c >= ncols_v) return;
  const int r0 = rg * rows_per_block;
  const int r1 = min(r0 + rows_per_block, n_rows);

  auto row = [&](int r) -> const V* {
    const float* base = (r < 0) ? halo_prev : (r >= n_rows ? halo_next : X + int64_t(r) * ldx);
    return reinterpret_cast<const V*>(base + c_off) + c;
  };

  V q[PF + 2];
  q[0] = ldv<V, NT_LOAD>(row(r0 - 1));
  q[1] = ldv<V, NT_LOAD>(row(r0));
#pragma unroll
  for (int k = 0; k < PF; ++k) q[2 + k] = ldv<V, NT_LOAD>(row(min(r0 + 1 + k, r1)));

  for (int i = r0; i < r1; i += PF) {
    V nx[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) nx[k] = ldv<V, NT_LOAD>(row(min(i + PF + 1 + k, r1)));
#pragma unroll
    for (int k = 0; k < PF; ++k) {
      const int r = i + k;
      if (r < r1) {
        V out = axpy0(wprev[r], q[k], wnext[r], q[k + 2]);
        const int64_t cf = c_off + c * Vec<V>::W;
        out = epi.apply(out, epi.template load<V>(r, cf), r, cf);
        stv<V, NT_STORE>(reinterpret_cast<V*>(Y + int64_t(r) * ldy + c_off) + c, out);
      }
    }
    q[0] = q[PF];
    q[1] = q[PF + 1];
#pragma unroll
    for (int k = 0; k < PF; ++k) q[2 + k] = nx[k];
  }
}



// The two boundary rows of a sharded ring block in ONE launch (the multi-GPU
// round, dolhip.parallel.ShardedRing: the interior rows are mixed while the
// halo rows travel, then these two): blockIdx.y = 0 -> row 0 (previous row =
// halo_prev), 1 -> row n_rows - 1 (next row = halo_next); with n_rows == 1 only
// y = 0 runs and uses both halos.  Same arithmetic as ring_mix_kernel.
template <typename V, class Epi = NoEpi>
__global__ __launch_bounds__(kThreads) void ring_edges_kernel(
    const float* __restrict__ X, int64_t ldx, float* __restrict__ Y, int64_t ldy, int n_rows, int64_t c_off,
    int64_t ncols_v, const float* __restrict__ halo_prev, const float* __restrict__ halo_next,
    const float* __restrict__ wprev, const float* __restrict__ wnext, Epi epi) {
  const int64_t c = int64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (c >= ncols_v) return;
  const int r = blockIdx.y == 0 ? 0 : n_rows - 1;
  const float* pv = r == 0 ? halo_prev : X + int64_t(r - 1) * ldx;
  const float* nx = r == n_rows - 1 ? halo_next : X + int64_t(r + 1) * ldx;
  const V a = reinterpret_cast<const V*>(pv + c_off)[c];
  const V b = reinterpret_cast<const V*>(nx + c_off)[c];
  V out = axpy0(wprev[r], a, wnext[r], b);
  const int64_t cf = c_off + c * Vec<V>::W;
  out = epi.apply(out, epi.template load<V>(r, cf), r, cf);
  reinterpret_cast<V*>(Y + int64_t(r) * ldy + c_off)[c] = out;
}

// LDS-DMA form of the ring mix (the default float4 path).  Each wave moves
// its 1 KiB quarter of the tile's R + 2 rows straight into LDS with
// global_load_lds_dwordx4 (default cache policy: the halo rows' second reads
// must hit L2), waits on its own vmcnt, reads its lanes back and stores with
// nontemporal stores.  No barrier: a wave only reads what it loaded.  On
// MI355X (tools/membench7/8.hip, same box): 6.17 TB/s vs 5.91 for the
// register-staged kernel, = the measured copy ceiling (6.16); nt loads on
// every row cost 17 % (they evict the halo rows from L2), but nt on the R - 2
// rows no other tile reads (NTI, default; DOL_RING_NTI=0 turns it off) gains
// 2.3 %: 10.90-10.93 vs 11.15-11.16 ms at 8192 x 2^20, three A/B pairs on
// one box (profiles/r01d_ring_nti.txt).  The same split in ring_steps_kernel
// gained nothing.
#define DOL_GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define DOL_LPTR(p) ((__attribute__((address_space(3))) void*)(p))

// COPY (roofline calibration only): the same loads, cache policies and stores,
// with the stencil replaced by the tile's own row (Y = X): the memory-system
// ceiling of exactly this kernel's access pattern.
template <int R, class Epi = NoEpi, bool NTI = false, bool COPY = false>
__global__ __launch_bounds__(kThreads) void ring_mix_dma_kernel(
    const float* __restrict__ X, int64_t ldx, float* __restrict__ Y, int64_t ldy, int n_rows,
    int64_t ncols_v, int64_t n_col_tiles, const float* __restrict__ halo_prev,
    const float* __restrict__ halo_next, const float* __restrict__ wprev, const float* __restrict__ wnext,
    Epi epi) {
  __shared__ __attribute__((aligned(16))) float lds[kThreads / 64][R + 2][256];
  const uint32_t b = blockIdx.x;
  const uint32_t nct = static_cast<uint32_t>(n_col_tiles);
  const uint32_t ct = b % nct;
  const int r0 = static_cast<int>(b / nct) * R;
  const int r1 = min(r0 + R, n_rows);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t c = int64_t(ct) * kThreads + threadIdx.x;  // f4 column
  if (c >= ncols_v) return;
  auto row = [&](int r) -> const float* {
    return (r < 0) ? halo_prev : (r >= n_rows ? halo_next : X + int64_t(r) * ldx);
  };
#pragma unroll
  for (int k = 0; k < R + 2; ++k) {
    const int r = min(r0 - 1 + k, r1);
    if (NTI && k >= 2 && k < R)  // rows no other tile reads: nontemporal
      __builtin_amdgcn_global_load_lds(DOL_GPTR(row(r) + 4 * c), DOL_LPTR(&lds[wave][k][0]), 16, 0, 2);
    else
      __builtin_amdgcn_global_load_lds(DOL_GPTR(row(r) + 4 * c), DOL_LPTR(&lds[wave][k][0]), 16, 0, 0);
  }
  decltype(epi.template load<f4>(0, 0)) es[R];  // epilogue operands ride with the DMA
#pragma unroll
  for (int k = 0; k < R; ++k) es[k] = epi.template load<f4>(min(r0 + k, r1 - 1), 4 * c);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  f4 v[R + 2];
#pragma unroll
  for (int k = 0; k < R + 2; ++k) v[k] = *reinterpret_cast<const f4*>(&lds[wave][k][lane * 4]);
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int r = r0 + k;
    if (r < r1)
      __builtin_nontemporal_store(COPY ? v[k + 1] : epi.apply(axpy0(wprev[r], v[k], wnext[r], v[k + 2]), es[k], r, 4 * c),
                                  reinterpret_cast<f4*>(Y + int64_t(r) * ldy) + c);
  }
}

// ----------------------------------------------------------------------------
// Temporally blocked ring mix: STEPS synchronous rounds in one HBM pass
// (FedLCon's eps consensus steps, DIST/simulators.py:190-196).  A tile of R
// output rows loads R + 2*STEPS rows once and applies the 3-point stencil
// STEPS times in registers; level t is valid on [t, R + 2*STEPS - t).  Every
// intermediate uses the single-round formula (fl(fl(+0 + wp*a) + wn*b)), so the
// result is bit-identical to STEPS launches of ring_mix_kernel.  Wrap-around
// ring inside X (one shard).
// Tried (profiles/r02_ring_steps_eps_experiments.txt): intermediate levels as
// fma(wp, a, +0) + wn*b (three packed ops instead of four; exact up to -0 for
// +0 on the intermediate levels, the last level kept as axpy0 restores the bits)
// cut the pk ops per thread and tile 1,040 -> 824 but ran 12.63-12.74 vs
// 12.14-12.16 ms at eps = 5, three A/B pairs on one box: the pass is not
// VALU-issue bound.
// ----------------------------------------------------------------------------
template <int STEPS, int R, typename V = f4>
__global__ __launch_bounds__(kThreads) void ring_steps_kernel(
    const float* __restrict__ X, int64_t ldx, float* __restrict__ Y, int64_t ldy, int n_rows,
    int64_t ncols_v, uint32_t n_col_tiles, const float* __restrict__ wprev,
    const float* __restrict__ wnext, uint32_t n_row_tiles) {
  constexpr int L = R + 2 * STEPS;
  // XCD-aware order: the dispatcher deals blocks round-robin over the 8 XCDs,
  // so XCD x = b % 8 takes column tiles x, x + 8, ... and walks each one's row
  // tiles in order — a tile's 2*STEPS halo rows were just loaded by its
  // predecessor into the same L2.  (Column-tile-fastest order put vertical
  // neighbours a residency generation apart: 385 vs 431 rounds/s at eps = 5,
  // 8192 x 2^20.)
  const uint32_t b = blockIdx.x;
  const uint32_t x = b & 7u, l = b >> 3;
  const uint32_t ct = (l / n_row_tiles) * 8 + x;
  const int r0 = static_cast<int>(l % n_row_tiles) * R;
  if (ct >= n_col_tiles) return;
  const int64_t c = int64_t(ct) * kThreads + threadIdx.x;
  if (c >= ncols_v) return;
  auto wrap = [&](int r) { r %= n_rows; return r < 0 ? r + n_rows : r; };
  V v[L];
#pragma unroll
  for (int i = 0; i < L; ++i) v[i] = reinterpret_cast<const V*>(X + int64_t(wrap(r0 - STEPS + i)) * ldx)[c];
#pragma unroll
  for (int t = 1; t <= STEPS; ++t) {
    V prev_old = v[t - 1];
#pragma unroll
    for (int i = t; i < L - t; ++i) {
      const int g = wrap(r0 - STEPS + i);
      const V cur_old = v[i];
      v[i] = axpy0(wprev[g], prev_old, wnext[g], v[i + 1]);
      prev_old = cur_old;
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = r0 + i;
    if (r < n_rows) __builtin_nontemporal_store(v[STEPS + i], reinterpret_cast<V*>(Y + int64_t(r) * ldy) + c);
  }
}

// ----------------------------------------------------------------------------
// Streaming temporal blocking (r03): the same STEPS synchronous rounds and the
// same bits as ring_steps_kernel, with each thread walking ONE f4 column down
// a tile of T rows (+ STEPS halo rows on each side) instead of holding the
// whole tile in registers: when level-0 row i arrives, level t is produced at
// index i - t from level t-1's values at i - t + 1 (this step) and i - t - 1
// (two steps ago), so each level keeps its last two values (the step parity
// picks the register set: no copies) and the loads run PF rows ahead.  HBM
// sees one continuous read stream per column (halo re-reads 2 STEPS / T of
// the tile, from L2: vertically adjacent tiles run back to back on one XCD)
// instead of ring_steps_kernel's load-all / compute / store bursts with 2
// STEPS / R = 45 % halo at R = 22.  The stencil has no diagonal term (circle
// W: W_ii = 0), so only the two neighbours enter, as in axpy0.
// ----------------------------------------------------------------------------
template <int S, int PF, bool INTERIOR, bool NT>
__device__ __forceinline__ void ring_stream_body(const f4* __restrict__ xc, int64_t ldv, float* __restrict__ Y,
                                                 int64_t ldy, int64_t c, int n_rows, int r0, int nT,
                                                 const float* __restrict__ wprev, const float* __restrict__ wnext) {
  const int nsteps = nT + 2 * S;
  auto wrap = [&](int g) {  // |g| within one ring length of [0, n_rows)
    if constexpr (!INTERIOR) g = g < 0 ? g + n_rows : (g >= n_rows ? g - n_rows : g);
    return g;
  };
  // the prefetch walks the input rows with a running pointer (one 64-bit add per
  // step, a wrap test on edge tiles); past the tile's last input row it stays on
  // that row (always valid, never used)
  int gl = wrap(r0 - S);
  const f4* lp = xc + int64_t(gl) * ldv;
  int left = nsteps;  // input rows not yet issued
  auto next = [&]() {
    const f4 v = NT ? __builtin_nontemporal_load(lp) : *lp;
    if (--left > 0) {
      ++gl;
      lp += ldv;
      if constexpr (!INTERIOR) {
        if (gl == n_rows) {
          gl = 0;
          lp = xc;
        }
      }
    }
    return v;
  };
  f4 pf[PF];
#pragma unroll
  for (int u = 0; u < PF; ++u) pf[u] = next();
  f4 hA[S], hB[S];  // level t's value from two steps back, even / odd steps
#pragma unroll
  for (int t = 0; t < S; ++t) hA[t] = hB[t] = f4{0.f, 0.f, 0.f, 0.f};
  f4* yp = reinterpret_cast<f4*>(Y + int64_t(r0) * ldy) + c;  // the next output row
  const int64_t ldyv = ldy / 4;
  struct Wn { float v[PF + S]; };  // the weights of rows r0 - 2S + i0 .. (one scalar load per array and PF steps)
  for (int i0 = 0; i0 < nsteps; i0 += PF) {
    Wn wp, wn;
    if constexpr (INTERIOR) {
      wp = *reinterpret_cast<const Wn*>(wprev + (r0 - 2 * S + i0));
      wn = *reinterpret_cast<const Wn*>(wnext + (r0 - 2 * S + i0));
    } else {
#pragma unroll
      for (int j = 0; j < PF + S; ++j) {
        const int g = wrap(r0 - 2 * S + min(i0 + j, nsteps + S - 1));
        wp.v[j] = wprev[g];
        wn.v[j] = wnext[g];
      }
    }
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int i = i0 + u;
      f4 nv = pf[u];  // level 0 at index i
      pf[u] = next();
#pragma unroll
      for (int t = 1; t <= S; ++t) {
        f4& hv = (u & 1) ? hB[t - 1] : hA[t - 1];
        const f4 old = hv;  // level t-1 at index i - t - 1
        hv = nv;            // level t-1 at index i - t + 1, for two steps on
        // row of index i - t = r0 - 2S + i0 + (u + S - t)
        nv = axpy0(wp.v[u + S - t], old, wn.v[u + S - t], nv);
      }
      if (i >= 2 * S && i < nsteps) {  // level S at index i - S = row r0 + i - 2S
        __builtin_nontemporal_store(nv, yp);
        yp += ldyv;
      }
    }
  }
}

template <int S, int PF, bool NT>
__global__ __launch_bounds__(kThreads) void ring_stream_kernel(
    const float* __restrict__ X, int64_t ldx, float* __restrict__ Y, int64_t ldy, int n_rows,
    int64_t ncols_v, uint32_t n_col_tiles, const float* __restrict__ wprev,
    const float* __restrict__ wnext, uint32_t n_row_tiles, int T) {
  static_assert(PF % 2 == 0, "the step parity selects the history registers");
  const uint32_t b = blockIdx.x;
  const uint32_t x = b & 7u, l = b >> 3;
  const uint32_t ct = (l / n_row_tiles) * 8 + x;
  const int r0 = static_cast<int>(l % n_row_tiles) * T;
  if (ct >= n_col_tiles) return;
  const int64_t c = int64_t(ct) * kThreads + threadIdx.x;
  if (c >= ncols_v) return;
  const int nT = min(T, n_rows - r0);
  const f4* xc = reinterpret_cast<const f4*>(X) + c;
  const int64_t ldv = ldx / 4;
  if (r0 - 2 * S >= 0 && r0 + nT + S + PF <= n_rows)  // every row and weight index in range
    ring_stream_body<S, PF, true, NT>(xc, ldv, Y, ldy, c, n_rows, r0, nT, wprev, wnext);
  else
    ring_stream_body<S, PF, false, NT>(xc, ldv, Y, ldy, c, n_rows, r0, nT, wprev, wnext);
}

// ----------------------------------------------------------------------------
// The streaming pass on the headline's load path (r04): the level arithmetic
// of ring_stream_body (same bits), with the input rows arriving by LDS-DMA
// (global_load_lds_dwordx4) into a per-wave ring of D 1-KiB rows instead of
// VGPRs.  Each wave streams its own 1 KiB column strip down the tile and reads
// back only what it loaded (no barrier; the covering vmcnt orders the wave's
// own reads), so D - 1 rows per wave stay in flight with no VGPR held for
// them.  Every step issues exactly one DMA and one store (buffer stores: the
// 2S prologue steps and the tail store out of range, dropped but counted;
// past the last input row the DMA re-reads that row into a consumed slot), so
// one wait, vmcnt(2D - 2), always retires exactly the row about to be read:
// after L(i) come D - 1 loads and D - 1 stores (the prologue pairs each of its
// D - 1 loads with a dropped store to keep that count from the first step).
// Halo rows (the first and last 2S of a tile) load with the default policy,
// so the neighbouring tile on the same XCD finds them in L2; the rest are
// nontemporal, as in ring_mix_dma_kernel.
// ----------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

using rsrc_t = __amdgpu_buffer_rsrc_t;
constexpr uint32_t kOOB = 0x80000000u;  // a buffer offset past every range: the access is dropped

template <int S, int D, int PF, bool INTERIOR, int PROBE = 0, bool SYNC = false>
__device__ __forceinline__ void ring_stream_dma_body(const float* __restrict__ X, int64_t ldx, float* __restrict__ Y,
                                                     int64_t ldy, int64_t c, int n_rows, int r0, int nT,
                                                     const float* __restrict__ wprev,
                                                     const float* __restrict__ wnext, float* ring, bool live) {
  static_assert(D == PF || D == 2 * PF, "ring slots are compile-time within a chunk");
  static_assert(2 * D - 2 <= 63, "vmcnt is 6 bits");
  const int nsteps = nT + 2 * S;
  const int ntot = (nsteps + PF - 1) / PF * PF;  // steps run, the tail past nsteps included
  const int lane = threadIdx.x & 63;
  auto wrap = [&](int g) {
    if constexpr (!INTERIOR) g = g < 0 ? g + n_rows : (g >= n_rows ? g - n_rows : g);
    return g;
  };
  int gl = wrap(r0 - S);
  const float* xc = X + 4 * c;
  const float* lp = xc + int64_t(gl) * ldx;
  int issued = 0;
  auto issue = [&](int j) {  // input index j into slot j % D (j >= nsteps: the last row again)
    float* dst = ring + (j & (D - 1)) * 256;
    if (j < 2 * S || j >= nsteps - 2 * S)  // halo rows: default policy (re-read from L2 by the next tile)
      __builtin_amdgcn_global_load_lds(DOL_GPTR(lp), DOL_LPTR(dst), 16, 0, 0);
    else
      __builtin_amdgcn_global_load_lds(DOL_GPTR(lp), DOL_LPTR(dst), 16, 0, 2);
    if (++issued < nsteps) {
      ++gl;
      lp += ldx;
      if constexpr (!INTERIOR) {
        if (gl == n_rows) {
          gl = 0;
          lp = xc;
        }
      }
    }
  };
  const uint32_t voff = static_cast<uint32_t>(c) * 16u;
  auto store = [&](int i, f4 v) {  // output of step i: row r0 + i - 2S when 2S <= i < nsteps, else dropped
    const bool ok = live && i >= 2 * S && i < nsteps;
    const uint32_t oob = kOOB + (uint32_t(i + D) << 4);  // distinct dropped addresses: no two dummy stores merge
    const int r = ok ? r0 + i - 2 * S : r0;
    const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(Y + int64_t(r) * ldy, 0, static_cast<int>(ldy * 4), 0x00020000);
    // nontemporal (2) and volatile (bit 31): the dropped stores must all be
    // issued -- the vmcnt accounting counts them -- and identical prologue
    // stores would otherwise be merged by dead-store elimination
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), rs, ok ? voff : oob, 0, int(0x80000002u));
  };
#pragma unroll
  for (int j = 0; j < D - 1; ++j) {
    issue(j);
    store(j - D, f4{0.f, 0.f, 0.f, 0.f});
  }
  f4 hA[S], hB[S];
#pragma unroll
  for (int t = 0; t < S; ++t) hA[t] = hB[t] = f4{0.f, 0.f, 0.f, 0.f};
  struct Wn { float v[PF + S]; };
  for (int i0 = 0; i0 < ntot; i0 += PF) {
    // SYNC: the block's four waves meet once per chunk, so the four 1-KiB pieces
    // of each row are requested together (raw s_barrier: no vmcnt drain)
    if constexpr (SYNC) __builtin_amdgcn_s_barrier();
    Wn wp, wn;
    if constexpr (INTERIOR) {
      wp = *reinterpret_cast<const Wn*>(wprev + (r0 - 2 * S + i0));
      wn = *reinterpret_cast<const Wn*>(wnext + (r0 - 2 * S + i0));
    } else {
#pragma unroll
      for (int j = 0; j < PF + S; ++j) {
        const int g = wrap(r0 - 2 * S + min(i0 + j, nsteps + S - 1));
        wp.v[j] = wprev[g];
        wn.v[j] = wnext[g];
      }
    }
    const float* slot0 = ring + (D == PF ? 0 : (i0 & (D - 1))) * 256 + lane * 4;
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int i = i0 + u;
      // keep the DMA below the previous step's read and store: the slot it
      // overwrites was read by that step (WAR), and the store order is counted
      asm volatile("" ::: "memory");
      issue(i + D - 1);
      vm_wait<2 * D - 2>();  // L(i) has landed
      f4 nv = *reinterpret_cast<const f4*>(slot0 + u * 256);  // level 0 at index i
      if constexpr (PROBE == 0) {  // PROBE 1 (diagnostics): a copy in this geometry, no levels
#pragma unroll
        for (int t = 1; t <= S; ++t) {
          f4& hv = (u & 1) ? hB[t - 1] : hA[t - 1];
          const f4 old = hv;
          hv = nv;
          nv = axpy0(wp.v[u + S - t], old, wn.v[u + S - t], nv);
        }
      }
      store(i, nv);
    }
  }
  vm_wait<0>();  // no LDS-DMA may land after the wave's LDS is released
}

template <int S, int D, int PF, int PROBE = 0, bool SYNC = false>
__global__ __launch_bounds__(kThreads) void ring_stream_dma_kernel(
    const float* __restrict__ X, int64_t ldx, float* __restrict__ Y, int64_t ldy, int n_rows,
    int64_t ncols_v, uint32_t n_col_tiles, const float* __restrict__ wprev,
    const float* __restrict__ wnext, uint32_t n_row_tiles, int T, int order) {
  __shared__ __attribute__((aligned(16))) float lds[kThreads / 64][D][256];
  const uint32_t b = blockIdx.x;
  uint32_t ct;
  int r0;
  if (order == 0) {  // XCD-aware: an XCD walks its column tiles' row tiles in order (halo rows from L2)
    const uint32_t x = b & 7u, l = b >> 3;
    ct = (l / n_row_tiles) * 8 + x;
    r0 = static_cast<int>(l % n_row_tiles) * T;
  } else {  // column tile fastest: the chip sweeps row bands, as ring_mix_dma_kernel does
    const uint32_t nct8 = (n_col_tiles + 7) / 8 * 8;
    ct = b % nct8;
    r0 = static_cast<int>(b / nct8) * T;
  }
  if (ct >= n_col_tiles) return;  // the whole block
  int64_t c = int64_t(ct) * kThreads + threadIdx.x;
  const bool live = c < ncols_v;
  if (!SYNC && !live) return;
  if (!live) c = ncols_v - 1;  // SYNC: every wave reaches the barriers; a dead lane loads a valid column, stores nothing
  const int nT = min(T, n_rows - r0);
  float* ring = &lds[threadIdx.x >> 6][0][0];
  if (r0 - 2 * S >= 0 && r0 + nT + S + PF <= n_rows)  // every row and weight index in range
    ring_stream_dma_body<S, D, PF, true, PROBE, SYNC>(X, ldx, Y, ldy, c, n_rows, r0, nT, wprev, wnext, ring, live);
  else
    ring_stream_dma_body<S, D, PF, false, PROBE, SYNC>(X, ldx, Y, ldy, c, n_rows, r0, nT, wprev, wnext, ring, live);
}

// ----------------------------------------------------------------------------
// Generic CSR mix.  Blocks are ordered row-group fastest so that all rows of
// one column tile are in flight together: a neighbour row segment fetched
// from HBM by one workgroup is re-read from L2 / Infinity Cache by the others.
// ----------------------------------------------------------------------------
template <typename V, int RPB, class Epi = NoEpi>
__global__ __launch_bounds__(kThreads) void csr_mix_kernel(
    const float* __restrict__ X, int64_t ldx, float* __restrict__ Y, int64_t ldy, int n_rows,
    int64_t c_off, int64_t ncols_v, int64_t n_row_groups, const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ col, const float* __restrict__ val, Epi epi) {
  const int64_t b = blockIdx.x;
  const int rg = static_cast<int>(b % n_row_groups);
  const int64_t ct = b / n_row_groups;
  const int64_t c = ct * kThreads + threadIdx.x;
  if (c >= ncols_v) return;
  const int r0 = rg * RPB;
  const int r1 = min(r0 + RPB, n_rows);
  const V* xb = reinterpret_cast<const V*>(X + c_off) + c;
  const int64_t cf = c_off + c * Vec<V>::W;
  for (int r = r0; r < r1; ++r) {
    const auto es = epi.template load<V>(r, cf);
    const int e0 = rowptr[r];
    const int e1 = rowptr[r + 1];
    V acc = vzero(V{});
    int e = e0;
    for (; e + 4 <= e1; e += 4) {
      const V x0 = xb[int64_t(col[e + 0]) * (ldx / Vec<V>::W)];
      const V x1 = xb[int64_t(col[e + 1]) * (ldx / Vec<V>::W)];
      const V x2 = xb[int64_t(col[e + 2]) * (ldx / Vec<V>::W)];
      const V x3 = xb[int64_t(col[e + 3]) * (ldx / Vec<V>::W)];
      acc = fmac(acc, val[e + 0], x0);
      acc = fmac(acc, val[e + 1], x1);
      acc = fmac(acc, val[e + 2], x2);
      acc = fmac(acc, val[e + 3], x3);
    }
    for (; e < e1; ++e) acc = fmac(acc, val[e], xb[int64_t(col[e]) * (ldx / Vec<V>::W)]);
    acc = epi.apply(acc, es, r, cf);
    __builtin_nontemporal_store(acc, reinterpret_cast<V*>(Y + int64_t(r) * ldy + c_off) + c);
  }
}


// XCD-pinned CSR mix for large graphs with non-local neighbours (random-
// regular, ER as sparse): a column tile is W f4 wide (512 B of a row), and
// every block of that tile has the same blockIdx % 8 — the dispatcher deals
// blocks round-robin over the 8 XCDs, so the tile's whole X slab (n rows x
// 512 B, 4 MiB at 8192 agents) is fetched once into ONE XCD's L2 and the deg
// re-reads of each row hit there.  Placement is a speed assumption only: any
// other block->XCD mapping gives the same results.  Measured at 8192 x 2^20,
// d = 4 (tools/membench6.hip): 4.04 TB/s vs 3.0 with 4 KiB tiles whose 32 MiB
// slabs re-read through the Infinity Cache.  Degree-4 rows (random-regular)
// gather all passes' indices before any neighbour load (16.68 vs 16.80 ms).
// A persistent variant (a fixed grid per XCD walking the tiles in step, so
// only one slab is live in L2) ran 25-46 ms: latency-bound, dropped.  A
// persistent sweep (each workgroup holding 64 rows' partial sums in LDS, every
// row group's neighbour lists merged into one j-ascending list, so all readers
// of a line touch it together) was bit-exact but ran 27 ms with either tile
// order (profiles/r01d_csr_sweep_kernel.txt), dropped.  Tile
// widths (same box, 8192 x 2^20): 512 B 16.7 ms, 384 B (240-thread blocks)
// 22.6 ms, 256 B 18.2 ms.
template <int W, int PASSES, class Epi = NoEpi>
__global__ __launch_bounds__(kThreads) void csr_xcd_kernel(
    const float* __restrict__ X, int64_t ldx, float* __restrict__ Y, int64_t ldy, int n_rows,
    uint32_t nrb, uint32_t ntiles, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, Epi epi) {
  constexpr int ROWS = kThreads / W;
  constexpr int RB = ROWS * PASSES;
  const uint32_t b = blockIdx.x;
  const uint32_t xcd = b & 7u, local = b >> 3;
  const uint32_t tloc = local / nrb, rb = local % nrb;
  const uint32_t ct = tloc * 8 + xcd;
  if (ct >= ntiles) return;
  const int lane_c = threadIdx.x % W, lane_r = threadIdx.x / W;
  const int64_t c = int64_t(ct) * W + lane_c;  // f4 column
  const f4* xb = reinterpret_cast<const f4*>(X) + c;
  const int64_t ldv = ldx / 4;
  // every pass's row extent first, then (degree-4 rows, the random-regular
  // case) every pass's neighbour indices, then all neighbour loads: three
  // dependent round trips per workgroup instead of three per pass
  int rr[PASSES], e0[PASSES], e1[PASSES];
  bool four = true;
#pragma unroll
  for (int p = 0; p < PASSES; ++p) {
    rr[p] = int(rb) * RB + p * ROWS + lane_r;
    const int rc = rr[p] < n_rows ? rr[p] : n_rows - 1;
    e0[p] = rowptr[rc];
    e1[p] = rowptr[rc + 1];
    four = four && (e1[p] - e0[p] == 4);
  }
  if (four) {
    int cc[PASSES][4];
    float vv[PASSES][4];
#pragma unroll
    for (int p = 0; p < PASSES; ++p)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        cc[p][q] = col[e0[p] + q];
        vv[p][q] = val[e0[p] + q];
      }
    f4 xs[PASSES][4];
#pragma unroll
    for (int p = 0; p < PASSES; ++p)
#pragma unroll
      for (int q = 0; q < 4; ++q) xs[p][q] = xb[int64_t(cc[p][q]) * ldv];
#pragma unroll
    for (int p = 0; p < PASSES; ++p) {
      if (rr[p] < n_rows) {
        const auto es = epi.template load<f4>(rr[p], 4 * c);
        f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 4; ++q) acc = fmac(acc, vv[p][q], xs[p][q]);
        acc = epi.apply(acc, es, rr[p], 4 * c);
        __builtin_nontemporal_store(acc, reinterpret_cast<f4*>(Y + int64_t(rr[p]) * ldy) + c);
      }
    }
    return;
  }
#pragma unroll
  for (int p = 0; p < PASSES; ++p) {
    const int r = rr[p];
    if (r < n_rows) {
      const auto es = epi.template load<f4>(r, 4 * c);
      f4 acc = f4{0.f, 0.f, 0.f, 0.f};
      int e = e0[p];
      for (; e + 4 <= e1[p]; e += 4) {
        const f4 x0 = xb[int64_t(col[e]) * ldv], x1 = xb[int64_t(col[e + 1]) * ldv];
        const f4 x2 = xb[int64_t(col[e + 2]) * ldv], x3 = xb[int64_t(col[e + 3]) * ldv];
        acc = fmac(acc, val[e], x0);
        acc = fmac(acc, val[e + 1], x1);
        acc = fmac(acc, val[e + 2], x2);
        acc = fmac(acc, val[e + 3], x3);
      }
      for (; e < e1[p]; ++e) acc = fmac(acc, val[e], xb[int64_t(col[e]) * ldv]);
      acc = epi.apply(acc, es, r, 4 * c);
      __builtin_nontemporal_store(acc, reinterpret_cast<f4*>(Y + int64_t(r) * ldy) + c);
    }
  }
}

// ----------------------------------------------------------------------------
// Fused prox / ADMM gradient term + momentum SGD.
// MODE: 0 = no momentum, 1 = momentum first step (buf = g'), 2 = momentum.
// ----------------------------------------------------------------------------
template <bool THETA, bool ALPHA, int MODE, bool WRITE_G, bool DUAL = false>
__device__ __forceinline__ void prox_sgd_lane(float& w, float& bf, float& g, float th, float& al,
                                              float rho, float neg_lr, float mom) {
  float gg = g;
  if constexpr (THETA) {
    float t = rho * (w - th);
    if constexpr (ALPHA) t = al + t;
    gg = gg + t;
  }
  if constexpr (WRITE_G) g = gg;
  float d = gg;
  if constexpr (MODE == 1) { bf = gg; d = gg; }
  if constexpr (MODE == 2) { bf = bf * mom + gg; d = bf; }
  w = __builtin_fmaf(neg_lr, d, w);
  if constexpr (DUAL) al = al + rho * (w - th);  // update_duals on the new w (DEC/clients.py:141-144)
}

template <typename V, bool THETA, bool ALPHA, int MODE, bool WRITE_G, bool DUAL = false>
__global__ __launch_bounds__(kThreads) void prox_sgd_kernel(
    float* __restrict__ W, int64_t ldw, float* __restrict__ B, int64_t ldb, float* __restrict__ G,
    int64_t ldg, const float* __restrict__ theta, float* __restrict__ A, int64_t lda,
    float rho, float neg_lr, float mom, int64_t c_off, int64_t ncols_v, int64_t n_col_tiles) {
  const int64_t blk = blockIdx.x;
  const int64_t agent = blk / n_col_tiles;
  const int64_t c = (blk % n_col_tiles) * kThreads + threadIdx.x;
  if (c >= ncols_v) return;
  V* wp = reinterpret_cast<V*>(W + agent * ldw + c_off) + c;
  V* gp = reinterpret_cast<V*>(G + agent * ldg + c_off) + c;
  // every per-agent row is read and written once: nontemporal both ways (r05:
  // 100 x 1,663,370 0.83 vs 0.90 ms, 1024 x 2^20 4.67 vs 4.96 ms,
  // profiles/r05zzr_prox_sgd_nt_ab.jsonl); theta is shared by all agents: cached
  constexpr bool DOL_PROX_NT = true;
  V w = ldv<V, DOL_PROX_NT>(wp), g = ldv<V, DOL_PROX_NT>(gp);
  V bf{}, th{}, al{};
  if constexpr (MODE == 2) bf = ldv<V, DOL_PROX_NT>(reinterpret_cast<V*>(B + agent * ldb + c_off) + c);
  if constexpr (THETA) th = *(reinterpret_cast<const V*>(theta + c_off) + c);
  if constexpr (ALPHA) al = ldv<V, DOL_PROX_NT>(reinterpret_cast<const V*>(A + agent * lda + c_off) + c);
  if constexpr (Vec<V>::W == 1) {
    prox_sgd_lane<THETA, ALPHA, MODE, WRITE_G, DUAL>(w, bf, g, th, al, rho, neg_lr, mom);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float wj = w[j], bj = bf[j], gj = g[j], aj = al[j];
      prox_sgd_lane<THETA, ALPHA, MODE, WRITE_G, DUAL>(wj, bj, gj, th[j], aj, rho, neg_lr, mom);
      w[j] = wj;
      bf[j] = bj;
      g[j] = gj;
      al[j] = aj;
    }
  }
  stv<V, DOL_PROX_NT>(wp, w);
  if constexpr (WRITE_G) stv<V, DOL_PROX_NT>(gp, g);
  if constexpr (MODE != 0) stv<V, DOL_PROX_NT>(reinterpret_cast<V*>(B + agent * ldb + c_off) + c, bf);
  if constexpr (DUAL) stv<V, DOL_PROX_NT>(reinterpret_cast<V*>(A + agent * lda + c_off) + c, al);
}

// Gradient term alone: g += rho*(w - theta) (+ alpha), w untouched.
template <typename V, bool ALPHA>
__global__ __launch_bounds__(kThreads) void prox_grad_kernel(
    float* __restrict__ G, int64_t ldg, const float* __restrict__ W, int64_t ldw,
    const float* __restrict__ theta, const float* __restrict__ A, int64_t lda, float rho,
    int64_t c_off, int64_t ncols_v, int64_t n_col_tiles) {
  const int64_t blk = blockIdx.x;
  const int64_t agent = blk / n_col_tiles;
  const int64_t c = (blk % n_col_tiles) * kThreads + threadIdx.x;
  if (c >= ncols_v) return;
  V* gp = reinterpret_cast<V*>(G + agent * ldg + c_off) + c;
  const V w = *(reinterpret_cast<const V*>(W + agent * ldw + c_off) + c);
  const V th = *(reinterpret_cast<const V*>(theta + c_off) + c);
  V t = rho * (w - th);
  if constexpr (ALPHA) t = *(reinterpret_cast<const V*>(A + agent * lda + c_off) + c) + t;
  *gp = *gp + t;
}

// ----------------------------------------------------------------------------
// ADMM dual update alpha += rho*(w - theta), with optional per-agent
// ||w-theta||^2 partials (fp64, fixed reduction tree -> deterministic).
// One block = kThreads lanes x kDualIters V-columns of one agent.
// ----------------------------------------------------------------------------
constexpr int kDualIters = 4;

__device__ __forceinline__ double block_sum_f64(double v, double* smem) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    for (int i = 0; i < kThreads / 64; ++i) s += smem[i];
  }
  return s;
}

__device__ __forceinline__ float dual_lane(float& a, float w, float th, float rho, double& r) {
  const float d = w - th;
  a = a + rho * d;
  r += double(d) * double(d);
  return d;
}

// VEC: columns [0, n4) as f4, then the (< 4) tail columns by the first
// lanes of the agent's last chunk; !VEC: all P columns scalar.
template <bool VEC, bool RESID>
__global__ __launch_bounds__(kThreads) void admm_dual_kernel(
    float* __restrict__ A, int64_t lda, const float* __restrict__ W, int64_t ldw,
    const float* __restrict__ theta, float rho, int64_t P, int64_t n_chunks,
    double* __restrict__ partial) {
  __shared__ double smem[kThreads / 64];
  const int64_t blk = blockIdx.x;
  const int64_t agent = blk / n_chunks;
  const int64_t chunk = blk % n_chunks;
  float* arow = A + agent * lda;
  const float* wrow = W + agent * ldw;
  double r = 0.0;
  if constexpr (VEC) {
    const int64_t n4 = P / 4;
#pragma unroll
    for (int it = 0; it < kDualIters; ++it) {
      const int64_t c = (chunk * kDualIters + it) * kThreads + threadIdx.x;
      if (c < n4) {
        // rows read / written once: nontemporal (r05: 100 x 1,663,370 0.378 vs
        // 0.395 ms, 1024 x 2^20 2.16 vs 2.37 ms, profiles/r05zzs_admm_dual_nt_ab.jsonl)
        constexpr bool DOL_DUAL_NT = true;
        f4* ap = reinterpret_cast<f4*>(arow) + c;
        const f4 w = ldv<f4, DOL_DUAL_NT>(reinterpret_cast<const f4*>(wrow) + c);
        const f4 th = reinterpret_cast<const f4*>(theta)[c];
        f4 a = ldv<f4, DOL_DUAL_NT>(ap);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float aj = a[j];
          dual_lane(aj, w[j], th[j], rho, r);
          a[j] = aj;
        }
        stv<f4, DOL_DUAL_NT>(ap, a);
      }
    }
    const int64_t tail = P - 4 * n4;
    if (chunk == n_chunks - 1 && threadIdx.x < tail) {
      const int64_t c = 4 * n4 + threadIdx.x;
      float a = arow[c];
      dual_lane(a, wrow[c], theta[c], rho, r);
      arow[c] = a;
    }
  } else {
#pragma unroll
    for (int it = 0; it < kDualIters; ++it) {
      const int64_t c = (chunk * kDualIters + it) * kThreads + threadIdx.x;
      if (c < P) {
        float a = arow[c];
        dual_lane(a, wrow[c], theta[c], rho, r);
        arow[c] = a;
      }
    }
  }
  if constexpr (RESID) {
    const double s = block_sum_f64(r, smem);
    if (threadIdx.x == 0) partial[agent * n_chunks + chunk] = s;
  }
}

// partial layout: [n_agents][n_chunks_total]; one block per agent, fixed order.
__global__ __launch_bounds__(kThreads) void resid_reduce_kernel(const double* __restrict__ partial,
                                                                int64_t n_chunks,
                                                                double* __restrict__ out) {
  __shared__ double smem[kThreads / 64];
  const int64_t agent = blockIdx.x;
  double v = 0.0;
  for (int64_t i = threadIdx.x; i < n_chunks; i += kThreads) v += partial[agent * n_chunks + i];
  const double s = block_sum_f64(v, smem);
  if (threadIdx.x == 0) out[agent] = s;
}

// ----------------------------------------------------------------------------
// One FedADMM client round on the separable least-squares objective
// f_k(w) = 1/2 ||w - t_k||^2 (BASELINE config 4's primal/dual side), fused
// per sampled agent k (row a = agents[k]) — the reference's
// FedAdmm_Client.update_weights (DEC/clients.py:36-53) with the CNN gradient
// replaced by the exact least-squares one:
//   w = theta                                   (load_state_dict(theta), :37)
//   local_steps times:  g = fl(w - t)
//     g' = fl(g + fl(alpha + fl(rho * fl(w - theta))))        (:132-135)
//     SGD(lr, momentum).step(): buf = first ? g' : fl(fl(buf*mu) + g'); w = fma(-lr, buf, w)
//   alpha = fl(alpha + fl(rho * fl(w - theta)))  (update_duals, :141-144, pre-round theta)
// Streams t, alpha (, buf) in and w, alpha (, buf) out once; w is never read.
// RESID: fp64 per-block partials of ||w - theta||^2 and ||alpha||^2 (fixed
// reduction tree, deterministic), as admm_dual_kernel.
// ----------------------------------------------------------------------------
template <bool MOM>
__device__ __forceinline__ void admm_ls_lane(float& w, float& b, float& a, float t, float th, float rho,
                                             float neg_lr, float mom, int steps, bool first, double& rw,
                                             double& ra) {
  w = th;
  for (int k = 0; k < steps; ++k) {
    const float g = w - t;
    const float gg = g + (a + rho * (w - th));
    float d = gg;
    if constexpr (MOM) {
      b = (first && k == 0) ? gg : b * mom + gg;
      d = b;
    }
    w = __builtin_fmaf(neg_lr, d, w);
  }
  const float dl = w - th;
  a = a + rho * dl;
  // the product of two floats is exact in double, so fma == the reference's
  // separately rounded rw + d*d, one instruction fewer
  rw = __builtin_fma(double(dl), double(dl), rw);
  ra = __builtin_fma(double(a), double(a), ra);
}

// The same lane on two columns at once: packed fp32 (v_pk_add / v_pk_mul /
// v_pk_fma_f32 on gfx950, each an IEEE operation per half), same rounding per
// element as admm_ls_lane.  At 10 local steps the round runs ~70 fp32 ops per
// element: unpacked that is ~60 % of the HBM time in VALU issue.
typedef float f2 __attribute__((ext_vector_type(2)));
template <bool MOM>
__device__ __forceinline__ void admm_ls_lane2(f2& w, f2& b, f2& a, f2 t, f2 th, float rho, float neg_lr, float mom,
                                              int steps, bool first, double& rw, double& ra) {
  const f2 rho2 = {rho, rho}, nlr2 = {neg_lr, neg_lr}, mom2 = {mom, mom};
  w = th;
  for (int k = 0; k < steps; ++k) {
    const f2 g = w - t;
    const f2 gg = g + (a + rho2 * (w - th));
    f2 d = gg;
    if constexpr (MOM) {
      b = (first && k == 0) ? gg : b * mom2 + gg;
      d = b;
    }
    w = __builtin_elementwise_fma(nlr2, d, w);
  }
  const f2 dl = w - th;
  a = a + rho2 * dl;
  rw = __builtin_fma(double(dl.x), double(dl.x), rw);
  rw = __builtin_fma(double(dl.y), double(dl.y), rw);
  ra = __builtin_fma(double(a.x), double(a.x), ra);
  ra = __builtin_fma(double(a.y), double(a.y), ra);
}
// f4 = two packed halves
template <bool MOM>
__device__ __forceinline__ void admm_ls_lane4(f4& w, f4& b, f4& a, f4 t, f4 th, float rho, float neg_lr, float mom,
                                              int steps, bool first, double& rw, double& ra) {
  f2 w0, w1, b0 = b.xy, b1 = b.zw, a0 = a.xy, a1 = a.zw;
  admm_ls_lane2<MOM>(w0, b0, a0, t.xy, th.xy, rho, neg_lr, mom, steps, first, rw, ra);
  admm_ls_lane2<MOM>(w1, b1, a1, t.zw, th.zw, rho, neg_lr, mom, steps, first, rw, ra);
  w = f4{w0.x, w0.y, w1.x, w1.y};
  b = f4{b0.x, b0.y, b1.x, b1.y};
  a = f4{a0.x, a0.y, a1.x, a1.y};
}

template <bool VEC, bool MOM, bool RESID>
__global__ __launch_bounds__(kThreads) void admm_ls_round_kernel(
    float* __restrict__ W, int64_t ldw, float* __restrict__ B, int64_t ldb, float* __restrict__ A, int64_t lda,
    const float* __restrict__ T, int64_t ldt, const float* __restrict__ theta, const int32_t* __restrict__ agents,
    const int32_t* __restrict__ first, int64_t P, float rho, float neg_lr, float mom, int steps, int64_t n_chunks,
    double* __restrict__ partial) {
  __shared__ double smem[kThreads / 64];
  // agent-major blocks (consecutive blocks stream one row; a column-major order
  // put 2048 rows 4 MiB apart in flight at once and ran 1-2 % slower).  The
  // rows stream with nontemporal loads / stores so theta (4 MiB at 2^20, one
  // XCD's L2) stays resident for the next row instead of being evicted by them
  const int64_t blk = blockIdx.x;
  const int64_t k = blk / n_chunks;
  const int64_t chunk = blk % n_chunks;
  const int64_t a_row = agents ? agents[k] : k;
  const bool fst = first ? first[k] != 0 : false;
  float* wr = W + a_row * ldw;
  float* br = B + a_row * ldb;
  float* ar = A + a_row * lda;
  const float* tr = T + a_row * ldt;
  double rw = 0.0, ra = 0.0;
  auto one = [&](int64_t c) {
    float w, b = MOM ? br[c] : 0.0f, a = ar[c];
    admm_ls_lane<MOM>(w, b, a, tr[c], theta[c], rho, neg_lr, mom, steps, fst, rw, ra);
    wr[c] = w;
    ar[c] = a;
    if constexpr (MOM) br[c] = b;
  };
  if constexpr (VEC) {
    const int64_t n4 = P / 4;
#pragma unroll
    for (int it = 0; it < kDualIters; ++it) {
      const int64_t c = (chunk * kDualIters + it) * kThreads + threadIdx.x;
      if (c < n4) {
        const f4 t = __builtin_nontemporal_load(reinterpret_cast<const f4*>(tr) + c);
        const f4 th = reinterpret_cast<const f4*>(theta)[c];
        f4 a = __builtin_nontemporal_load(reinterpret_cast<const f4*>(ar) + c);
        f4 b = MOM ? __builtin_nontemporal_load(reinterpret_cast<const f4*>(br) + c) : f4{0.f, 0.f, 0.f, 0.f};
        f4 w;
        admm_ls_lane4<MOM>(w, b, a, t, th, rho, neg_lr, mom, steps, fst, rw, ra);
        __builtin_nontemporal_store(w, reinterpret_cast<f4*>(wr) + c);
        __builtin_nontemporal_store(a, reinterpret_cast<f4*>(ar) + c);
        if constexpr (MOM) __builtin_nontemporal_store(b, reinterpret_cast<f4*>(br) + c);
      }
    }
    const int64_t tail = P - 4 * n4;
    if (chunk == n_chunks - 1 && threadIdx.x < tail) one(4 * n4 + threadIdx.x);
  } else {
#pragma unroll
    for (int it = 0; it < kDualIters; ++it) {
      const int64_t c = (chunk * kDualIters + it) * kThreads + threadIdx.x;
      if (c < P) one(c);
    }
  }
  if constexpr (RESID) {
    const double sw = block_sum_f64(rw, smem);
    __syncthreads();
    const double sa = block_sum_f64(ra, smem);
    if (threadIdx.x == 0) {
      partial[k * n_chunks + chunk] = sw;
      partial[(gridDim.x / n_chunks + k) * n_chunks + chunk] = sa;
    }
  }
}

// ----------------------------------------------------------------------------
// Ordered sum / mean over gathered rows: acc = w[o0]; acc += w[o1]; ...
// Column-parallel; the row loop is unrolled so 8 row loads are in flight.
// ----------------------------------------------------------------------------
template <typename V>
__global__ __launch_bounds__(kThreads) void ordered_sum_kernel(
    const float* __restrict__ W, int64_t ldw, const int32_t* __restrict__ order, int m,
    int64_t c_off, int64_t ncols_v, const float* __restrict__ acc_in, float* __restrict__ out,
    float scale, int do_div) {
  const int64_t c = int64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (c >= ncols_v) return;
  const V* wb = reinterpret_cast<const V*>(W + c_off) + c;
  const int64_t ldv = ldw / Vec<V>::W;
  V acc;
  int k;
  if (acc_in) {
    acc = *(reinterpret_cast<const V*>(acc_in + c_off) + c);
    k = 0;
  } else {
    acc = wb[int64_t(order[0]) * ldv];
    k = 1;
  }
  // the rows are read once: nontemporal loads (8192 x 2^20: 5.07-5.14 ms =
  // 6.77 TB/s vs 5.66-5.74 ms plain; 16 rows in flight instead of 8: no change;
  // profiles/r05zze_ordered_sum_ab.jsonl)
  for (; k + 8 <= m; k += 8) {
    V x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = __builtin_nontemporal_load(wb + int64_t(order[k + u]) * ldv);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = vadd(acc, x[u]);
  }
  for (; k < m; ++k) acc = vadd(acc, __builtin_nontemporal_load(wb + int64_t(order[k]) * ldv));
  if (do_div) acc = vdiv(acc, scale);
  *(reinterpret_cast<V*>(out + c_off) + c) = acc;
}

// ----------------------------------------------------------------------------
// The FedADMM client round fused with the server's ordered mean (one round of
// DEC/servers.py:50-81 on least squares: every sampled client's
// update_weights, DEC/clients.py:36-53, then average_weights, :42-48).
// Column-strip major: each lane owns one V-column and walks the m sampled
// agents in the given order, running admm_ls_lane on (agent, column) and
// chaining acc = w(first) ; acc = fl(acc + w) — the ordered_sum_kernel's
// association, so theta_next is the same bits as admm_ls_round_kernel +
// ordered_sum_kernel — while the w rows are still in registers: the separate
// mean read every sampled row back from HBM (34 GB at 8192 x 2^20, 15 % of the
// round's bytes).  theta is read once per lane, not once per (agent, column).
// The next agent group's t / alpha / buf loads are issued before the current
// group's steps (kRoundPF agents in flight per lane).
// RESID: fp64 per-lane sums over the agents of (w - theta)^2 and alpha^2, a
// fixed block tree, one partial per block; resid_reduce_kernel folds the
// blocks in a fixed order (the round's totals, not per agent).
// ----------------------------------------------------------------------------
constexpr int kRoundPF = 3;

template <bool MOM>
__device__ __forceinline__ void admm_ls_lane_v(float& w, float& b, float& a, float t, float th, float rho, float neg_lr,
                                               float mom, int steps, bool first, double& rw, double& ra) {
  admm_ls_lane<MOM>(w, b, a, t, th, rho, neg_lr, mom, steps, first, rw, ra);
}
// packed (measured at 8192 x 2^20, 10 steps: 34.6-35.1 ms vs 36.0-36.5 with
// the per-element scalar form, profiles/r05zw_admm_round_ab.jsonl)
template <bool MOM>
__device__ __forceinline__ void admm_ls_lane_v(f4& w, f4& b, f4& a, f4 t, f4 th, float rho, float neg_lr, float mom,
                                               int steps, bool first, double& rw, double& ra) {
  admm_ls_lane4<MOM>(w, b, a, t, th, rho, neg_lr, mom, steps, first, rw, ra);
}
__device__ __forceinline__ float ldnt(const float* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ f4 ldnt(const f4* p) { return __builtin_nontemporal_load(p); }
// nontemporal buffer store of lane value v at byte offset voff of the row at
// base (row-uniform resource); voff = kOOB drops it (still issued and counted)
__device__ __forceinline__ void st_row(float v, float* base, int64_t nbytes, uint32_t voff) {
  const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, static_cast<int>(nbytes), 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, voff, 0, 2);
}
__device__ __forceinline__ void st_row(f4 v, float* base, int64_t nbytes, uint32_t voff) {
  const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, static_cast<int>(nbytes), 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), rs, voff, 0, 2);
}

template <int NT>
__device__ __forceinline__ double block_sum_f64_nt(double v, double* smem) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    for (int i = 0; i < NT / 64; ++i) s += smem[i];
  }
  return s;
}

template <typename V, bool MOM, bool RESID, int NT, int PF = kRoundPF>
__global__ __launch_bounds__(NT) void admm_ls_round_mean_kernel(
    float* __restrict__ W, int64_t ldw, float* __restrict__ B, int64_t ldb, float* __restrict__ A, int64_t lda,
    const float* __restrict__ T, int64_t ldt, const float* __restrict__ theta, const int32_t* __restrict__ agents,
    const int32_t* __restrict__ first, int m, int64_t c_off, int64_t ncols_v, float rho, float neg_lr, float mom,
    int steps, float* __restrict__ out, float scale, int do_div, double* __restrict__ partial, int64_t part_off,
    int64_t part_stride) {
  __shared__ double smem[NT / 64];
  const int64_t c = int64_t(blockIdx.x) * NT + threadIdx.x;
  const bool live = c < ncols_v;
  if (!RESID && !live) return;
  // dead lanes (RESID only) read the last real column and compute on it; their
  // stores are buffer stores pointed out of range (dropped, still counted, so
  // every lane issues the same memory ops and the loop's vmcnt waits stay
  // exact) and their residual terms are dropped
  const int64_t cc = live ? c : ncols_v - 1;
  const uint32_t voff = live ? uint32_t(c) * uint32_t(sizeof(V)) : kOOB;
  auto st = [&](V v, float* base, int64_t ld, int64_t row) {
    st_row(v, base + row * ld + c_off, std::min<int64_t>((ld - c_off) * 4, 0x7ffffff0), voff);
  };
  auto cptr = [&](const float* base, int64_t ld, int64_t row) {
    return reinterpret_cast<const V*>(base + row * ld + c_off) + cc;
  };
  auto row_of = [&](int k) -> int64_t {  // agent k's row; k past m: the last agent's (a harmless re-read)
    k = min(k, m - 1);
    return agents ? agents[k] : k;
  };
  const V th = *cptr(theta, 0, 0);
  V acc = vzero(th);
  double rw = 0.0, ra = 0.0;
  struct Grp {
    V t[PF], a[PF], b[PF];
    int64_t row[PF];
  };
  auto load = [&](Grp& g, int k0) {  // agents k0 .. k0 + PF - 1, unconditionally (rows clamped)
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      g.row[u] = row_of(k0 + u);
      g.t[u] = ldnt(cptr(T, ldt, g.row[u]));
      g.a[u] = ldnt(cptr(A, lda, g.row[u]));
      if constexpr (MOM) g.b[u] = ldnt(cptr(B, ldb, g.row[u]));
    }
  };
  auto run = [&](Grp& g, int u, int k) {  // agent k = group slot u: its steps, stores, and the chain
    const bool fst = first ? first[k] != 0 : false;
    V w, bu = MOM ? g.b[u] : vzero(th), au = g.a[u];
    double rwu = 0.0, rau = 0.0;
    admm_ls_lane_v<MOM>(w, bu, au, g.t[u], th, rho, neg_lr, mom, steps, fst, rwu, rau);
    st(w, W, ldw, g.row[u]);
    st(au, A, lda, g.row[u]);
    if constexpr (MOM) st(bu, B, ldb, g.row[u]);
    rw += live ? rwu : 0.0;
    ra += live ? rau : 0.0;
    acc = k == 0 ? w : vadd(acc, w);
  };
  const int ng = (m + PF - 1) / PF;  // groups; all but the last are full
  Grp nxt, cur;
  load(nxt, 0);
  for (int gi = 0; gi + 1 < ng; ++gi) {  // straight-line body: the same memory ops every trip
    cur = nxt;
    load(nxt, (gi + 1) * PF);      // the next group's loads fly during this group's steps
#pragma unroll
    for (int u = 0; u < PF; ++u) run(cur, u, gi * PF + u);
  }
#pragma unroll
  for (int u = 0; u < PF; ++u) {   // the last group (maybe partial)
    const int k = (ng - 1) * PF + u;
    if (k < m) run(nxt, u, k);
  }
  if (live) {
    if (do_div) acc = vdiv(acc, scale);
    *(reinterpret_cast<V*>(out + c_off) + c) = acc;
  }
  if constexpr (RESID) {
    const double sw = block_sum_f64_nt<NT>(rw, smem);
    __syncthreads();
    const double sa = block_sum_f64_nt<NT>(ra, smem);
    if (threadIdx.x == 0) {
      partial[part_off + blockIdx.x] = sw;
      partial[part_stride + part_off + blockIdx.x] = sa;
    }
  }
}

// Calibration copy: each block streams one contiguous 16 KiB chunk (4 x f4
// per lane, nontemporal both ways) and exits — 6.26 TB/s on MI355X, the
// measured ceiling the mixing kernels are compared with (tools/membench.hip).
__global__ __launch_bounds__(kThreads) void copy_kernel(const f4* __restrict__ src, f4* __restrict__ dst,
                                                        int64_t n) {
  const int64_t base = int64_t(blockIdx.x) * kThreads * 4 + threadIdx.x;
  f4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (base + u * kThreads < n) v[u] = __builtin_nontemporal_load(src + base + u * kThreads);
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (base + u * kThreads < n) __builtin_nontemporal_store(v[u], dst + base + u * kThreads);
}

__global__ __launch_bounds__(kThreads) void copy_scalar_kernel(const float* __restrict__ src,
                                                               float* __restrict__ dst, int64_t n) {
  const int64_t stride = int64_t(gridDim.x) * kThreads;
  for (int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}


// ----------------------------------------------------------------------------
// Dense mix Y = W X on fp32 MFMA (v_mfma_f32_32x32x2_f32), for dense W
// (complete / Erdos-Renyi / time-varying graphs).  Block tile 128 x 128,
// BK = 32; 4 waves in 2 x 2, each owning a 64 x 64 output sub-tile as 2 x 2
// MFMA accumulators (64 AGPR/VGPR).  The next K-tile is loaded into registers
// while the current one feeds the MFMAs (one LDS buffer, two barriers per K
// tile).  A is stored k-major in LDS so both fragments are 32 consecutive
// floats per half-wave (conflict-free ds_read_b32).  Numerics: each output is
// an fma chain over k ascending (exact f32 MFMA), NOT the reference's
// mul-then-add with W_ij <= 0 skipped — a tolerance path, opt-in.
// ----------------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kDBM = 128, kDBN = 128, kDBK = 32, kDPad = 4;

template <bool VEC_A, bool VEC_B>
__global__ __launch_bounds__(256, 1) void dense_mix_mfma_kernel(
    const float* __restrict__ W, int64_t ldw, const float* __restrict__ X, int64_t ldx,
    float* __restrict__ Y, int64_t ldy, int M, int K, int64_t P, uint32_t n_row_tiles) {
  __shared__ float As[kDBK][kDBM + kDPad];
  __shared__ float Bs[kDBK][kDBN + kDPad];
  const uint32_t b = blockIdx.x;
  const int m0 = int(b % n_row_tiles) * kDBM;       // row tiles fastest: an X panel is
  const int64_t n0 = int64_t(b / n_row_tiles) * kDBN;  // reused by consecutive blocks
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // staging maps: A 128 rows x 32 k (4 f4 per thread), B 32 k x 128 cols (4 f4 per thread)
  const int ar = t >> 1, ak = (t & 1) * 16;
  const int bk = t >> 3, bc = (t & 7) * 16;
  f4 ra[4], rb[4];
  auto load_tiles = [&](int k0) {
    const int row = m0 + ar;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + ak + 4 * j;
      if constexpr (VEC_A) {
        ra[j] = (row < M && k < K) ? *reinterpret_cast<const f4*>(W + int64_t(row) * ldw + k) : f4{0.f, 0.f, 0.f, 0.f};
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) ra[j][q] = (row < M && k + q < K) ? W[int64_t(row) * ldw + k + q] : 0.f;
      }
    }
    const int kr = k0 + bk;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t c = n0 + bc + 4 * j;
      if (kr < K && c + 3 < P && VEC_B) {
        rb[j] = *reinterpret_cast<const f4*>(X + int64_t(kr) * ldx + c);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) rb[j][q] = (kr < K && c + q < P) ? X[int64_t(kr) * ldx + c + q] : 0.f;
      }
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  load_tiles(0);
  for (int k0 = 0; k0 < K; k0 += kDBK) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) As[ak + 4 * j + q][ar] = ra[j][q];
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<f4*>(&Bs[bk][bc + 4 * j]) = rb[j];
    __syncthreads();
    if (k0 + kDBK < K) load_tiles(k0 + kDBK);
    const int kh = lane >> 5, li = lane & 31;
#pragma unroll
    for (int kk = 0; kk < kDBK / 2; ++kk) {
      const int k = 2 * kk + kh;
      const float a0 = As[k][wm * 64 + li], a1 = As[k][wm * 64 + 32 + li];
      const float b0 = Bs[k][wn * 64 + li], b1 = Bs[k][wn * 64 + 32 + li];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
  // C/D map (gfx950, dtype-independent): col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wn * 64 + j * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < M && col < P) Y[int64_t(row) * ldy + col] = acc[i][j][r];
      }
    }
}

// ----------------------------------------------------------------------------
// host-side launch helpers
// ----------------------------------------------------------------------------
inline int64_t cdiv(int64_t a, int64_t b) { return a / b + (a % b != 0); }
// a * b saturated at INT64_MAX: block-count checks of absurd sizes must fail, not overflow
inline int64_t mul_sat(int64_t a, int64_t b) {
  int64_t r;
  return __builtin_mul_overflow(a, b, &r) ? INT64_MAX : r;
}

// Split [0, P) into a f4 part and a scalar tail; returns whether the
// f4 path is legal for all given (base, ld) pairs.
struct ColSplit {
  bool vec;
  int64_t n4;    // f4 columns
  int64_t tail;  // scalar columns after 4*n4 (or all P when !vec)
};

inline ColSplit split_cols(int64_t P, bool vec_ok) {
  if (!vec_ok) return {false, 0, P};
  return {true, P / 4, P % 4};
}

inline bool row_vec_ok(const void* base, int64_t ld) { return base == nullptr || (aligned16(base) && (ld % 4) == 0); }

template <typename V, int PF, bool NTL, bool NTS, class Epi = NoEpi>
void launch_ring(const float* X, int64_t ldx, float* Y, int64_t ldy, int n_rows, int64_t c_off,
                 int64_t ncols_v, int rpb, const float* hp, const float* hn, const float* wp,
                 const float* wn, hipStream_t s, const Epi& epi = Epi{}) {
  const int64_t n_col_tiles = cdiv(ncols_v, kThreads);
  const int64_t n_rg = cdiv(n_rows, rpb);
  const int64_t grid = n_col_tiles * n_rg;
  hipLaunchKernelGGL((ring_mix_kernel<V, PF, NTL, NTS, Epi>), dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, s,
                     X, ldx, Y, ldy, n_rows, c_off, ncols_v, n_col_tiles, rpb, hp, hn, wp, wn, epi);
}

template <typename V>
void launch_ring_variant(int pf, int nt, const float* X, int64_t ldx, float* Y, int64_t ldy,
                         int n_rows, int64_t c_off, int64_t ncols_v, int rpb, const float* hp,
                         const float* hn, const float* wp, const float* wn, hipStream_t s) {
  // nt bit0 = nontemporal loads, bit1 = nontemporal stores
#define DOL_RING_CASE(PFV, NTL, NTS)                                                         \
  if (pf == PFV && nt == (NTL + 2 * NTS)) {                                                \
    launch_ring<V, PFV, NTL, NTS>(X, ldx, Y, ldy, n_rows, c_off, ncols_v, rpb, hp, hn, wp, wn, s); \
    return;                                                                                \
  }
  DOL_RING_CASE(2, 0, 1)
  DOL_RING_CASE(4, 0, 1)
  DOL_RING_CASE(8, 0, 1)
  DOL_RING_CASE(4, 0, 0)
  DOL_RING_CASE(4, 1, 1)
  DOL_RING_CASE(8, 1, 1)
  DOL_RING_CASE(4, 1, 0)
#undef DOL_RING_CASE
  launch_ring<V, 4, false, true>(X, ldx, Y, ldy, n_rows, c_off, ncols_v, rpb, hp, hn, wp, wn, s);
}

int ring_rows_per_block(int n_rows, int64_t n_col_tiles, int pf) {
  int r = env_int("DOL_RING_ROWS", 0);
  if (r > 0) return r;
  (void)n_col_tiles;
  return pf < 4 ? pf : 4;  // see the ring kernel comment: 4 rows per tile, all loads up front
}

template <typename V, int RPB, class Epi = NoEpi>
void launch_csr(const float* X, int64_t ldx, float* Y, int64_t ldy, int n_rows, int64_t c_off,
                int64_t ncols_v, const int32_t* rowptr, const int32_t* col, const float* val,
                hipStream_t s, const Epi& epi = Epi{}) {
  const int64_t n_col_tiles = cdiv(ncols_v, kThreads);
  const int64_t n_rg = cdiv(n_rows, RPB);
  hipLaunchKernelGGL((csr_mix_kernel<V, RPB, Epi>), dim3(static_cast<unsigned>(n_col_tiles * n_rg)), dim3(kThreads), 0,
                     s, X, ldx, Y, ldy, n_rows, c_off, ncols_v, n_rg, rowptr, col, val, epi);
}

template <typename V, bool TH, bool AL, int MODE, bool WG>
void launch_prox(float* w, int64_t ldw, float* b, int64_t ldb, float* g, int64_t ldg,
                 const float* th, const float* a, int64_t lda, float rho, float lr, float mom,
                 int n_agents, int64_t c_off, int64_t ncols_v, hipStream_t s) {
  const int64_t n_col_tiles = cdiv(ncols_v, kThreads);
  // alpha is only read on this path (the kernel's pointer is non-const for the fused-dual variant)
  hipLaunchKernelGGL((prox_sgd_kernel<V, TH, AL, MODE, WG>), dim3(static_cast<unsigned>(n_col_tiles * n_agents)),
                     dim3(kThreads), 0, s, w, ldw, b, ldb, g, ldg, th, const_cast<float*>(a), lda, rho, -lr, mom,
                     c_off, ncols_v, n_col_tiles);
}

template <typename V, bool TH, bool AL, int MODE>
void dispatch_prox_wg(bool wg, float* w, int64_t ldw, float* b, int64_t ldb, float* g, int64_t ldg,
                      const float* th, const float* a, int64_t lda, float rho, float lr, float mom,
                      int n, int64_t c_off, int64_t nc, hipStream_t s) {
  if (wg) launch_prox<V, TH, AL, MODE, true>(w, ldw, b, ldb, g, ldg, th, a, lda, rho, lr, mom, n, c_off, nc, s);
  else launch_prox<V, TH, AL, MODE, false>(w, ldw, b, ldb, g, ldg, th, a, lda, rho, lr, mom, n, c_off, nc, s);
}

template <typename V, bool TH, bool AL>
void dispatch_prox_mode(int mode, bool wg, float* w, int64_t ldw, float* b, int64_t ldb, float* g,
                        int64_t ldg, const float* th, const float* a, int64_t lda, float rho,
                        float lr, float mom, int n, int64_t c_off, int64_t nc, hipStream_t s) {
  if (mode == 0) dispatch_prox_wg<V, TH, AL, 0>(wg, w, ldw, b, ldb, g, ldg, th, a, lda, rho, lr, mom, n, c_off, nc, s);
  else if (mode == 1) dispatch_prox_wg<V, TH, AL, 1>(wg, w, ldw, b, ldb, g, ldg, th, a, lda, rho, lr, mom, n, c_off, nc, s);
  else dispatch_prox_wg<V, TH, AL, 2>(wg, w, ldw, b, ldb, g, ldg, th, a, lda, rho, lr, mom, n, c_off, nc, s);
}

template <typename V>
void dispatch_prox(bool th, bool al, int mode, bool wg, float* w, int64_t ldw, float* b,
                   int64_t ldb, float* g, int64_t ldg, const float* tp, const float* ap,
                   int64_t lda, float rho, float lr, float mom, int n, int64_t c_off, int64_t nc,
                   hipStream_t s) {
  if (!th) dispatch_prox_mode<V, false, false>(mode, wg, w, ldw, b, ldb, g, ldg, tp, ap, lda, rho, lr, mom, n, c_off, nc, s);
  else if (!al) dispatch_prox_mode<V, true, false>(mode, wg, w, ldw, b, ldb, g, ldg, tp, ap, lda, rho, lr, mom, n, c_off, nc, s);
  else dispatch_prox_mode<V, true, true>(mode, wg, w, ldw, b, ldb, g, ldg, tp, ap, lda, rho, lr, mom, n, c_off, nc, s);
}


// Shared bodies of the plain and epilogue (DGD) forms of the two sparse mixes.
template <class Epi>
int mix_csr_impl(const char* nm, const float* X, int64_t ldx, int32_t x_rows, float* Y, int64_t ldy,
                 int32_t n_rows, int64_t P, const int32_t* rowptr, const int32_t* col, const float* val,
                 const Epi& epi, bool epi_vec_ok, hipStream_t s) {
  if (n_rows < 0 || P < 0 || x_rows < 0) return fail(DOL_EINVAL, "%s: negative size", nm);
  if (n_rows == 0 || P == 0) { g_err[0] = '\0'; return DOL_OK; }
  if (!X || !Y || !rowptr || (!col && x_rows > 0) || (!val && x_rows > 0))
    return fail(DOL_EINVAL, "%s: null pointer", nm);
  if (ldx < P || ldy < P) return fail(DOL_EINVAL, "%s: ld < P", nm);
  if (X == Y) return fail(DOL_EINVAL, "%s: X and Y alias (Jacobi mix needs two buffers)", nm);
  const bool vec_ok = row_vec_ok(X, ldx) && row_vec_ok(Y, ldy) && epi_vec_ok;
  const ColSplit cs = split_cols(P, vec_ok);
  constexpr int RPB = 16;
  constexpr int XW = 32, XPASSES = 2;  // XCD-pinned tiles: 512 B of a row, 16 rows per block
  // 0 = 4 KiB tiles, 1 = XCD-pinned (DOL_CSR_MODE; default: XCD-pinned from 512 rows)
  const int mode = env_int("DOL_CSR_MODE", -1);
  if (mul_sat(cdiv(cs.n4, kThreads), cdiv(n_rows, RPB)) > kMaxBlocks)
    return fail(DOL_EINVAL, "%s: problem too large for one launch", nm);
  int64_t done4 = 0;
  const bool use_xcd = cs.n4 >= XW && (mode == 1 || (mode < 0 && n_rows >= 512));
  if (use_xcd) {
    const int passes = env_int("DOL_CSR_PASSES", XPASSES);
    auto go = [&](auto pc) {
      constexpr int PS = decltype(pc)::value;
      const int64_t nt = cs.n4 / XW;
      const int64_t nrb = cdiv(n_rows, (kThreads / XW) * PS);
      const int64_t grid = cdiv(nt, 8) * 8 * nrb;
      if (grid > kMaxBlocks * 8) return false;
      hipLaunchKernelGGL((csr_xcd_kernel<XW, PS, Epi>), dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, s, X,
                         ldx, Y, ldy, n_rows, static_cast<uint32_t>(nrb), static_cast<uint32_t>(nt), rowptr, col,
                         val, epi);
      done4 = nt * XW;
      return true;
    };
    using std::integral_constant;
    const bool ok = passes == 1 ? go(integral_constant<int, 1>{})
                    : passes == 4 ? go(integral_constant<int, 4>{}) : go(integral_constant<int, XPASSES>{});
    if (!ok) return fail(DOL_EINVAL, "%s: problem too large for one launch", nm);
  }
  if (cs.n4 > done4)  // column offset through c_off so the epilogue sees absolute columns
    launch_csr<f4, RPB, Epi>(X, ldx, Y, ldy, n_rows, done4 * 4, cs.n4 - done4, rowptr, col, val, s, epi);
  if (cs.tail > 0)
    launch_csr<float, RPB, Epi>(X, ldx, Y, ldy, n_rows, cs.n4 * 4, cs.tail, rowptr, col, val, s, epi);
  return check_launch(nm);
}

template <class Epi>
int mix_ring_impl(const char* nm, const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t n_rows, int64_t P,
                  const float* halo_prev, const float* halo_next, const float* w_prev, const float* w_next,
                  const Epi& epi, bool epi_vec_ok, hipStream_t s) {
  constexpr bool kPlain = std::is_same<Epi, NoEpi>::value;
  if (n_rows < 0 || P < 0) return fail(DOL_EINVAL, "%s: negative size", nm);
  if (n_rows == 0 || P == 0) { g_err[0] = '\0'; return DOL_OK; }
  if (!X || !Y || !w_prev || !w_next) return fail(DOL_EINVAL, "%s: null pointer", nm);
  if (ldx < P || ldy < P) return fail(DOL_EINVAL, "%s: ld < P", nm);
  if (X == Y) return fail(DOL_EINVAL, "%s: X and Y alias (Jacobi mix needs two buffers)", nm);
  if ((halo_prev == nullptr) != (halo_next == nullptr)) return fail(DOL_EINVAL, "%s: pass both halos or neither", nm);
  if (!halo_prev) {
    if (n_rows < 3) return fail(DOL_EINVAL, "%s: wrap-around ring needs n_rows >= 3", nm);
    halo_prev = X + int64_t(n_rows - 1) * ldx;
    halo_next = X;
  }
  const bool vec_ok = row_vec_ok(X, ldx) && row_vec_ok(Y, ldy) && aligned16(halo_prev) && aligned16(halo_next) &&
                      epi_vec_ok;
  const ColSplit cs = split_cols(P, vec_ok);
  if (cs.n4 > 0) {
    const int64_t nct = cdiv(cs.n4, kThreads);
    bool dma = true;
    if constexpr (kPlain) dma = env_int("DOL_RING_DMA", 1) != 0;
    if (dma) {
      constexpr int R = 4;
      if (mul_sat(nct, cdiv(n_rows, R)) > kMaxBlocks) return fail(DOL_EINVAL, "%s: problem too large for one launch", nm);
      if (env_int("DOL_RING_NTI", 1))
        hipLaunchKernelGGL((ring_mix_dma_kernel<R, Epi, true>), dim3(static_cast<unsigned>(nct * cdiv(n_rows, R))),
                           dim3(kThreads), 0, s, X, ldx, Y, ldy, n_rows, cs.n4, nct, halo_prev, halo_next, w_prev, w_next, epi);
      else
      hipLaunchKernelGGL((ring_mix_dma_kernel<R, Epi>), dim3(static_cast<unsigned>(nct * cdiv(n_rows, R))), dim3(kThreads),
                         0, s, X, ldx, Y, ldy, n_rows, cs.n4, nct, halo_prev, halo_next, w_prev, w_next, epi);
    } else if constexpr (kPlain) {
      const int pf = env_int("DOL_RING_PF", 4);
      const int nt = env_int("DOL_RING_NT", 2);
      const int rpb = ring_rows_per_block(n_rows, nct, pf);
      if (mul_sat(nct, cdiv(n_rows, rpb)) > kMaxBlocks) return fail(DOL_EINVAL, "%s: problem too large for one launch", nm);
      launch_ring_variant<f4>(pf, nt, X, ldx, Y, ldy, n_rows, 0, cs.n4, rpb, halo_prev, halo_next, w_prev, w_next, s);
    }
  }
  if (cs.tail > 0) {
    const int rpb = ring_rows_per_block(n_rows, cdiv(cs.tail, kThreads), 4);
    if (mul_sat(cdiv(cs.tail, kThreads), cdiv(n_rows, rpb)) > kMaxBlocks)
      return fail(DOL_EINVAL, "%s: problem too large for one launch", nm);
    launch_ring<float, 4, false, true, Epi>(X, ldx, Y, ldy, n_rows, cs.n4 * 4, cs.tail, rpb, halo_prev, halo_next,
                                            w_prev, w_next, s, epi);
  }
  return check_launch(nm);
}

template <class Epi>
int ring_edges_impl(const char* nm, const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t n_rows, int64_t P,
                    const float* halo_prev, const float* halo_next, const float* w_prev, const float* w_next,
                    const Epi& epi, bool epi_vec_ok, hipStream_t s) {
  if (n_rows < 0 || P < 0) return fail(DOL_EINVAL, "%s: negative size", nm);
  if (n_rows == 0 || P == 0) { g_err[0] = '\0'; return DOL_OK; }
  if (!X || !Y || !w_prev || !w_next || !halo_prev || !halo_next) return fail(DOL_EINVAL, "%s: null pointer", nm);
  if (ldx < P || ldy < P) return fail(DOL_EINVAL, "%s: ld < P", nm);
  if (X == Y) return fail(DOL_EINVAL, "%s: X and Y alias (Jacobi mix needs two buffers)", nm);
  const bool vec_ok = row_vec_ok(X, ldx) && row_vec_ok(Y, ldy) && aligned16(halo_prev) && aligned16(halo_next) &&
                      epi_vec_ok;
  const ColSplit cs = split_cols(P, vec_ok);
  const unsigned ny = n_rows == 1 ? 1u : 2u;
  if (cs.n4 > 0)
    hipLaunchKernelGGL((ring_edges_kernel<f4, Epi>), dim3(static_cast<unsigned>(cdiv(cs.n4, kThreads)), ny),
                       dim3(kThreads), 0, s, X, ldx, Y, ldy, n_rows, int64_t(0), cs.n4, halo_prev, halo_next, w_prev,
                       w_next, epi);
  if (cs.tail > 0)
    hipLaunchKernelGGL((ring_edges_kernel<float, Epi>), dim3(static_cast<unsigned>(cdiv(cs.tail, kThreads)), ny),
                       dim3(kThreads), 0, s, X, ldx, Y, ldy, n_rows, cs.n4 * 4, cs.tail, halo_prev, halo_next, w_prev,
                       w_next, epi);
  return check_launch(nm);
}

}  // namespace

// ============================================================================
// C-ABI
// ============================================================================
extern "C" {

int dol_version(void) { return 100; }

const char* dol_last_error(void) { return g_err; }

struct BankBlock {
  hipMemGenericAllocationHandle_t handle;
  size_t size;    // the mapped (granularity-rounded) size: what unmap / address-free take
  int stage = 0;  // 0 mapped, 1 unmapped, 2 range freed (dol_bank_free resumes from here)
};
static std::mutex g_bank_mu;  // dol_bank_alloc's live blocks: VA -> physical handle + mapped size
static std::unordered_map<void*, BankBlock> g_bank_handles;
// Virtual address space retired by dol_bank_free (see there) -- counted, and
// capped: past the cap dol_bank_alloc refuses new blocks instead of reserving
// address space without bound.  Guarded by g_bank_mu.
static int64_t g_bank_retired = 0;
static int64_t g_bank_retired_blocks = 0;

int64_t dol_bank_retired_cap_bytes(void) {
  const int64_t gib = env_int("DOL_BANK_RETIRED_VA_CAP_GIB", 4096);  // 4 TiB: 128 retired 32 GiB matrices
  return gib > 0 ? gib << 30 : 0;
}

int64_t dol_bank_retired_bytes(void) {
  std::lock_guard<std::mutex> lk(g_bank_mu);
  return g_bank_retired;
}

int64_t dol_bank_retired_blocks(void) {
  std::lock_guard<std::mutex> lk(g_bank_mu);
  return g_bank_retired_blocks;
}

// A bank buffer as ONE physical allocation (hipMemCreate) mapped into a
// reserved VA range, instead of whatever hipMalloc's suballocator returns
// (tools/alloc_probe.hip measures the ring round on both).
int dol_bank_alloc(int64_t bytes, void** ptr, int64_t* mapped_bytes) {
  if (!ptr || !mapped_bytes || bytes <= 0 || bytes > 4 * dol::kMaxDim)
    return fail(DOL_EINVAL, "dol_bank_alloc: bad arguments");
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(DOL_EINVAL, "dol_bank_alloc: no device");
  *ptr = nullptr;
  *mapped_bytes = 0;
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gran = 0;
  hipError_t e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended);
  if (e != hipSuccess || gran == 0) return fail(-static_cast<int>(e ? e : hipErrorInvalidValue), "dol_bank_alloc: granularity: %s", hipGetErrorString(e));
  const size_t size = (static_cast<size_t>(bytes) + gran - 1) / gran * gran;
  if (!env_int("DOL_BANK_FREE_VA", 0)) {  // this block's range will be retired when freed: stay under the cap
    std::lock_guard<std::mutex> lk(g_bank_mu);
    int64_t live = 0;
    for (const auto& kv : g_bank_handles) live += static_cast<int64_t>(kv.second.size);
    const int64_t cap = dol_bank_retired_cap_bytes();
    if (g_bank_retired + live + static_cast<int64_t>(size) > cap)
      return fail(DOL_ECAP, "dol_bank_alloc: %zu bytes would take the retired + live mapped address space "
                  "(%lld + %lld bytes) past its cap of %lld bytes (DOL_BANK_RETIRED_VA_CAP_GIB); use torch's "
                  "allocator (DOL_BANK_ALLOC=torch)", size, static_cast<long long>(g_bank_retired),
                  static_cast<long long>(live), static_cast<long long>(cap));
  }
  hipMemGenericAllocationHandle_t h{};
  if ((e = hipMemCreate(&h, size, &prop, 0)) != hipSuccess)
    return fail(-static_cast<int>(e), "dol_bank_alloc: hipMemCreate(%zu): %s", size, hipGetErrorString(e));
  void* va = nullptr;
  if ((e = hipMemAddressReserve(&va, size, gran, nullptr, 0)) != hipSuccess) {
    (void)hipMemRelease(h);
    return fail(-static_cast<int>(e), "dol_bank_alloc: hipMemAddressReserve: %s", hipGetErrorString(e));
  }
  if ((e = hipMemMap(va, size, 0, h, 0)) != hipSuccess) {
    (void)hipMemAddressFree(va, size);
    (void)hipMemRelease(h);
    return fail(-static_cast<int>(e), "dol_bank_alloc: hipMemMap: %s", hipGetErrorString(e));
  }
  hipMemAccessDesc acc{};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  if ((e = hipMemSetAccess(va, size, &acc, 1)) != hipSuccess) {
    (void)hipMemUnmap(va, size);
    (void)hipMemAddressFree(va, size);
    (void)hipMemRelease(h);
    return fail(-static_cast<int>(e), "dol_bank_alloc: hipMemSetAccess: %s", hipGetErrorString(e));
  }
  {  // the handle lives until dol_bank_free has unmapped the range (create, map ... unmap, release)
    std::lock_guard<std::mutex> lk(g_bank_mu);
    g_bank_handles[va] = BankBlock{h, size};
  }
  *ptr = va;
  *mapped_bytes = static_cast<int64_t>(size);
  g_err[0] = '\0';
  return DOL_OK;
}

// Unmap, free the range, release the handle -- with the size recorded at
// allocation (mapped_bytes must match it).  The entry is erased only after all
// three succeed, so a failed step leaves the block registered and a later call
// retries from that step.
int dol_bank_free(void* ptr, int64_t mapped_bytes) {
  if (!ptr) return DOL_OK;
  std::lock_guard<std::mutex> lk(g_bank_mu);
  auto it = g_bank_handles.find(ptr);
  if (it == g_bank_handles.end()) return fail(DOL_EINVAL, "dol_bank_free: %p is not a dol_bank_alloc block", ptr);
  BankBlock& blk = it->second;
  if (mapped_bytes != static_cast<int64_t>(blk.size))
    return fail(DOL_EINVAL, "dol_bank_free: size %lld differs from the mapped %zu bytes",
                static_cast<long long>(mapped_bytes), blk.size);
  hipError_t e = hipSuccess;
  if (blk.stage == 0) {
    if ((e = hipMemUnmap(ptr, blk.size)) != hipSuccess)
      return fail(-static_cast<int>(e), "dol_bank_free: hipMemUnmap: %s", hipGetErrorString(e));
    blk.stage = 1;
  }
  if (blk.stage == 1 && !env_int("DOL_BANK_FREE_VA", 0)) {
    // The virtual range stays reserved (retired, never handed out again): on
    // this ROCm stack a new physical allocation mapped at a range a freed block
    // used is not what the GPU then reads and writes -- stale translations of
    // the old block.  tools/vmm_remap_probe.py, 12 map/free cycles in one
    // process (profiles/r05c_vmm_remap_probe.jsonl): with the range freed and
    // re-used, 7 of 11 re-mapped cycles returned wrong mix results; with the
    // range retired, or with nothing freed, all 12 were bit-exact.  A stale
    // translation to a released range is also the r04k illegal-address fault.
    // Retiring costs address space only (the physical memory is released).
    // DOL_BANK_FREE_VA=1 restores the freeing order (diagnostics only).
    // Counted in g_bank_retired (dol_bank_retired_bytes) against the cap that
    // dol_bank_alloc enforces.
    blk.stage = 2;
    g_bank_retired += static_cast<int64_t>(blk.size);
    g_bank_retired_blocks += 1;
  }
  if (blk.stage == 1) {
    if ((e = hipMemAddressFree(ptr, blk.size)) != hipSuccess)
      return fail(-static_cast<int>(e), "dol_bank_free: hipMemAddressFree: %s", hipGetErrorString(e));
    blk.stage = 2;
  }
  if ((e = hipMemRelease(blk.handle)) != hipSuccess)
    return fail(-static_cast<int>(e), "dol_bank_free: hipMemRelease: %s", hipGetErrorString(e));
  g_bank_handles.erase(it);
  g_err[0] = '\0';
  return DOL_OK;
}

int dol_mix_csr_f32(const float* X, int64_t ldx, int32_t x_rows, float* Y, int64_t ldy,
                    int32_t n_rows, int64_t P, const int32_t* rowptr, const int32_t* col,
                    const float* val, hipStream_t s) {
  DOL_DIMS_OK("dol_mix_csr_f32", ldx, ldy, P);
  return mix_csr_impl("dol_mix_csr_f32", X, ldx, x_rows, Y, ldy, n_rows, P, rowptr, col, val, NoEpi{}, true, s);
}

int dol_mix_ring_f32(const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t n_rows, int64_t P,
                     const float* halo_prev, const float* halo_next, const float* w_prev,
                     const float* w_next, hipStream_t s) {
  DOL_DIMS_OK("dol_mix_ring_f32", ldx, ldy, P);
  return mix_ring_impl("dol_mix_ring_f32", X, ldx, Y, ldy, n_rows, P, halo_prev, halo_next, w_prev, w_next,
                       NoEpi{}, true, s);
}

int dol_mix_ring_edges_f32(const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t n_rows, int64_t P,
                           const float* halo_prev, const float* halo_next, const float* w_prev,
                           const float* w_next, hipStream_t s) {
  DOL_DIMS_OK("dol_mix_ring_edges_f32", ldx, ldy, P);
  return ring_edges_impl("dol_mix_ring_edges_f32", X, ldx, Y, ldy, n_rows, P, halo_prev, halo_next, w_prev, w_next,
                         NoEpi{}, true, s);
}

}  // extern "C"

namespace {
// validation + dispatch of the BASELINE config-3 round (mix + local steps)
struct DgdArgs {
  const float* T; int64_t ldt; float* M; int64_t ldm;
  int32_t objective, steps; float lr, momentum; int first_step;
};

int check_dgd(const char* nm, const DgdArgs& d, int64_t P, bool* evec, int* mode) {
  if (!d.T) return fail(DOL_EINVAL, "%s: null target", nm);
  if (d.objective != 0 && d.objective != 1) return fail(DOL_EINVAL, "%s: objective must be 0 (least squares) or 1 (logistic)", nm);
  if (d.steps < 1) return fail(DOL_EINVAL, "%s: local_steps must be >= 1", nm);
  if (d.ldt < P) return fail(DOL_EINVAL, "%s: ldt < P", nm);
  *mode = (d.momentum == 0.0f) ? 0 : (d.first_step ? 1 : 2);
  if (*mode != 0 && (!d.M || d.ldm < P)) return fail(DOL_EINVAL, "%s: momentum needs a momentum buffer with ldm >= P", nm);
  *evec = row_vec_ok(d.T, d.ldt) && (*mode == 0 || row_vec_ok(d.M, d.ldm));
  return DOL_OK;
}

template <class F>
int with_dgd_epi(const DgdArgs& d, int mode, int64_t P, F&& f) {
  static const int nt_env = env_int("DOL_DGD_EPI_NT", 3);
  // buffer offsets are 32-bit (rows of < 2^29 floats); longer rows: plain loads
  const int nt = (nt_env == 3 && P > (int64_t(1) << 29) - 16) ? 0 : nt_env;
  auto mk = [&](auto obj, auto md) {
    return f(DgdEpi<decltype(obj)::value, decltype(md)::value>{d.T, d.ldt, d.M, d.ldm, -d.lr, d.momentum, d.steps, nt});
  };
  using std::integral_constant;
  if (d.objective == 0) {
    if (mode == 0) return mk(integral_constant<int, 0>{}, integral_constant<int, 0>{});
    if (mode == 1) return mk(integral_constant<int, 0>{}, integral_constant<int, 1>{});
    return mk(integral_constant<int, 0>{}, integral_constant<int, 2>{});
  }
  if (mode == 0) return mk(integral_constant<int, 1>{}, integral_constant<int, 0>{});
  if (mode == 1) return mk(integral_constant<int, 1>{}, integral_constant<int, 1>{});
  return mk(integral_constant<int, 1>{}, integral_constant<int, 2>{});
}
}  // namespace

extern "C" {

int dol_dgd_ring_f32(const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t n_rows, int64_t P,
                     const float* halo_prev, const float* halo_next, const float* w_prev, const float* w_next,
                     const float* target, int64_t ldt, float* mom, int64_t ldm, int32_t objective,
                     int32_t local_steps, float lr, float momentum, int first_step, hipStream_t s) {
  DOL_DIMS_OK("dol_dgd_ring_f32", ldx, ldy, P, ldt, ldm);
  const char* nm = "dol_dgd_ring_f32";
  const DgdArgs d{target, ldt, mom, ldm, objective, local_steps, lr, momentum, first_step};
  bool evec = false;
  int mode = 0;
  if (n_rows > 0 && P > 0) {
    const int rc = check_dgd(nm, d, P, &evec, &mode);
    if (rc) return rc;
  }
  return with_dgd_epi(d, mode, P, [&](auto epi) {
    return mix_ring_impl(nm, X, ldx, Y, ldy, n_rows, P, halo_prev, halo_next, w_prev, w_next, epi, evec, s);
  });
}

int dol_dgd_ring_edges_f32(const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t n_rows, int64_t P,
                           const float* halo_prev, const float* halo_next, const float* w_prev, const float* w_next,
                           const float* target, int64_t ldt, float* mom, int64_t ldm, int32_t objective,
                           int32_t local_steps, float lr, float momentum, int first_step, hipStream_t s) {
  DOL_DIMS_OK("dol_dgd_ring_edges_f32", ldx, ldy, P, ldt, ldm);
  const char* nm = "dol_dgd_ring_edges_f32";
  const DgdArgs d{target, ldt, mom, ldm, objective, local_steps, lr, momentum, first_step};
  bool evec = false;
  int mode = 0;
  if (n_rows > 0 && P > 0) {
    const int rc = check_dgd(nm, d, P, &evec, &mode);
    if (rc) return rc;
  }
  return with_dgd_epi(d, mode, P, [&](auto epi) {
    return ring_edges_impl(nm, X, ldx, Y, ldy, n_rows, P, halo_prev, halo_next, w_prev, w_next, epi, evec, s);
  });
}

int dol_dgd_csr_f32(const float* X, int64_t ldx, int32_t x_rows, float* Y, int64_t ldy, int32_t n_rows, int64_t P,
                    const int32_t* rowptr, const int32_t* col, const float* val, const float* target, int64_t ldt,
                    float* mom, int64_t ldm, int32_t objective, int32_t local_steps, float lr, float momentum,
                    int first_step, hipStream_t s) {
  DOL_DIMS_OK("dol_dgd_csr_f32", ldx, ldy, P, ldt, ldm);
  const char* nm = "dol_dgd_csr_f32";
  const DgdArgs d{target, ldt, mom, ldm, objective, local_steps, lr, momentum, first_step};
  bool evec = false;
  int mode = 0;
  if (n_rows > 0 && P > 0) {
    const int rc = check_dgd(nm, d, P, &evec, &mode);
    if (rc) return rc;
  }
  return with_dgd_epi(d, mode, P, [&](auto epi) {
    return mix_csr_impl(nm, X, ldx, x_rows, Y, ldy, n_rows, P, rowptr, col, val, epi, evec, s);
  });
}

int dol_mix_dense_f32(const float* W, int64_t ldw, const float* X, int64_t ldx, float* Y, int64_t ldy,
                      int32_t M, int32_t K, int64_t P, hipStream_t s) {
  DOL_DIMS_OK("dol_mix_dense_f32", ldw, ldx, ldy, P);
  if (M < 0 || K < 0 || P < 0) return fail(DOL_EINVAL, "dol_mix_dense_f32: negative size");
  if (M == 0 || P == 0) { g_err[0] = '\0'; return DOL_OK; }
  if (!W || !X || !Y) return fail(DOL_EINVAL, "dol_mix_dense_f32: null pointer");
  if (ldw < K || ldx < P || ldy < P) return fail(DOL_EINVAL, "dol_mix_dense_f32: ld too small");
  if (X == Y) return fail(DOL_EINVAL, "dol_mix_dense_f32: X and Y alias");
  const uint32_t nrt = static_cast<uint32_t>(cdiv(M, kDBM));
  const int64_t nct = cdiv(P, kDBN);
  if (int64_t(nrt) * nct > (int64_t(1) << 31)) return fail(DOL_EINVAL, "dol_mix_dense_f32: too large");
  const bool va = aligned16(W) && ldw % 4 == 0 && K % 4 == 0;
  const bool vb = aligned16(X) && ldx % 4 == 0;
  const dim3 grid(static_cast<unsigned>(int64_t(nrt) * nct));
  if (va && vb) hipLaunchKernelGGL((dense_mix_mfma_kernel<true, true>), grid, dim3(256), 0, s, W, ldw, X, ldx, Y, ldy, M, K, P, nrt);
  else if (va) hipLaunchKernelGGL((dense_mix_mfma_kernel<true, false>), grid, dim3(256), 0, s, W, ldw, X, ldx, Y, ldy, M, K, P, nrt);
  else if (vb) hipLaunchKernelGGL((dense_mix_mfma_kernel<false, true>), grid, dim3(256), 0, s, W, ldw, X, ldx, Y, ldy, M, K, P, nrt);
  else hipLaunchKernelGGL((dense_mix_mfma_kernel<false, false>), grid, dim3(256), 0, s, W, ldw, X, ldx, Y, ldy, M, K, P, nrt);
  return check_launch("dol_mix_dense_f32");
}

// kernel of dol_mix_ring_steps_f32 chosen by dol_ring_steps_set_variant (0:
// DOL_RING_STREAM); atomic, so a setter on one thread never tears a launch's
// read on another (dol_mix_ring_steps_ex_f32 takes the variant per call)
static std::atomic<int> g_ring_steps_variant{0};

int dol_ring_steps_set_variant(int32_t variant) {
  if (variant < 0 || variant > kRingStepsVariants)
    return fail(DOL_EINVAL, "dol_ring_steps_set_variant: variant %d outside 0 (default) / 1 (tiles) / 2 (stream) / 3-5 (LDS-DMA stream: plain, synchronised, sweep)", variant);
  const int prev = g_ring_steps_variant.exchange(variant, std::memory_order_relaxed);
  g_err[0] = '\0';
  return prev;
}

int dol_mix_ring_steps_f32(const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t n_rows,
                           int64_t P, int32_t steps, const float* w_prev, const float* w_next,
                           hipStream_t s) {
  return dol_mix_ring_steps_ex_f32(X, ldx, Y, ldy, n_rows, P, steps, w_prev, w_next, 0, s);
}

int dol_mix_ring_steps_ex_f32(const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t n_rows,
                              int64_t P, int32_t steps, const float* w_prev, const float* w_next,
                              int32_t variant, hipStream_t s) {
  DOL_DIMS_OK("dol_mix_ring_steps_f32", ldx, ldy, P);
  if (variant < 0 || variant > kRingStepsVariants)
    return fail(DOL_EINVAL, "dol_mix_ring_steps_ex_f32: variant %d outside 0 (process setting) / 1 (tiles) / 2 (stream) / 3-5 (LDS-DMA stream: plain, synchronised, sweep)", variant);
  if (n_rows < 0 || P < 0 || steps < 0) return fail(DOL_EINVAL, "dol_mix_ring_steps_f32: negative size");
  if (n_rows == 0 || P == 0) { g_err[0] = '\0'; return DOL_OK; }
  if (!X || !Y || !w_prev || !w_next) return fail(DOL_EINVAL, "dol_mix_ring_steps_f32: null pointer");
  if (ldx < P || ldy < P) return fail(DOL_EINVAL, "dol_mix_ring_steps_f32: ld < P");
  if (X == Y) return fail(DOL_EINVAL, "dol_mix_ring_steps_f32: X and Y alias");
  if (n_rows < 3) return fail(DOL_EINVAL, "dol_mix_ring_steps_f32: a ring needs n_rows >= 3");
  if (steps == 0) return fail(DOL_EINVAL, "dol_mix_ring_steps_f32: steps must be >= 1");
  const bool vec = row_vec_ok(X, ldx) && row_vec_ok(Y, ldy) && P % 4 == 0;
  if (!vec || steps > 8) return fail(DOL_EINVAL, "dol_mix_ring_steps_f32: needs 16-B aligned rows, P %% 4 == 0 and steps <= 8 (compose launches otherwise)");
  // The register-tile ring_steps_kernel unless DOL_RING_STREAM=1
  // (ring_stream_kernel: 1024-row tiles, 8 rows in flight, nontemporal loads).
  // eps = 5 at 8192 x 2^20, alternating on one box (profiles/r03_eps_stream.txt):
  // box A stream 12.38 / 12.39 vs tiles 12.61 / 12.62 ms; box C stream-NT 11.60 /
  // 12.00 / 11.76 vs tiles 11.90 / 11.92 / 11.80; box E stream-NT 12.95-13.19 vs
  // tiles 11.96-12.67; the stream kernel alone ran 10.66 ms on one box and 12.72
  // on another with the same ring round (10.92 ms): no consistent winner, so the
  // r02 default stays.  Clock 1 % below the ring kernel's for both (2424 / 2408
  // vs 2439 MHz, GRBM_GUI_ACTIVE per XCD over the kernel's time).
  // Which of the two wins follows where the bank's pages landed, as for the
  // parameter-major mix (profiles/r03_pm_stage_order.txt): ops.tune_ring_steps_variant
  // times both on the buffers in use and keeps the faster (dol_ring_steps_set_variant).
  static const int stream_env = [] { const char* e = getenv("DOL_RING_STREAM"); return e ? atoi(e) : 0; }();
  const int v = variant != 0 ? variant : g_ring_steps_variant.load(std::memory_order_relaxed);
  // stream: 0 register tiles, 1 register stream, 3 / 4 / 5 LDS-DMA stream
  // (plain / block-synchronised / column-tile-fastest sweep of 64-row tiles)
  const int stream = v == 0 ? stream_env : (v == 2 ? 1 : v >= 3 ? v : 0);
  static const int stream_t = [] { const char* e = getenv("DOL_RING_STREAM_T"); return e ? atoi(e) : 1024; }();
  static const int stream_pf = [] { const char* e = getenv("DOL_RING_STREAM_PF"); return e ? atoi(e) : 8; }();
  static const int stream_nt = [] { const char* e = getenv("DOL_RING_STREAM_NT"); return e ? atoi(e) : 1; }();
  auto go_stream_pf = [&](auto steps_c, int T, auto pf_c) {
    constexpr int S = decltype(steps_c)::value, PF = decltype(pf_c)::value;
    const int64_t nv = P / 4;
    const uint32_t nct = static_cast<uint32_t>(cdiv(nv, kThreads));
    const int64_t nrt = cdiv(n_rows, T);
    const int64_t grid = cdiv(nct, 8) * 8 * nrt;
    if (grid > kMaxBlocks) return fail(DOL_EINVAL, "dol_mix_ring_steps_f32: too large");
    // DOL_RING_STREAM_LDS (diagnostics): bytes of unused LDS per block, to cap
    // the blocks per CU (the kernel itself uses none)
    static const int pad_lds = [] { const char* e = getenv("DOL_RING_STREAM_LDS"); return e ? atoi(e) : 0; }();
    auto go_k = [&](auto kern) {
      if (pad_lds > 65536)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, pad_lds);
      hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(grid)), dim3(kThreads), pad_lds, s, X, ldx, Y, ldy, n_rows, nv,
                         nct, w_prev, w_next, static_cast<uint32_t>(nrt), T);
    };
    if (stream_nt) go_k(ring_stream_kernel<S, PF, true>);
    else go_k(ring_stream_kernel<S, PF, false>);
    return check_launch("dol_mix_ring_steps_f32");
  };
  // variant 3: ring_stream_dma_kernel, D-row LDS-DMA ring per wave (DOL_RING_DMA_D 8 / 16)
  static const int dma_d = [] { const char* e = getenv("DOL_RING_DMA_D"); return e ? atoi(e) : 8; }();
  // DOL_RING_DMA_SYNC=1: one raw barrier per 8 steps keeps a block's waves on the same rows
  static const int dma_sync = [] { const char* e = getenv("DOL_RING_DMA_SYNC"); return e ? atoi(e) : 0; }();
  // DOL_RING_DMA_ORDER: 0 = XCD-aware row-tile order, 1 = column tile fastest (sweep)
  static const int dma_order = [] { const char* e = getenv("DOL_RING_DMA_ORDER"); return e ? atoi(e) : 0; }();
  auto go_stream_dma = [&](auto steps_c, int T) {
    constexpr int S = decltype(steps_c)::value;
    const bool sync = stream == 4 || dma_sync;
    const int order = stream == 5 ? 1 : dma_order;
    if (stream == 5) T = 64;
    const int64_t nv = P / 4;
    const uint32_t nct = static_cast<uint32_t>(cdiv(nv, kThreads));
    const int64_t nrt = cdiv(n_rows, T);
    const int64_t grid = cdiv(nct, 8) * 8 * nrt;
    if (grid > kMaxBlocks) return fail(DOL_EINVAL, "dol_mix_ring_steps_f32: too large");
    // DOL_RING_DMA_PROBE=1 (diagnostics, wrong results): the same kernel as a copy
    static const int dma_probe = [] { const char* e = getenv("DOL_RING_DMA_PROBE"); return e ? atoi(e) : 0; }();
    if constexpr (S == 5) {
      if (dma_probe == 1) {
        hipLaunchKernelGGL((ring_stream_dma_kernel<S, 8, 8, 1>), dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, s,
                           X, ldx, Y, ldy, n_rows, nv, nct, w_prev, w_next, static_cast<uint32_t>(nrt), T, order);
        return check_launch("dol_mix_ring_steps_f32");
      }
    }
    if (sync)
      hipLaunchKernelGGL((ring_stream_dma_kernel<S, 8, 8, 0, true>), dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, s,
                         X, ldx, Y, ldy, n_rows, nv, nct, w_prev, w_next, static_cast<uint32_t>(nrt), T, order);
    else if (dma_d == 16)
      hipLaunchKernelGGL((ring_stream_dma_kernel<S, 16, 8>), dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, s, X,
                         ldx, Y, ldy, n_rows, nv, nct, w_prev, w_next, static_cast<uint32_t>(nrt), T, order);
    else
      hipLaunchKernelGGL((ring_stream_dma_kernel<S, 8, 8>), dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, s, X,
                         ldx, Y, ldy, n_rows, nv, nct, w_prev, w_next, static_cast<uint32_t>(nrt), T, order);
    return check_launch("dol_mix_ring_steps_f32");
  };
  auto go_stream = [&](auto steps_c, int T) {
    if (stream >= 3) return go_stream_dma(steps_c, T);
    if (stream_pf == 16) return go_stream_pf(steps_c, T, std::integral_constant<int, 16>{});
    if (stream_pf == 4) return go_stream_pf(steps_c, T, std::integral_constant<int, 4>{});
    return go_stream_pf(steps_c, T, std::integral_constant<int, 8>{});
  };

  auto go_v = [&](auto steps_c, auto r_c, auto v_c) {
    constexpr int S = decltype(steps_c)::value, R = decltype(r_c)::value;
    // the stream kernels wrap at most once (PF <= 16); the LDS-DMA one's buffer
    // stores address a row in 32 bits
    if (stream && n_rows >= 2 * S + 16 + 1 && (stream < 3 || ldy * 4 < (int64_t(1) << 31))) {
      return go_stream(steps_c, stream_t >= 64 ? stream_t : 1024);
    }
    using V = typename decltype(v_c)::type;
    const int64_t nv = P / Vec<V>::W;
    const uint32_t nct = static_cast<uint32_t>(cdiv(nv, kThreads));
    const int64_t nrt = cdiv(n_rows, R);
    const int64_t grid = cdiv(nct, 8) * 8 * nrt;
    if (grid > kMaxBlocks) return fail(DOL_EINVAL, "dol_mix_ring_steps_f32: too large");
    hipLaunchKernelGGL((ring_steps_kernel<S, R, V>), dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, s, X, ldx, Y,
                       ldy, n_rows, nv, nct, w_prev, w_next, static_cast<uint32_t>(nrt));
    return check_launch("dol_mix_ring_steps_f32");
  };
  struct TF4 { using type = f4; };
  auto go = [&](auto steps_c, auto r_c) { return go_v(steps_c, r_c, TF4{}); };
  using std::integral_constant;
  // tile heights measured at 8192 x 2^20 (tools/bench_configs.py ring-eps<S>):
  // R = 6 for S <= 3, 14 for S = 4, 22 for S = 5-6, 30 for S = 7-8
  switch (steps) {
    case 1: return go(integral_constant<int, 1>{}, integral_constant<int, 4>{});
    case 2: return go(integral_constant<int, 2>{}, integral_constant<int, 6>{});
    case 3: return go(integral_constant<int, 3>{}, integral_constant<int, 6>{});
    case 4: return go(integral_constant<int, 4>{}, integral_constant<int, 14>{});
    case 5: return go(integral_constant<int, 5>{}, integral_constant<int, 22>{});
    case 6: return go(integral_constant<int, 6>{}, integral_constant<int, 22>{});
    case 7: return go(integral_constant<int, 7>{}, integral_constant<int, 30>{});
    default: return go(integral_constant<int, 8>{}, integral_constant<int, 30>{});
  }
}

int dol_prox_admm_sgd_f32(float* w, int64_t ldw, float* buf, int64_t ldb, float* g, int64_t ldg,
                          const float* theta, const float* alpha, int64_t lda, float rho, float lr,
                          float momentum, int first_step, int write_grad, int32_t n_agents,
                          int64_t P, hipStream_t s) {
  DOL_DIMS_OK("dol_prox_admm_sgd_f32", ldw, ldb, ldg, lda, P);
  if (n_agents < 0 || P < 0) return fail(DOL_EINVAL, "dol_prox_admm_sgd_f32: negative size");
  if (n_agents == 0 || P == 0) { g_err[0] = '\0'; return DOL_OK; }
  if (!w || !g) return fail(DOL_EINVAL, "dol_prox_admm_sgd_f32: null w or g");
  if (alpha && !theta) return fail(DOL_EINVAL, "dol_prox_admm_sgd_f32: alpha without theta");
  const int mode = (momentum == 0.0f) ? 0 : (first_step ? 1 : 2);
  if (mode != 0 && !buf) return fail(DOL_EINVAL, "dol_prox_admm_sgd_f32: momentum needs buf");
  if (ldw < P || ldg < P || (mode != 0 && ldb < P) || (alpha && lda < P))
    return fail(DOL_EINVAL, "dol_prox_admm_sgd_f32: ld < P");
  const bool vec_ok = row_vec_ok(w, ldw) && row_vec_ok(g, ldg) && (mode == 0 || row_vec_ok(buf, ldb)) &&
                      row_vec_ok(theta, 0) && row_vec_ok(alpha, alpha ? lda : 0);
  const ColSplit cs = split_cols(P, vec_ok);
  if (mul_sat(cdiv(cs.n4 + cs.tail, kThreads), n_agents) > kMaxBlocks)
    return fail(DOL_EINVAL, "dol_prox_admm_sgd_f32: problem too large for one launch");
  const bool th = theta != nullptr, al = alpha != nullptr, wg = write_grad != 0;
  if (cs.n4 > 0)
    dispatch_prox<f4>(th, al, mode, wg, w, ldw, buf, ldb, g, ldg, theta, alpha, lda, rho, lr,
                          momentum, n_agents, 0, cs.n4, s);
  if (cs.tail > 0)
    dispatch_prox<float>(th, al, mode, wg, w, ldw, buf, ldb, g, ldg, theta, alpha, lda, rho, lr,
                         momentum, n_agents, cs.n4 * 4, cs.tail, s);
  return check_launch("dol_prox_admm_sgd_f32");
}

int dol_admm_step_dual_f32(float* w, int64_t ldw, float* buf, int64_t ldb, float* g, int64_t ldg,
                           const float* theta, float* alpha, int64_t lda, float rho, float lr,
                           float momentum, int first_step, int write_grad, int32_t n_agents, int64_t P,
                           hipStream_t s) {
  DOL_DIMS_OK("dol_admm_step_dual_f32", ldw, ldb, ldg, lda, P);
  if (n_agents < 0 || P < 0) return fail(DOL_EINVAL, "dol_admm_step_dual_f32: negative size");
  if (n_agents == 0 || P == 0) { g_err[0] = '\0'; return DOL_OK; }
  if (!w || !g || !theta || !alpha) return fail(DOL_EINVAL, "dol_admm_step_dual_f32: null pointer");
  const int mode = (momentum == 0.0f) ? 0 : (first_step ? 1 : 2);
  if (mode != 0 && !buf) return fail(DOL_EINVAL, "dol_admm_step_dual_f32: momentum needs buf");
  if (ldw < P || ldg < P || lda < P || (mode != 0 && ldb < P)) return fail(DOL_EINVAL, "dol_admm_step_dual_f32: ld < P");
  const bool vec_ok = row_vec_ok(w, ldw) && row_vec_ok(g, ldg) && (mode == 0 || row_vec_ok(buf, ldb)) &&
                      row_vec_ok(theta, 0) && row_vec_ok(alpha, lda);
  const ColSplit cs = split_cols(P, vec_ok);
  if (mul_sat(cdiv(cs.n4 + cs.tail, kThreads), n_agents) > kMaxBlocks) return fail(DOL_EINVAL, "dol_admm_step_dual_f32: too large");
  auto launch = [&](auto vtag, auto mode_c, auto wg_c, int64_t c_off, int64_t nc) {
    using V = decltype(vtag);
    constexpr int M = decltype(mode_c)::value;
    constexpr bool WG = decltype(wg_c)::value;
    const int64_t nct = cdiv(nc, kThreads);
    hipLaunchKernelGGL((prox_sgd_kernel<V, true, true, M, WG, true>), dim3(static_cast<unsigned>(nct * n_agents)),
                       dim3(kThreads), 0, s, w, ldw, buf, ldb, g, ldg, theta, alpha, lda, rho, -lr, momentum, c_off,
                       nc, nct);
  };
  auto by_mode = [&](auto vtag, int64_t c_off, int64_t nc) {
    using std::integral_constant;
    const bool wg = write_grad != 0;
    if (mode == 0) { if (wg) launch(vtag, integral_constant<int, 0>{}, std::true_type{}, c_off, nc); else launch(vtag, integral_constant<int, 0>{}, std::false_type{}, c_off, nc); }
    else if (mode == 1) { if (wg) launch(vtag, integral_constant<int, 1>{}, std::true_type{}, c_off, nc); else launch(vtag, integral_constant<int, 1>{}, std::false_type{}, c_off, nc); }
    else { if (wg) launch(vtag, integral_constant<int, 2>{}, std::true_type{}, c_off, nc); else launch(vtag, integral_constant<int, 2>{}, std::false_type{}, c_off, nc); }
  };
  if (cs.n4 > 0) by_mode(f4{}, 0, cs.n4);
  if (cs.tail > 0) by_mode(float{}, cs.n4 * 4, cs.tail);
  return check_launch("dol_admm_step_dual_f32");
}

int dol_prox_grad_f32(float* g, int64_t ldg, const float* w, int64_t ldw, const float* theta,
                      const float* alpha, int64_t lda, float rho, int32_t n_agents, int64_t P,
                      hipStream_t s) {
  DOL_DIMS_OK("dol_prox_grad_f32", ldg, ldw, lda, P);
  if (n_agents < 0 || P < 0) return fail(DOL_EINVAL, "dol_prox_grad_f32: negative size");
  if (n_agents == 0 || P == 0) { g_err[0] = '\0'; return DOL_OK; }
  if (!g || !w || !theta) return fail(DOL_EINVAL, "dol_prox_grad_f32: null pointer");
  if (ldg < P || ldw < P || (alpha && lda < P)) return fail(DOL_EINVAL, "dol_prox_grad_f32: ld < P");
  const bool vec_ok = row_vec_ok(g, ldg) && row_vec_ok(w, ldw) && row_vec_ok(theta, 0) &&
                      row_vec_ok(alpha, alpha ? lda : 0);
  const ColSplit cs = split_cols(P, vec_ok);
  auto launch = [&](auto vtag, int64_t c_off, int64_t nc) {
    using V = decltype(vtag);
    const int64_t nct = cdiv(nc, kThreads);
    const dim3 grid(static_cast<unsigned>(nct * n_agents));
    if (alpha) hipLaunchKernelGGL((prox_grad_kernel<V, true>), grid, dim3(kThreads), 0, s, g, ldg, w, ldw, theta, alpha, lda, rho, c_off, nc, nct);
    else hipLaunchKernelGGL((prox_grad_kernel<V, false>), grid, dim3(kThreads), 0, s, g, ldg, w, ldw, theta, alpha, lda, rho, c_off, nc, nct);
  };
  if (mul_sat(cdiv(cs.n4 + cs.tail, kThreads), n_agents) > kMaxBlocks) return fail(DOL_EINVAL, "dol_prox_grad_f32: too large");
  if (cs.n4 > 0) launch(f4{}, 0, cs.n4);
  if (cs.tail > 0) launch(float{}, cs.n4 * 4, cs.tail);
  return check_launch("dol_prox_grad_f32");
}

int64_t dol_admm_dual_workspace_bytes(int32_t n_agents, int64_t P) {
  if (n_agents <= 0 || P <= 0 || P > dol::kMaxDim) return 0;
  // the scalar path has the most chunks: cdiv(P, kThreads*kDualIters)
  return int64_t(n_agents) * cdiv(P, int64_t(kThreads) * kDualIters) * int64_t(sizeof(double));
}

int dol_admm_dual_f32(float* alpha, int64_t lda, const float* w, int64_t ldw, const float* theta,
                      float rho, int32_t n_agents, int64_t P, double* resid_sq, void* work,
                      hipStream_t s) {
  DOL_DIMS_OK("dol_admm_dual_f32", lda, ldw, P);
  if (n_agents < 0 || P < 0) return fail(DOL_EINVAL, "dol_admm_dual_f32: negative size");
  if (n_agents == 0) { g_err[0] = '\0'; return DOL_OK; }
  if (P > 0 && (!alpha || !w || !theta)) return fail(DOL_EINVAL, "dol_admm_dual_f32: null pointer");
  if (resid_sq && !work && P > 0) return fail(DOL_EINVAL, "dol_admm_dual_f32: resid_sq needs a workspace");
  if (lda < P || ldw < P) return fail(DOL_EINVAL, "dol_admm_dual_f32: ld < P");
  if (P == 0) {
    if (resid_sq) (void)hipMemsetAsync(resid_sq, 0, sizeof(double) * n_agents, s);
    return check_launch("dol_admm_dual_f32");
  }
  const bool vec = row_vec_ok(alpha, lda) && row_vec_ok(w, ldw) && row_vec_ok(theta, 0);
  const int64_t per_block = int64_t(kThreads) * kDualIters;
  const int64_t chunks = vec ? std::max<int64_t>(1, cdiv(P / 4, per_block)) : cdiv(P, per_block);
  if (mul_sat(chunks, n_agents) > kMaxBlocks) return fail(DOL_EINVAL, "dol_admm_dual_f32: problem too large");
  double* partial = static_cast<double*>(work);
  const dim3 grid(static_cast<unsigned>(chunks * n_agents));
  if (resid_sq) {
    if (vec) hipLaunchKernelGGL((admm_dual_kernel<true, true>), grid, dim3(kThreads), 0, s, alpha, lda, w, ldw, theta, rho, P, chunks, partial);
    else hipLaunchKernelGGL((admm_dual_kernel<false, true>), grid, dim3(kThreads), 0, s, alpha, lda, w, ldw, theta, rho, P, chunks, partial);
    hipLaunchKernelGGL(resid_reduce_kernel, dim3(n_agents), dim3(kThreads), 0, s, partial, chunks, resid_sq);
  } else {
    if (vec) hipLaunchKernelGGL((admm_dual_kernel<true, false>), grid, dim3(kThreads), 0, s, alpha, lda, w, ldw, theta, rho, P, chunks, partial);
    else hipLaunchKernelGGL((admm_dual_kernel<false, false>), grid, dim3(kThreads), 0, s, alpha, lda, w, ldw, theta, rho, P, chunks, partial);
  }
  return check_launch("dol_admm_dual_f32");
}

int64_t dol_admm_ls_round_workspace_bytes(int32_t m, int64_t P) {
  if (m <= 0 || P <= 0 || P > dol::kMaxDim) return 0;
  return 2 * dol_admm_dual_workspace_bytes(m, P);  // ||w - theta||^2 and ||alpha||^2 partials
}

int dol_admm_ls_round_f32(float* w, int64_t ldw, float* buf, int64_t ldb, float* alpha, int64_t lda,
                          const float* target, int64_t ldt, const float* theta, const int32_t* agents,
                          const int32_t* first, int32_t m, int64_t P, float rho, float lr, float momentum,
                          int32_t local_steps, double* resid_sq, double* alpha_sq, void* work, hipStream_t s) {
  DOL_DIMS_OK("dol_admm_ls_round_f32", ldw, ldb, lda, ldt, P);
  const char* nm = "dol_admm_ls_round_f32";
  if (m < 0 || P < 0 || local_steps < 0) return fail(DOL_EINVAL, "%s: negative size", nm);
  if (m == 0) { g_err[0] = '\0'; return DOL_OK; }
  const bool mom = momentum != 0.0f;
  if (P > 0 && (!w || !alpha || !target || !theta || (mom && !buf))) return fail(DOL_EINVAL, "%s: null pointer", nm);
  if ((resid_sq == nullptr) != (alpha_sq == nullptr)) return fail(DOL_EINVAL, "%s: pass both residual outputs or neither", nm);
  if (resid_sq && !work && P > 0) return fail(DOL_EINVAL, "%s: residuals need a workspace", nm);
  if (ldw < P || lda < P || ldt < P || (mom && ldb < P)) return fail(DOL_EINVAL, "%s: ld < P", nm);
  if (P == 0) {
    if (resid_sq) {
      (void)hipMemsetAsync(resid_sq, 0, sizeof(double) * m, s);
      (void)hipMemsetAsync(alpha_sq, 0, sizeof(double) * m, s);
    }
    return check_launch(nm);
  }
  const bool vec = row_vec_ok(w, ldw) && row_vec_ok(alpha, lda) && row_vec_ok(target, ldt) && row_vec_ok(theta, 0) &&
                   (!mom || row_vec_ok(buf, ldb));
  const int64_t per_block = int64_t(kThreads) * kDualIters;
  const int64_t chunks = vec ? std::max<int64_t>(1, cdiv(P / 4, per_block)) : cdiv(P, per_block);
  if (mul_sat(chunks, m) > kMaxBlocks) return fail(DOL_EINVAL, "%s: problem too large", nm);
  double* partial = static_cast<double*>(work);
  const dim3 grid(static_cast<unsigned>(chunks * m));
  auto go = [&](auto vc, auto mc, auto rc) {
    hipLaunchKernelGGL((admm_ls_round_kernel<decltype(vc)::value, decltype(mc)::value, decltype(rc)::value>), grid,
                       dim3(kThreads), 0, s, w, ldw, buf, ldb, alpha, lda, target, ldt, theta, agents, first, P, rho,
                       -lr, momentum, local_steps, chunks, partial);
  };
  using std::integral_constant;
  using Tb = integral_constant<bool, true>;
  using Fb = integral_constant<bool, false>;
  if (vec) {
    if (mom) { if (resid_sq) go(Tb{}, Tb{}, Tb{}); else go(Tb{}, Tb{}, Fb{}); }
    else { if (resid_sq) go(Tb{}, Fb{}, Tb{}); else go(Tb{}, Fb{}, Fb{}); }
  } else {
    if (mom) { if (resid_sq) go(Fb{}, Tb{}, Tb{}); else go(Fb{}, Tb{}, Fb{}); }
    else { if (resid_sq) go(Fb{}, Fb{}, Tb{}); else go(Fb{}, Fb{}, Fb{}); }
  }
  if (resid_sq) {
    hipLaunchKernelGGL(resid_reduce_kernel, dim3(m), dim3(kThreads), 0, s, partial, chunks, resid_sq);
    hipLaunchKernelGGL(resid_reduce_kernel, dim3(m), dim3(kThreads), 0, s, partial + int64_t(m) * chunks, chunks,
                       alpha_sq);
  }
  return check_launch(nm);
}

int64_t dol_admm_ls_round_mean_workspace_bytes(int64_t P) {
  if (P <= 0 || P > dol::kMaxDim) return 0;
  return 2 * (cdiv(P, 64) + 2) * int64_t(sizeof(double));  // [2][blocks]: (w - theta)^2, alpha^2 (64-lane blocks)
}

int dol_admm_ls_round_mean_f32(float* w, int64_t ldw, float* buf, int64_t ldb, float* alpha, int64_t lda,
                               const float* target, int64_t ldt, const float* theta, const int32_t* agents,
                               const int32_t* first, int32_t m, int64_t P, float rho, float lr, float momentum,
                               int32_t local_steps, float* theta_out, float scale, double* resid_total, void* work,
                               hipStream_t s) {
  DOL_DIMS_OK("dol_admm_ls_round_mean_f32", ldw, ldb, lda, ldt, P);
  const char* nm = "dol_admm_ls_round_mean_f32";
  if (m < 1) return fail(DOL_EINVAL, "%s: m must be >= 1 (the average indexes w[0])", nm);
  if (P < 0 || local_steps < 0) return fail(DOL_EINVAL, "%s: negative size", nm);
  if (!(scale > 0.0f)) return fail(DOL_EINVAL, "%s: scale must be > 0", nm);
  const bool mom = momentum != 0.0f;
  if (P > 0 && (!w || !alpha || !target || !theta || !theta_out || (mom && !buf)))
    return fail(DOL_EINVAL, "%s: null pointer", nm);
  if (theta_out == w || theta_out == alpha || theta_out == target || (mom && theta_out == buf))
    return fail(DOL_EINVAL, "%s: theta_out aliases the rows", nm);
  if (resid_total && !work && P > 0) return fail(DOL_EINVAL, "%s: resid_total needs a workspace", nm);
  if (ldw < P || lda < P || ldt < P || (mom && ldb < P)) return fail(DOL_EINVAL, "%s: ld < P", nm);
  if (P > (int64_t(1) << 29) - 16) return fail(DOL_EINVAL, "%s: P >= 2^29 (row offsets are 32-bit buffer offsets)", nm);
  if (P == 0) {
    if (resid_total) (void)hipMemsetAsync(resid_total, 0, 2 * sizeof(double), s);
    return check_launch(nm);
  }
  const bool vec_ok = row_vec_ok(w, ldw) && row_vec_ok(alpha, lda) && row_vec_ok(target, ldt) &&
                      row_vec_ok(theta, 0) && row_vec_ok(theta_out, 0) && (!mom || row_vec_ok(buf, ldb));
  const ColSplit cs = split_cols(P, vec_ok);
  // column strip per workgroup: 1024 lanes (16 KiB of each row per workgroup,
  // one workgroup per CU at 2^20 columns) unless DOL_ADMM_ROUND_THREADS=256.
  // Narrower blocks (fewer than 1024 lanes per CU) take 256-lane strips: the
  // strips are the only parallelism (the sum over agents is sequential per
  // column).  At 8192 x 2^17 (a column-sharded rank's block at 8 ranks):
  // 18.6 ms with 1024-lane strips, 7.4 with 256, 7.65 with one-wave strips
  // and 8 agents in flight -- and 5.15 for the two-kernel round (row-major
  // client round + ordered sum), which SeparableADMM(shard="columns") takes
  // there (profiles/r06c_admm_narrow_ab.jsonl).
  static const int threads_env = env_int("DOL_ADMM_ROUND_THREADS", 0);
  static const int n_cu = [] {
    int dev = 0, cu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cu = 256;
    return cu > 0 ? cu : 256;
  }();
  const int64_t lanes = std::max<int64_t>(cs.n4, cs.tail);
  const int nt = threads_env == 256 || threads_env == 64 || threads_env == 1024 ? threads_env
                 : (lanes >= int64_t(1024) * n_cu ? 1024 : 256);
  const bool wide = nt == 1024;
  const int64_t nb4 = cdiv(cs.n4, nt), nbt = cdiv(cs.tail, nt);
  const int64_t nb = nb4 + nbt;
  double* partial = static_cast<double*>(work);
  const int do_div = scale != 1.0f;
  auto go = [&](auto vt, auto mc, auto rc, int64_t c_off, int64_t ncols, int64_t blocks, int64_t part_off) {
    using V = decltype(vt);
    constexpr bool M = decltype(mc)::value, R = decltype(rc)::value;
    auto k = wide ? admm_ls_round_mean_kernel<V, M, R, 1024>
                  : nt == 256 ? admm_ls_round_mean_kernel<V, M, R, 256> : admm_ls_round_mean_kernel<V, M, R, 64, 8>;
    hipLaunchKernelGGL(k, dim3(static_cast<unsigned>(blocks)), dim3(nt), 0, s, w, ldw, buf, ldb, alpha,
                       lda, target, ldt, theta, agents, first, m, c_off, ncols, rho, -lr, momentum, local_steps,
                       theta_out, scale, do_div, partial, part_off, nb);
  };
  using std::integral_constant;
  using Tb = integral_constant<bool, true>;
  using Fb = integral_constant<bool, false>;
  auto both = [&](auto vt, int64_t c_off, int64_t ncols, int64_t blocks, int64_t part_off) {
    if (mom) { if (resid_total) go(vt, Tb{}, Tb{}, c_off, ncols, blocks, part_off); else go(vt, Tb{}, Fb{}, c_off, ncols, blocks, part_off); }
    else { if (resid_total) go(vt, Fb{}, Tb{}, c_off, ncols, blocks, part_off); else go(vt, Fb{}, Fb{}, c_off, ncols, blocks, part_off); }
  };
  if (cs.n4 > 0) both(f4{}, 0, cs.n4, nb4, 0);
  if (cs.tail > 0) both(float{}, cs.n4 * 4, cs.tail, nbt, nb4);
  if (resid_total) hipLaunchKernelGGL(resid_reduce_kernel, dim3(2), dim3(kThreads), 0, s, partial, nb, resid_total);
  return check_launch(nm);
}

int dol_ordered_sum_f32(const float* W, int64_t ldw, const int32_t* order, int32_t m, int64_t P,
                        const float* acc_in, float* acc_out, float scale, hipStream_t s) {
  DOL_DIMS_OK("dol_ordered_sum_f32", ldw, P);
  if (m < 0 || P < 0) return fail(DOL_EINVAL, "dol_ordered_sum_f32: negative size");
  if (P == 0) { g_err[0] = '\0'; return DOL_OK; }
  if (m == 0 && !acc_in) return fail(DOL_EINVAL, "dol_ordered_sum_f32: m == 0 needs acc_in");
  if (!acc_out || (m > 0 && (!W || !order))) return fail(DOL_EINVAL, "dol_ordered_sum_f32: null pointer");
  if (m > 0 && ldw < P) return fail(DOL_EINVAL, "dol_ordered_sum_f32: ld < P");
  if (!(scale > 0.0f)) return fail(DOL_EINVAL, "dol_ordered_sum_f32: scale must be > 0");
  const bool vec_ok = row_vec_ok(W, ldw) && row_vec_ok(acc_in, 0) && row_vec_ok(acc_out, 0);
  const ColSplit cs = split_cols(P, vec_ok);
  const int do_div = scale != 1.0f;
  if (cs.n4 > 0)
    hipLaunchKernelGGL(ordered_sum_kernel<f4>, dim3(static_cast<unsigned>(cdiv(cs.n4, kThreads))), dim3(kThreads), 0,
                       s, W, ldw, order, m, int64_t(0), cs.n4, acc_in, acc_out, scale, do_div);
  if (cs.tail > 0)
    hipLaunchKernelGGL(ordered_sum_kernel<float>, dim3(static_cast<unsigned>(cdiv(cs.tail, kThreads))), dim3(kThreads), 0,
                       s, W, ldw, order, m, cs.n4 * 4, cs.tail, acc_in, acc_out, scale, do_div);
  return check_launch("dol_ordered_sum_f32");
}

int dol_ordered_mean_f32(const float* W, int64_t ldw, const int32_t* order, int32_t m, int64_t P,
                         float* theta, hipStream_t s) {
  DOL_DIMS_OK("dol_ordered_mean_f32", ldw, P);
  if (m <= 0) return fail(DOL_EINVAL, "dol_ordered_mean_f32: m must be >= 1 (reference indexes w[0])");
  if (theta == W) return fail(DOL_EINVAL, "dol_ordered_mean_f32: theta aliases W");
  return dol_ordered_sum_f32(W, ldw, order, m, P, nullptr, theta, static_cast<float>(m), s);
}

int dol_stream_copy_f32(const float* src, float* dst, int64_t n, hipStream_t s) {
  DOL_DIMS_OK("dol_stream_copy_f32", n);
  if (n < 0) return fail(DOL_EINVAL, "dol_stream_copy_f32: negative size");
  if (n == 0) { g_err[0] = '\0'; return DOL_OK; }
  if (!src || !dst) return fail(DOL_EINVAL, "dol_stream_copy_f32: null pointer");
  if (aligned16(src) && aligned16(dst)) {
    const int64_t n4 = n / 4;
    if (n4 > 0) {
      const int64_t grid = cdiv(n4, int64_t(kThreads) * 4);
      if (grid > kMaxBlocks * 8) return fail(DOL_EINVAL, "dol_stream_copy_f32: too large");
      hipLaunchKernelGGL(copy_kernel, dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, s,
                         reinterpret_cast<const f4*>(src), reinterpret_cast<f4*>(dst), n4);
    }
    if (n % 4)
      hipLaunchKernelGGL(copy_scalar_kernel, dim3(1), dim3(kThreads), 0, s, src + 4 * n4, dst + 4 * n4, n % 4);
  } else {
    hipLaunchKernelGGL(copy_scalar_kernel, dim3(2048), dim3(kThreads), 0, s, src, dst, n);
  }
  return check_launch("dol_stream_copy_f32");
}

int dol_stream_copy_rows_f32(const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t n_rows, int64_t P,
                             hipStream_t s) {
  DOL_DIMS_OK("dol_stream_copy_rows_f32", ldx, ldy, P);
  const char* nm = "dol_stream_copy_rows_f32";
  if (n_rows < 0 || P < 0) return fail(DOL_EINVAL, "%s: negative size", nm);
  if (n_rows == 0 || P == 0) { g_err[0] = '\0'; return DOL_OK; }
  if (!X || !Y) return fail(DOL_EINVAL, "%s: null pointer", nm);
  if (ldx < P || ldy < P) return fail(DOL_EINVAL, "%s: ld < P", nm);
  if (n_rows < 3 || !row_vec_ok(X, ldx) || !row_vec_ok(Y, ldy) || P % 4)
    return fail(DOL_EINVAL, "%s: needs >= 3 rows, 16-B aligned rows and P %% 4 == 0", nm);
  constexpr int R = 4;
  const int64_t n4 = P / 4, nct = cdiv(n4, kThreads);
  if (mul_sat(nct, cdiv(n_rows, R)) > kMaxBlocks) return fail(DOL_EINVAL, "%s: too large", nm);
  // the ring mix's launch with COPY: halo rows = the wrap-around neighbours, weights unused
  const float* hp = X + int64_t(n_rows - 1) * ldx;
  hipLaunchKernelGGL((ring_mix_dma_kernel<R, NoEpi, true, true>), dim3(static_cast<unsigned>(nct * cdiv(n_rows, R))),
                     dim3(kThreads), 0, s, X, ldx, Y, ldy, n_rows, n4, nct, hp, X, X, X, NoEpi{});
  return check_launch(nm);
}

}  // extern "C"
