// mlp_step.hip — one fused local step of N independent per-agent MLPs on fp32 MFMA.
//
// Each agent k owns nn.Sequential(Linear(d, h), ReLU(), Linear(h, c)) whose
// parameters are row k of the stacked bank (state_dict order: W1 [h,d], b1 [h],
// W2 [c,h], b2 [c]).  One workgroup (4 waves) runs one agent's whole step —
// the body of the reference's per-agent local_update loop (DIST/clients.py:
// 34-59: forward, CrossEntropyLoss, backward, optimizer.step(); with the
// FedProx / FedADMM gradient terms of DEC/clients.py:101-139) — in ONE pass:
//
//   F1  Z1^T = W1 X^T          v_mfma_f32_32x32x2_f32, K = d, W1 / X streamed as 64 B/lane
//       H = relu(Z1 + b1)      -> LDS  Hs[b][h]
//   F2  Z2 = H W2^T + b2       VALU (c is tiny), W2 staged in LDS
//   CE  dZ2 = (softmax(Z2) - onehot(y)) / B, loss = mean_b(lse - Z2[y])
//   B2  dW2 = dZ2^T H, db2, dZ1 = (dZ2 W2) * [H > 0], db1     VALU, LDS
//   B1  dW1 = dZ1^T X          MFMA, K = B; each 32x32 tile of dW1 is consumed
//                              in registers by the fused update of the W1 tile.
//
// Two launches: mlp_fwd_kernel (one workgroup per agent: F1 .. B2 and the
// updates of b1, W2, b2; dZ1 goes to a B x h workspace per agent) and
// mlp_dw1_kernel (one short-lived workgroup per agent x 32-column tile of W1:
// B1 + the W1 update).  W1 / momentum dominate the bytes and stream through
// the second kernel at full occupancy; a single-kernel version that walked
// each agent's 25 W1 tiles inside the per-agent workgroup ran 2.4x slower
// (one HBM round trip per tile, 2-3 waves per SIMD; tools/mlp_phase.hip).
// Phases at 1024 agents (tools/mlp_phase.hip, r02): the forward runs as two
// lock-stepped waves of 512 workgroups (two per CU by LDS), each ~90 us:
// staging + F1 56-71 us (4.6 TB/s), F2 + CE 5-6, B2 15-16, HBM idle in the
// last two.  Tried (r02): agent pieces with the forwards on a side stream and
// each piece's dW1 on the caller's stream after its forward, so dW1(q)
// overlaps forward(q + 1): local step 0.496-0.500 ms (2 pieces) / 0.510-0.518
// (4) vs 0.492-0.493 unsplit, same box (profiles/r02_mlp_split.txt): dropped.
// Also tried: F1 in 16-wide k chunks (64-B rows) with 4 / 6 stages, 40 / 60 KiB
// of LDS, so all 1024 workgroups are resident at once: 0.515 / 0.522-0.524 vs
// 0.505 ms (profiles/r02_mlp_split.txt): dropped.
// dW1 as the transposed product (operands swapped, so a lane holds 4
// consecutive W1 columns and W1 / momentum move as 16-B buffer ops, 4 + 4
// per lane and tile instead of 16 + 16): 0.577-0.579 vs 0.505 ms; each 16-B
// instruction then touches 32 W1 rows' lines instead of 2 (same profile): dropped.
// dW1 compiled for >= 5 / 6 waves per SIMD (96 / 80 VGPRs, 20 / 84 B of
// scratch) instead of 4 (104): 0.534 / 0.761 vs 0.506 ms (same profile).
//   update (every parameter, as dol_prox_admm_sgd_f32):
//       g' = g [+ (alpha +) rho*(w - theta)];  buf = mom*buf + g' (buf = g' on the
//       first step);  w = fma(-lr, buf, w)
//
// The per-agent gradients never touch HBM (unless write_grad asks for them),
// so a step moves W1 in + out, the momentum buffer in + out and X in, instead
// of the unfused path's extra gradient write + read.  GEMM numerics: fp32
// MFMA = a k-ordered f32 fma chain; the reference's torch CPU GEMMs use a
// different blocking, so this path is tolerance-checked (tests/test_mlp_gpu.py),
// not bit-exact.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <math.h>
#include <type_traits>

#include "../../include/dol_hip.h"
#include "dol_common.h"

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kMaxB = 64, kMaxH = 256, kMaxC = 32;

struct MlpArgs {
  float* W; int64_t ldw;         // parameter rows
  float* G; int64_t ldg;         // gradient rows (written when write_grad), nullable
  float* M; int64_t ldm;         // momentum rows, nullable when mode == 0
  const float* theta;            // [P] global model (FedProx / FedADMM), nullable
  const float* A; int64_t lda;   // ADMM duals, nullable
  const float* X; int64_t ldxa, ldxb;  // batch: agent stride, sample stride (floats)
  const int64_t* Y; int64_t ldya;      // labels [n][B]
  float* loss;                   // [n] mean CE per agent, nullable
  int B, d, h, c;
  float neg_lr, mom, rho;
  int mode;                      // 0 plain SGD, 1 momentum first step, 2 momentum
  int update;                    // 0: gradients only (forward_backward)
  int f1_keep;                   // F1 stages W1 / X with the default cache policy (DOL_MLP_F1_KEEP, default 1)
  int dw1_reverse;               // dW1 walks the agents last to first (DOL_MLP_DW1_REVERSE, default 1)
  // forward phase offset (DOL_MLP_FWD_STAGGER): workgroups lo, lo + step, .. < hi
  // start `stagger` x s_sleep(127) late, so co-resident workgroups run F1 and
  // the HBM-idle tail out of step
  int stagger, stagger_lo, stagger_hi, stagger_step;
#ifdef DOL_MLP_TRACE
  long long* trace;              // tools/mlp_phase.hip: per-agent phase timestamps
#endif
};

#ifdef DOL_MLP_TRACE
#define DOL_TRACE(i) \
  if (threadIdx.x == 0 && a.trace) a.trace[int64_t(blockIdx.x) * 8 + (i)] = wall_clock64();
#else
#define DOL_TRACE(i)
#endif

// Gradient term + optimizer update of N parameters (same rounding sequence as
// prox_sgd_lane in dol_hip.hip).  All loads of the batch are issued before any
// store (load() first, e.g. ahead of the MFMAs that produce the gradients, then
// commit()): the rows are plain float*, so a load-update-store per element
// would serialise one memory round trip per element.  Loads are unconditional
// from always-valid addresses (idx(i) stays in the row even for dead lanes):
// a predicated load compiles to a branch + s_waitcnt vmcnt(0) per element.
// UPD: 0 = gradients only, 1 = SGD, 2 = momentum first step, 3 = momentum.
// TH / AL: the FedProx / FedADMM terms are compiled in (theta / alpha non-null).
template <int N, int UPD, bool TH, bool AL>
struct ParamBatch {
  float w[N], m[N], th[N], al[N];

  // idx(i): row offset of element i (valid even when !ok(i)); ok(i): element i is live
  template <class Idx>
  __device__ __forceinline__ void load(const MlpArgs& a, const float* wrow, const float* mrow, const float* arow,
                                       Idx idx) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      if constexpr (UPD > 0 || TH) w[i] = wrow[idx(i)];
      if constexpr (UPD == 3) m[i] = mrow[idx(i)];
      if constexpr (TH) th[i] = a.theta[idx(i)];
      if constexpr (AL) al[i] = arow[idx(i)];
    }
  }

  // g[i]: raw loss gradient of element i
  template <class Idx, class Ok>
  __device__ __forceinline__ void commit(const MlpArgs& a, float* wrow, float* grow, float* mrow, const float (&g)[N],
                                         Idx idx, Ok ok) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      float gg = g[i];
      if constexpr (TH) {
        float t = a.rho * (w[i] - th[i]);
        if constexpr (AL) t = al[i] + t;
        gg = gg + t;
      }
      float dd = gg;
      if constexpr (UPD == 2) {
        m[i] = gg;
      } else if constexpr (UPD == 3) {
        m[i] = m[i] * a.mom + gg;
        dd = m[i];
      }
      if (!ok(i)) continue;
      if (grow) grow[idx(i)] = gg;
      if constexpr (UPD > 0) __builtin_nontemporal_store(__builtin_fmaf(a.neg_lr, dd, w[i]), wrow + idx(i));
      if constexpr (UPD >= 2) __builtin_nontemporal_store(m[i], mrow + idx(i));
    }
  }
};

#define DOL_GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define DOL_LPTR(p) ((__attribute__((address_space(3))) void*)(p))

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the immediate must be a constant)
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
#define DOL_VMC(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
#define DOL_VMC8(N) DOL_VMC(N) DOL_VMC(N + 1) DOL_VMC(N + 2) DOL_VMC(N + 3) DOL_VMC(N + 4) DOL_VMC(N + 5) DOL_VMC(N + 6) DOL_VMC(N + 7)
    DOL_VMC8(0) DOL_VMC8(8) DOL_VMC8(16) DOL_VMC8(24) DOL_VMC8(32) DOL_VMC8(40) DOL_VMC8(48) DOL_VMC8(56)
#undef DOL_VMC8
#undef DOL_VMC
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// global -> LDS copy of n floats by the workgroup, N loads in flight per thread
// (r04): a plain strided loop waits one memory round trip per iteration --
// the tail of mlp_fwd_kernel PH 2 spent ~16 of them loading H
template <int N, class Src, class Dst>
__device__ __forceinline__ void lds_fill(int n, Src src, Dst dst) {
  const int t = threadIdx.x;
  for (int o0 = 0; o0 < n; o0 += N * kThreads) {
    float v[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int o = o0 + i * kThreads + t;
      v[i] = src(o < n ? o : 0);  // unconditional, from a valid address: no branch per load
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int o = o0 + i * kThreads + t;
      if (o < n) dst(o, v[i]);
    }
  }
}

// workgroup barrier for LDS traffic only (r04): __syncthreads() also drains
// vmcnt, so every barrier after a batch of parameter stores (or with LDS-DMA
// chunks in flight) waited a full HBM round trip; no barrier in these kernels
// orders global memory between threads
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// two arrays in one round trip when each fits one batch
template <int N1, int N2, class S1, class D1, class S2, class D2>
__device__ __forceinline__ void lds_fill2(int n1, S1 src1, D1 dst1, int n2, S2 src2, D2 dst2) {
  if (n1 > N1 * kThreads || n2 > N2 * kThreads) {
    lds_fill<N1>(n1, src1, dst1);
    lds_fill<N2>(n2, src2, dst2);
    return;
  }
  const int t = threadIdx.x;
  float v1[N1], v2[N2];
#pragma unroll
  for (int i = 0; i < N1; ++i) v1[i] = src1(i * kThreads + t < n1 ? i * kThreads + t : 0);
#pragma unroll
  for (int i = 0; i < N2; ++i) v2[i] = src2(i * kThreads + t < n2 ? i * kThreads + t : 0);
#pragma unroll
  for (int i = 0; i < N1; ++i)
    if (i * kThreads + t < n1) dst1(i * kThreads + t, v1[i]);
#pragma unroll
  for (int i = 0; i < N2; ++i)
    if (i * kThreads + t < n2) dst2(i * kThreads + t, v2[i]);
}

constexpr int kStages = 3;  // default F1 LDS-DMA pipeline depth (NS - 1 chunks in flight during the MFMAs)

// LDS layout of mlp_fwd_kernel (floats): [ union: F1 staging | Hs, W2s, Zs ] [ b1s, b2s, ls ] [ ys ];
// the fused kernel (PH 3) keeps them apart: [ staging ] [ Hs, W2s, Zs ] [ ... ]
__host__ __device__ inline int64_t fwd_staging_floats(int B, int h, int ns) {
  return int64_t(ns) * (h + 32 * ((B + 31) / 32)) * 32;
}
// PH 3: W1 chunks parked in LDS instead of registers (the last KL of NK; 16 KiB each)
__host__ __device__ constexpr int fused_park_chunks(int nk, int ns) { return nk <= 8 ? 0 : ns <= 4 ? 3 : ns == 5 ? 2 : 0; }
__host__ __device__ inline int64_t fwd_union_floats(int B, int h, int c, int ns = kStages, bool fused = false,
                                                    int park = 0) {
  const int64_t staging = fwd_staging_floats(B, h, ns);
  const int64_t post = int64_t(B) * (h + 4) + int64_t(c) * (h + 4) + int64_t(B) * c;
  return fused ? staging + 4096 * int64_t(park) + post : staging > post ? staging : post;
}

// Buffer-descriptor memory ops (mlp_fused_dw1, mlp_dw1_kernel): dead lanes
// point out of range (loads return 0, stores are dropped).
using rsrc_t = __amdgpu_buffer_rsrc_t;
constexpr uint32_t kOOB = 0x80000000u;  // any lane offset >= every buffer's size

__device__ __forceinline__ rsrc_t make_rsrc(const float* p, int64_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, static_cast<int>(nbytes), 0x00020000);
}
__device__ __forceinline__ float bload(rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, static_cast<int>(voff), static_cast<int>(soff), 0));
}
__device__ __forceinline__ void bstore_nt(rsrc_t r, uint32_t voff, uint32_t soff, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, static_cast<int>(voff), static_cast<int>(soff), 2);
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// plain (write-back) 16-B stores: each one writes two 16-B pieces of 32 rows, and
// the nontemporal hint on that pattern made the B1 phase 4x slower (261 vs 66 us
// per agent, tools/mlp_phase.hip) -- the partial lines must merge in L2
__device__ __forceinline__ void bstore4(rsrc_t r, uint32_t voff, f4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, static_cast<int>(voff), 0, 0);
}

// B1 + the W1 update of the fused step (mlp_fwd_kernel PH 3), on the W1 that
// F1 left in registers.  Per 32-column chunk dt: the dW1^T tile [32 d x 32 h] =
// X^T dZ1 on MFMA (K = B), with the tile's d rows permuted -- A row i holds
// column sigma(i) = 16 ((i >> 2) & 1) + 4 (i >> 3) + (i & 3) -- so accumulator
// r = 4 j + q of lane (li, hh) is the gradient of W1[32 wave + li][32 dt + 16 hh +
// 4 j + q] = wres[dt][j][q]: exactly where F1 left that weight.  The products
// and their k order are those of mlp_dw1_kernel with A and B swapped (two
// chains, even / odd k-steps): bit-identical.  Momentum and X chunks stream
// through the F1 staging ring (LDS-DMA, NS deep; the first NS - 1 were issued
// before F2 and landed during F2 .. B2).  W1 / momentum / gradient tiles go out
// as 16-B buffer stores that are always issued (masked lanes point out of
// range, absent buffers have size 0), so the per-chunk vmcnt below can count
// them: vector memory ops retire in issue order on gfx9, loads and stores alike.
template <int UPD, int NS, int NK, int KL, class Issue>
__device__ __forceinline__ void mlp_fused_dw1(const MlpArgs& a, const f4 (&wres)[NK - KL][4], const float* park, const float* Hs,
                                              const float* stg, int rows, float* wrow, float* grow, float* mrow,
                                              Issue& issue, int i0, int ipw) {
  const int B = a.B, d = a.d, h = a.h;
  const int hp = h + 4;
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));  // fresh lane-derived addresses: no CSE with F1's, held live across it
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 31, hh = lane >> 5;
  const int64_t P = int64_t(h) * d + h + int64_t(a.c) * h + a.c;
  const rsrc_t rW = make_rsrc(wrow, P * 4);
  const rsrc_t rM = make_rsrc(UPD >= 2 ? mrow : wrow, UPD >= 2 ? P * 4 : 0);
  const rsrc_t rG = make_rsrc(grow ? grow : wrow, grow ? P * 4 : 0);
  float bz[16];  // B operand: dZ1[b = 2 s + hh][32 wave + li]
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int b = 2 * s + hh;
    const float v = Hs[min(b, B - 1) * hp + 32 * wave + li];  // unconditional read, then select (no branch)
    bz[s] = b < B ? v : 0.f;
  }
  const int sg = 16 * ((li >> 2) & 1) + 4 * (li >> 3) + (li & 3);  // sigma(li)
  const int xp = sg >> 2, xe = sg & 3;                               // its 16-B piece, element
  const int ipw_b1 = ipw - i0;                                       // DMA instructions per wave per chunk
  constexpr int kSt = 12;                                            // 16-B stores per lane per tile
  const uint32_t rowoff = uint32_t(((32 * wave + li) * d + 16 * hh) * 4);
#pragma unroll
  for (int dt = 0; dt < NK; ++dt) {
    // ops issued after chunk dt's DMA: the next chunks' DMAs and the last tiles' stores
    const int later = min(NS - 2, NK - 1 - dt) * ipw_b1 + min(dt, NS - 1) * kSt;
    wait_vmcnt(min(later, 63));
    __builtin_amdgcn_s_barrier();  // chunk dt landed for every wave; stage (dt - 1) % NS is free
    if (dt + NS - 1 < NK) issue(dt + NS - 1, mrow, i0);
    const float* st = stg + (dt % NS) * rows * 32;
    float xv[16];  // A operand: X[b = 2 s + hh][32 dt + sigma(li)]
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int b = 2 * s + hh;  // < 32: always inside the staged X rows
      const float v = st[(h + b) * 32 + ((xp ^ (b & 7)) * 4) + xe];
      xv[s] = b < B ? v : 0.f;
    }
    f32x16 acc, acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = acc1[r] = 0.f;
#pragma unroll
    for (int s = 0; s < 16; s += 2) {
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xv[s], bz[s], acc, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(xv[s + 1], bz[s + 1], acc1, 0, 0, 0);
    }
    acc += acc1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f4 mv = {0.f, 0.f, 0.f, 0.f};
      if constexpr (UPD == 3) mv = *reinterpret_cast<const f4*>(st + (32 * wave + li) * 32 + ((4 * hh + j) ^ (li & 7)) * 4);
      const f4 w0 = dt < NK - KL ? wres[dt < NK - KL ? dt : 0][j]
                                 : *reinterpret_cast<const f4*>(park + ((dt - (NK - KL)) * 16 + wave * 4 + j) * 256 + lane * 4);
      f4 g, w, m;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float gg = acc[4 * j + q];
        float dd = gg, mr = 0.f;
        if constexpr (UPD == 2) {
          mr = gg;
        } else if constexpr (UPD == 3) {
          mr = mv[q] * a.mom + gg;
          dd = mr;
        }
        g[q] = gg;
        m[q] = mr;
        w[q] = __builtin_fmaf(a.neg_lr, dd, w0[q]);
      }
      const uint32_t vo = 32 * dt + 16 * hh + 4 * j < d ? rowoff + uint32_t((32 * dt + 4 * j) * 4) : kOOB;
      bstore4(rG, vo, g);
      bstore4(rW, vo, w);
      bstore4(rM, vo, m);
    }
  }
}

// Per-agent part: forward, CE, backward down to dZ1 (-> ws[agent][b][h]),
// updates of b1, W2, b2.
// F1 streams W1 and X through LDS with global_load_lds (LDS-DMA): each
// 32-wide k chunk of the h + Bp rows lands as 128-B rows whose 16-B pieces are
// XOR-swizzled by row (piece p of row r at slot p ^ (r & 7)), three stages
// deep; a row-contiguous load touches 8 lines per instruction where reading
// the MFMA fragments straight from HBM touched 64 (2.3 TB/s effective).
// NT = accumulator tiles per wave: 1 when h * ceil(B/32) <= 128, else 4.
// PH (r03): 0 = the whole per-agent part in one kernel; 1 = F1 only, H (after
// bias + relu) to ws[agent][b][h] (LDS = the F1 staging alone); 2 = the rest
// (F2, CE, B2, dZ1 -> ws) from that H.  1 + 2 run the same operations in the
// same order as 0 (bit-identical); the split lets F1 stream W1 without the
// HBM-idle tail and with deeper staging.
// PH 3 (r03): the whole step in one kernel for h = 128, B <= 32 and NK = d / 32
// chunks known at compile time -- F1 keeps every W1 fragment it reads (NK x 16
// floats per lane: the agent's 128 x d W1 lives in the CU's register file), so
// B1 + the W1 update run on the resident W1 and W1 is read from HBM once, not
// twice; see mlp_fused_dw1 above.  Bit-identical to 0 + mlp_dw1_kernel
// (tests/test_mlp_gpu.py::test_step_paths_bit_identical), opt-in
// (DOL_MLP_FUSED=1): see the measurement at the dispatch below.
template <int NT, int UPD, bool TH, bool AL, int NS = kStages, int PH = 0, int NK = 0>
__device__ __forceinline__ void mlp_fwd_body(MlpArgs a, float* __restrict__ ws) {
  static_assert(PH != 3 || (NT == 1 && NK > 0 && !TH && !AL && UPD >= 1), "fused step: plain / momentum SGD, one tile per wave");
  if (a.stagger > 0) {
    const int bx = int(blockIdx.x);
    if (bx >= a.stagger_lo && bx < a.stagger_hi && (bx - a.stagger_lo) % a.stagger_step == 0)
      for (int i = 0; i < a.stagger; ++i) __builtin_amdgcn_s_sleep(127);
  }
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int B = a.B, d = a.d, h = a.h, c = a.c;
  const int hp = h + 4;  // padded LDS rows: 16-B aligned, rows 4 banks apart
  constexpr int KL = PH == 3 ? fused_park_chunks(NK, NS) : 0;
  float* park = lds + fwd_staging_floats(B, h, NS);  // PH 3: [KL][4 waves][4 j][64 lanes] f4
  float* Hs = lds + (PH == 3 ? fwd_staging_floats(B, h, NS) + 4096 * KL : 0);  // [B][hp]  H, later dZ1   (after F1)
  float* W2s = Hs + B * hp;          // [c][hp]                 (after F1)
  float* Zs = W2s + c * hp;          // [B][c]   Z2, later dZ2
  float* b1s = lds + fwd_union_floats(B, h, c, NS, PH == 3, KL);  // [h]
  float* b2s = b1s + h;              // [c]
  float* ls = b2s + c;               // [B] per-sample loss
  int* ys = reinterpret_cast<int*>(ls + B);  // [B]

  const int agent = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int li = lane & 31, hh = lane >> 5;
  float* wrow = a.W + int64_t(agent) * a.ldw;
  float* grow = a.G ? a.G + int64_t(agent) * a.ldg : nullptr;
  float* mrow = a.M ? a.M + int64_t(agent) * a.ldm : nullptr;
  const float* arow = a.A ? a.A + int64_t(agent) * a.lda : nullptr;
  const float* xa = a.X + int64_t(agent) * a.ldxa;
  const int64_t oW1 = 0, ob1 = int64_t(h) * d, oW2 = ob1 + h, ob2 = oW2 + int64_t(c) * h;

  DOL_TRACE(0)
  // update operands of W2 (first 8 * 256 entries), b1 and b2 go out now, so
  // their round trips overlap F1 instead of serialising the B2 phase
  auto ok_w2 = [&](int i) { return i * kThreads + t < c * h; };
  auto idx_w2 = [&](int i) { return oW2 + (ok_w2(i) ? i * kThreads + t : 0); };
  auto ok_b1 = [&](int) { return t < h; };
  auto idx_b1 = [&](int) { return ob1 + (t < h ? t : 0); };
  auto ok_b2 = [&](int) { return t < c; };
  auto idx_b2 = [&](int) { return ob2 + (t < c ? t : 0); };
  ParamBatch<8, UPD, TH, AL> pw2;
  ParamBatch<1, UPD, TH, AL> pb1, pb2;
  auto load_small = [&] {
    pw2.load(a, wrow, mrow, arow, idx_w2);
    pb1.load(a, wrow, mrow, arow, idx_b1);
    pb2.load(a, wrow, mrow, arow, idx_b2);
  };
  if constexpr (PH != 1) {
    if constexpr (PH != 3) load_small();  // PH 3: after F1 (the registers hold W1 during F1)
    if (t < c) b2s[t] = wrow[ob2 + t];
    if (t < B) ys[t] = static_cast<int>(a.Y[int64_t(agent) * a.ldya + t]);
  }
  if constexpr (PH == 0 || PH == 3)
    for (int i = t; i < h; i += kThreads) b1s[i] = wrow[ob1 + i];
  if constexpr (PH != 1) lds_barrier();  // PH 1: the staging is the whole LDS (b1 read from memory below)
  float* wsa = ws + int64_t(agent) * B * h;  // H (PH 1 -> 2), then dZ1 for mlp_dw1_kernel
  // pw2 holds W2 itself when the update (or the prox term) loaded it and it fits one batch
  const bool w2_in_regs = (UPD > 0 || TH) && c * h <= 8 * kThreads;
  // ---- F1: Z1^T tiles (32 h x 32 b) on MFMA, K = d in chunks of 32
  const int nht = h / 32, nbt = (B + 31) / 32;
  const int Bp = 32 * nbt, rows = PH == 3 ? 160 : h + Bp;  // staged rows per chunk (W1 rows, then X rows)
  const int ipw = rows / 32;               // DMA instructions per wave per chunk (8 rows each)
  const int nk = NK > 0 ? NK : (d + 31) / 32;
  float* stg = lds;
  // PH 3 stages through buffer descriptors: one 32-bit lane offset per staged
  // row serves W1 and momentum alike (chunk kc in the SGPR offset), and the
  // k >= d pieces of a tail chunk read as zeros (out-of-range lanes): few VGPRs
  // beside the resident W1, no zeroing pass.
  const int64_t P1 = int64_t(h) * d + h + int64_t(c) * h + c;
  const rsrc_t rsW = make_rsrc(wrow, P1 * 4);
  const rsrc_t rsM = make_rsrc(UPD == 3 && PH == 3 ? mrow : wrow, P1 * 4);
  const rsrc_t rsX = make_rsrc(xa, (int64_t(B - 1) * a.ldxb + d) * 4);
  uint32_t voff3[5];  // PH 3: per staged row group i (4 x W1 / momentum, 1 x X)
  if constexpr (PH == 3) {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int r = 8 * (wave + kWaves * i) + (lane >> 3);
      const int ch = (lane & 7) ^ (lane >> 3);
      voff3[i] = i < 4 ? uint32_t((r * d + 4 * ch) * 4) : uint32_t((min(r - h, B - 1) * a.ldxb + 4 * ch) * 4);
    }
  }
  // stage chunk kc of rows [i0 * 32, rows) (W1 / momentum rows from `top`, then X)
  auto issue = [&](int kc, const float* top, int i0) {
    float* st = stg + (kc % NS) * rows * 32;
    if constexpr (PH == 3) {
      const bool tail = kc == nk - 1 && (d & 31);  // (compile-time false before the last chunk)
      const bool pok = 32 * kc + 4 * ((lane & 7) ^ (lane >> 3)) < d;
#pragma unroll
      for (int i = i0; i < 5; ++i) {
        const uint32_t vo = !tail || pok ? voff3[i] : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 4 ? (top == wrow ? rsW : rsM) : rsX,
                                                 DOL_LPTR(st + (wave + kWaves * i) * 256), 16, static_cast<int>(vo),
                                                 kc * 128, 0, 0);
      }
      return;
    }
    for (int i = i0; i < ipw; ++i) {
      const int ins = wave + kWaves * i;
      const int r = 8 * ins + (lane >> 3);
      const int ch = (lane & 7) ^ (lane >> 3);
      int k = kc * 32 + 4 * ch;
      k = k < d ? k : 0;  // clamped in-bounds; zeroed after landing
      const float* src = (r < h) ? top + oW1 + int64_t(r) * d + k
                                 : xa + int64_t(min(r - h, B - 1)) * a.ldxb + k;
      // default policy with dW1 reversed (r06, see dol_mlp_step_f32); nontemporal with
      // dW1 in agent order (r05: 0.489-0.491 vs 0.496-0.499 ms, profiles/r05zzf_mlp_load_policy_ab.jsonl)
      if (a.f1_keep)
        __builtin_amdgcn_global_load_lds(DOL_GPTR(src), DOL_LPTR(st + ins * 256), 16, 0, 0);
      else
        __builtin_amdgcn_global_load_lds(DOL_GPTR(src), DOL_LPTR(st + ins * 256), 16, 0, 2);
    }
  };
  // PH 3: W1[32 wave + li][32 kc + 16 hh + 4 j + q] = wres[kc][j][q] (the last KL chunks: park)
  f4 wres[PH == 3 ? NK - KL : 1][4];
  const int i0_b1 = UPD == 3 ? 0 : PH == 3 ? 4 : h / 32;  // PH 3's B1 chunks: momentum rows (UPD 3) + X rows, or X rows only
  if constexpr (PH == 2) {  // H from the F1 kernel
    if (w2_in_regs)
      lds_fill<16>(B * h, [&](int o) { return wsa[o]; }, [&](int o, float v) { Hs[(o / h) * hp + (o % h)] = v; });
    else
      lds_fill2<16, 8>(B * h, [&](int o) { return wsa[o]; }, [&](int o, float v) { Hs[(o / h) * hp + (o % h)] = v; },
                       c * h, [&](int o) { return wrow[oW2 + o]; }, [&](int o, float v) { W2s[(o / h) * hp + o % h] = v; });
  } else {

  f32x16 acc[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
  for (int s0 = 0; s0 < NS - 1 && s0 < nk; ++s0) issue(s0, wrow, 0);
  auto f1_chunk = [&](int kc) __attribute__((always_inline)) {
    wait_vmcnt(min(NS - 2, nk - 1 - kc) * ipw);  // chunk kc landed (the next NS - 2 may still fly)
    __builtin_amdgcn_s_barrier();                 // ... for every wave; and stage (kc + NS - 1) % NS is free
    const float* st = stg + (kc % NS) * rows * 32;
    if (PH != 3 && kc == nk - 1 && (d & 31)) {  // zero the clamped k >= d pieces of the tail chunk
      for (int i = 0; i < ipw; ++i) {
        const int ins = wave + kWaves * i;
        if (kc * 32 + 4 * ((lane & 7) ^ (lane >> 3)) >= d)
          *reinterpret_cast<f4*>(const_cast<float*>(st) + ins * 256 + lane * 4) = f4{0.f, 0.f, 0.f, 0.f};
      }
      lds_barrier();
    }
    if (kc + NS - 1 < nk) issue(kc + NS - 1, wrow, 0);
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int tile = wave + kWaves * u;
      if (tile < nht * nbt) {
        const int ht = tile % nht, bt = tile / nht;
        const float* ar = st + (32 * ht + li) * 32;
        const float* xr = st + (h + 32 * bt + li) * 32;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int pos = ((4 * hh + j) ^ (li & 7)) * 4;
          const f4 av = *reinterpret_cast<const f4*>(ar + pos);
          const f4 xv = *reinterpret_cast<const f4*>(xr + pos);
          if constexpr (PH == 3) {
            if (kc < NK - KL) wres[kc < NK - KL ? kc : 0][j] = av;
            else *reinterpret_cast<f4*>(park + ((kc - (NK - KL)) * 16 + wave * 4 + j) * 256 + lane * 4) = av;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], xv[q], acc[u], 0, 0, 0);
        }
      }
    }
  };
  if constexpr (PH == 3) {
#pragma unroll
    for (int kc = 0; kc < NK; ++kc) f1_chunk(kc);
  } else {
    for (int kc = 0; kc < nk; ++kc) f1_chunk(kc);
  }
  lds_barrier();  // staging is dead: Hs / W2s / Zs reuse it (PH 3: the momentum / X chunks of B1 start landing)
  // PH 3: B1's first NS - 1 chunks (momentum rows when UPD == 3, then X) fly during F2 .. B2
  if constexpr (PH == 3) {
    load_small();
    for (int s0 = 0; s0 < NS - 1 && s0 < NK; ++s0) issue(s0, mrow, i0_b1);
  }
  // C/D map: col (b) = lane & 31, row (h) = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int u = 0; u < NT; ++u) {
    const int tile = wave + kWaves * u;
    if (tile < nht * nbt) {
      const int ht = tile % nht, bt = tile / nht;
      const int brow = 32 * bt + li;
      if (brow < B) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int hr = 32 * ht + (r & 3) + 8 * (r >> 2) + 4 * hh;
          const float z = acc[u][r] + (PH == 1 ? wrow[ob1 + hr] : b1s[hr]);
          const float hz = (z > 0.0f || z != z) ? z : 0.0f;  // relu, NaN propagates like torch
          if constexpr (PH == 1) wsa[brow * h + hr] = hz;
          else Hs[brow * hp + hr] = hz;
        }
      }
    }
  }
  if constexpr (PH == 1) return;
  }  // PH != 2
  if (w2_in_regs) {  // W2 from the update operands loaded at the start: no memory round trip here
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (ok_w2(i)) W2s[((i * kThreads + t) / h) * hp + (i * kThreads + t) % h] = pw2.w[i];
  } else if constexpr (PH != 2) {  // (PH 2 filled W2s together with H)
    lds_fill<8>(c * h, [&](int o) { return wrow[oW2 + o]; }, [&](int o, float v) { W2s[(o / h) * hp + o % h] = v; });
  }
  lds_barrier();

  DOL_TRACE(1)
  // ---- F2: Z2 = H W2^T + b2
  for (int o = t; o < B * c; o += kThreads) {
    const int b = o / c, j = o % c;
    float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;  // h % 32 == 0
#pragma unroll 8
    for (int k = 0; k < h; k += 4) {
      const f4 hv = *reinterpret_cast<const f4*>(Hs + b * hp + k);
      const f4 wv = *reinterpret_cast<const f4*>(W2s + j * hp + k);
      s0 = s0 + hv.x * wv.x;
      s1 = s1 + hv.y * wv.y;
      s2 = s2 + hv.z * wv.z;
      s3 = s3 + hv.w * wv.w;
    }
    Zs[o] = ((s0 + s1) + (s2 + s3)) + b2s[j];
  }
  lds_barrier();

  // ---- CE: log-softmax per sample, dZ2 = (p - onehot) / B
  if (t < B) {
    float* z = Zs + t * c;
    float m = z[0];
    for (int j = 1; j < c; ++j) m = fmaxf(m, z[j]);
    float s = 0.0f;
    for (int j = 0; j < c; ++j) s = s + expf(z[j] - m);
    const float lse = m + logf(s);
    const int y = ys[t];
    const bool yok = y >= 0 && y < c;
    ls[t] = yok ? lse - z[yok ? y : 0] : __builtin_nanf("");
    const float invB = 1.0f / static_cast<float>(B);
    for (int j = 0; j < c; ++j) z[j] = (expf(z[j] - lse) - (j == y ? 1.0f : 0.0f)) * invB;
  }
  lds_barrier();
  if (t == 0 && a.loss) {
    float s = 0.0f;
#pragma unroll 8
    for (int b = 0; b < B; ++b) s = s + ls[b];
    a.loss[agent] = s / static_cast<float>(B);
  }

  DOL_TRACE(2)
  // ---- B2a: dW2 = dZ2^T H, db2 = sum_b dZ2 (and their parameter updates; the
  // forward already used W2 / b2 from LDS)
  for (int o0 = 0; o0 < c * h; o0 += 8 * kThreads) {
    ParamBatch<8, UPD, TH, AL> pb;
    float g[8];
    auto ok = [&](int i) { return o0 + i * kThreads + t < c * h; };
    auto idx = [&](int i) { return oW2 + (ok(i) ? o0 + i * kThreads + t : 0); };
    if (o0 > 0) pb.load(a, wrow, mrow, arow, idx);
    if (kThreads % h == 0) {  // k = t % h for all 8 outputs: one H read per sample serves them all (r04)
      const int k = t % h;
      int jj[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        jj[i] = ok(i) ? (o0 + i * kThreads + t) / h : 0;
        g[i] = 0.0f;
      }
#pragma unroll 4
      for (int b = 0; b < B; ++b) {  // per output the same products, summed over b ascending
        const float hv = Hs[b * hp + k];
        const float* zr = Zs + b * c;
#pragma unroll
        for (int i = 0; i < 8; ++i) g[i] = g[i] + zr[jj[i]] * hv;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int o = ok(i) ? o0 + i * kThreads + t : 0;
        const int j = o / h, k = o % h;
        float s = 0.0f;
        for (int b = 0; b < B; ++b) s = s + Zs[b * c + j] * Hs[b * hp + k];
        g[i] = s;
      }
    }
    if (o0 == 0) pw2.commit(a, wrow, grow, mrow, g, idx, ok);
    else pb.commit(a, wrow, grow, mrow, g, idx, ok);
  }
  DOL_TRACE(5)
  if (t < 64) {  // db2 (c <= 32 lanes of wave 0)
    float g[1];
    const int j = t < c ? t : 0;
    float s = 0.0f;
#pragma unroll 8
    for (int b = 0; b < B; ++b) s = s + Zs[b * c + j];
    g[0] = s;
    pb2.commit(a, wrow, grow, mrow, g, idx_b2, ok_b2);
  }
  lds_barrier();
  DOL_TRACE(6)

  // ---- B2b: dZ1 = (dZ2 W2) * [H > 0], in place over H
  if (kThreads % h == 0 && B * h <= 16 * kThreads) {
    // k = t % h for every output of this thread: one W2 read per class serves
    // up to 16 samples (r04; per output the same products, j ascending)
    const int k = t % h, b0 = t / h, bs = kThreads / h;
    float sm[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) sm[m] = 0.0f;
    for (int j = 0; j < c; ++j) {
      const float w2 = W2s[j * hp + k];
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int b = b0 + m * bs;
        // unconditional read (b clamped; rows b >= B are never stored): a branch per
        // sample serialised the 16 reads, one LDS round trip each (8.5 us per agent)
        sm[m] = sm[m] + Zs[min(b, B - 1) * c + j] * w2;
      }
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int b = b0 + m * bs;
      if (b < B) {
        float* hv = Hs + b * hp + k;
        *hv = (*hv > 0.0f) ? sm[m] : 0.0f;
      }
    }
  } else {
#pragma unroll 4
    for (int o = t; o < B * h; o += kThreads) {
      const int b = o / h, k = o % h;
      float s = 0.0f;
      for (int j = 0; j < c; ++j) s = s + Zs[b * c + j] * W2s[j * hp + k];
      float* hv = Hs + b * hp + k;
      *hv = (*hv > 0.0f) ? s : 0.0f;
    }
  }
  lds_barrier();
  DOL_TRACE(7)

  // ---- db1 (h <= kThreads)
  {
    float g[1];
    float s = 0.0f;
    if (t < h)
#pragma unroll 8
      for (int b = 0; b < B; ++b) s = s + Hs[b * hp + t];
    g[0] = s;
    pb1.commit(a, wrow, grow, mrow, g, idx_b1, ok_b1);
  }

  if constexpr (PH == 3) {
    DOL_TRACE(3)
    lds_barrier();  // dZ1 complete in Hs
    mlp_fused_dw1<UPD, NS, NK, KL>(a, wres, park, Hs, stg, rows, wrow, grow, mrow, issue, i0_b1, ipw);
    DOL_TRACE(4)
    return;
  }
  // dZ1 for the W1 tiles of mlp_dw1_kernel
  for (int o = t; o < B * h; o += kThreads) wsa[o] = Hs[(o / h) * hp + (o % h)];
  DOL_TRACE(3)
}

template <int NT, int UPD, bool TH, bool AL, int NS = kStages, int PH = 0, int NK = 0>
__global__ __launch_bounds__(kThreads) void mlp_fwd_kernel(MlpArgs a, float* __restrict__ ws) {
  mlp_fwd_body<NT, UPD, TH, AL, NS, PH, NK>(a, ws);
}

// the per-agent tail (PH 2) compiled for four waves per SIMD (<= 128 VGPRs,
// r04): at the default three (151 VGPRs) 1024 agents ran as two rounds of
// 768 + 256 workgroups (tools/mlp_phase.hip 't')
template <int NT, int UPD, bool TH, bool AL>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void mlp_tail_kernel(
    MlpArgs a, float* __restrict__ ws) {
  mlp_fwd_body<NT, UPD, TH, AL, 1, 2, 0>(a, ws);
}

// F1 as one single-wave workgroup per (agent, 32-row h-tile), B <= 32 (r04):
// H[:, 32 ht .. 32 ht + 32) = relu(W1[32 ht ..] X^T + b1) -> ws[agent][b][h],
// then mlp_fwd_kernel PH 2 runs the per-agent tail from ws.  The per-agent F1
// (4 waves, 61 KiB of staging, 2 workgroups per CU) streamed at 4.6 TB/s and
// sat in lock step with the HBM-idle tail; here each wave owns its own
// NS-deep LDS-DMA ring (W1 rows 0..31, X rows 32..63 of each 32-wide k chunk,
// 16-B pieces swizzled by row as in mlp_fwd_kernel), no barriers, 8 KiB per
// stage, so 4 - 5 independent rings share a CU.  X is fetched once per h-tile:
// the nht tiles of an agent run on one XCD (blockIdx % 8 = agent % 8, tiles
// consecutive), so the repeats meet in its L2.  Tail chunk pieces with k >= d
// are out-of-range buffer lanes: they land as zeros, as mlp_fwd_kernel zeroes
// them.  The MFMA sequence of a tile is the per-agent kernel's (same k order,
// same operands): bit-identical H.
// KW (k chunk width): 32 = 128-B row pieces, 8 rows per DMA instruction; 64 =
// 256-B pieces, 4 rows per instruction, each 64-wide chunk consumed as two
// 32-wide halves in k order (a half wholly past d is skipped, as the 32-wide
// kernel never stages it): the same MFMA sequence either way.
template <int NS, int KW = 32>
__global__ __launch_bounds__(64) void mlp_f1_tile_kernel(MlpArgs a, float* __restrict__ ws, int n_agents) {
  static_assert(KW == 32 || KW == 64, "k chunk: 32 or 64 floats");
  constexpr int PPR = KW / 4;     // 16-B pieces per staged row (slot = piece ^ (row % PPR))
  constexpr int RPI = 64 / PPR;   // staged rows per DMA instruction
  constexpr int NI = 64 / RPI;    // DMA instructions per stage (64 staged rows)
  __shared__ __attribute__((aligned(16))) float stg[NS * 64 * KW];
  const int B = a.B, d = a.d, h = a.h;
  const int nht = h / 32;
  const uint32_t bx = blockIdx.x, l = bx >> 3;
  const int ht = static_cast<int>(l % uint32_t(nht));
  const int agent = static_cast<int>((l / uint32_t(nht)) * 8 + (bx & 7));
  if (agent >= n_agents) return;
  const int lane = threadIdx.x;
  const int li = lane & 31, hh = lane >> 5;
  const float* wrow = a.W + int64_t(agent) * a.ldw;
  const int64_t P1 = int64_t(h) * d + h + int64_t(a.c) * h + a.c;
  const rsrc_t rsW = make_rsrc(wrow, P1 * 4);
  const rsrc_t rsX = make_rsrc(a.X + int64_t(agent) * a.ldxa, (int64_t(B - 1) * a.ldxb + d) * 4);
  const int nk = (d + KW - 1) / KW;
  // staged row r = RPI i + lane / PPR: W1 row 32 ht + r (r < 32), X row min(r - 32, B - 1) (r >= 32);
  // lane's LDS slot lane % PPR holds piece slot ^ (r % PPR)
  uint32_t voff[NI];
  int pc[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int r = RPI * i + lane / PPR;
    pc[i] = (lane % PPR) ^ (r % PPR);
    voff[i] = r < 32 ? uint32_t(((32 * ht + r) * d + 4 * pc[i]) * 4) : uint32_t((min(r - 32, B - 1) * a.ldxb + 4 * pc[i]) * 4);
  }
  auto issue = [&](int kc) {
    float* st = stg + (kc % NS) * 64 * KW;
#pragma unroll
    for (int i = 0; i < NI; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(RPI * i < 32 ? rsW : rsX, DOL_LPTR(st + i * 256), 16,
                                               static_cast<int>(KW * kc + 4 * pc[i] < d ? voff[i] : kOOB), kc * KW * 4,
                                               0, 0);
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int s0 = 0; s0 < NS - 1 && s0 < nk; ++s0) issue(s0);
  for (int kc = 0; kc < nk; ++kc) {
    wait_vmcnt(min(NS - 2, nk - 1 - kc) * NI);             // chunk kc landed (the next NS - 2 may still fly)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    // last chunk's LDS reads done: its stage is free
    if (kc + NS - 1 < nk) issue(kc + NS - 1);
    const float* st = stg + (kc % NS) * 64 * KW;
    const float* ar = st + li * KW;
    const float* xr = st + (32 + li) * KW;
#pragma unroll
    for (int h2 = 0; h2 < KW / 32; ++h2) {
      if (h2 > 0 && KW * kc + 32 * h2 >= d) break;  // a half wholly past d (wave-uniform)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int pos = ((8 * h2 + 4 * hh + j) ^ (li % PPR)) * 4;
        const f4 av = *reinterpret_cast<const f4*>(ar + pos);
        const f4 xv = *reinterpret_cast<const f4*>(xr + pos);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], xv[q], acc, 0, 0, 0);
      }
    }
  }
  // C/D map: col (b) = lane & 31, row (h) = (r&3) + 8*(r>>2) + 4*(lane>>5); bias + relu as mlp_fwd_kernel PH 1
  if (li < B) {
    float* wsa = ws + int64_t(agent) * B * h;
    const int64_t ob1 = int64_t(h) * d;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int hr = 32 * ht + (r & 3) + 8 * (r >> 2) + 4 * hh;
      const float z = acc[r] + wrow[ob1 + hr];
      wsa[li * h + hr] = (z > 0.0f || z != z) ? z : 0.0f;
    }
  }
}

// B1 + W1 update: block agent * ndt + dt owns columns [32 dt, 32 dt + 32) of W1
// for all h rows; wave w takes h-tiles w, w + 4, ...  A = dZ1^T from the
// workspace (L2), B = X[:, cols].  Memory goes through wave-uniform buffer
// descriptors: one 32-bit lane offset per tile, the row step of each of the
// 16 accumulator rows in the SGPR soffset, dead lanes pointed out of range
// (loads return 0, stores are dropped), and every load of the tile issued
// before the MFMA chain (sched_barrier) so the W1 / momentum reads overlap it.
// KS = MFMA k-steps (2 samples each): 16 for B <= 32, 32 for B <= 64.
// (buffer helpers: above mlp_fused_dw1)

// XG (r04): XCD-grouped tile order.  With d = 784 a W1 row is 24.5 lines, so
// the 128-B column piece of every odd row straddles two lines that the
// neighbouring tile (dt +- 1) shares; the dispatcher deals consecutive blocks
// to different XCDs, so with blockIdx = agent * ndt + dt both XCDs fetched
// (and partially wrote back) those lines.  XG = 1 keeps every tile of an
// agent on ONE XCD (blockIdx % 8 = agent % 8, tiles in order), so the shared
// lines meet in that XCD's L2.  Same arithmetic per tile: same bits.
template <int KS, int UPD, bool TH, bool AL, int CH = 1, int XG = 0>
__device__ __forceinline__ void mlp_dw1_body(MlpArgs a, const float* __restrict__ ws, int n_agents) {
  const int B = a.B, d = a.d, h = a.h, c = a.c;
  const int ndt = (d + 31) / 32;
  int dt, agent;
  if constexpr (XG) {
    const uint32_t b = blockIdx.x, l = b >> 3;
    dt = static_cast<int>(l % uint32_t(ndt));
    uint32_t lg = l / uint32_t(ndt);
    if (a.dw1_reverse) lg = uint32_t((n_agents + 7) / 8) - 1 - lg;  // last agents first, each on its forward's XCD
    agent = static_cast<int>(lg * 8 + (b & 7));
    if (agent >= n_agents) return;
  } else {
    dt = static_cast<int>(blockIdx.x % ndt);
    agent = static_cast<int>(blockIdx.x / ndt);
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 31, hh = lane >> 5;
  const int64_t P = int64_t(h) * d + h + int64_t(c) * h + c;
  const rsrc_t rW = make_rsrc(a.W + int64_t(agent) * a.ldw, P * 4);
  const rsrc_t rM = make_rsrc(UPD == 3 || UPD == 2 ? a.M + int64_t(agent) * a.ldm : a.W, P * 4);
  const rsrc_t rG = make_rsrc(a.G ? a.G + int64_t(agent) * a.ldg : a.W, a.G ? P * 4 : 0);
  const rsrc_t rT = make_rsrc(TH ? a.theta : a.W, TH ? P * 4 : 0);
  const rsrc_t rA = make_rsrc(AL ? a.A + int64_t(agent) * a.lda : a.W, AL ? P * 4 : 0);
  const rsrc_t rX = make_rsrc(a.X + int64_t(agent) * a.ldxa, (int64_t(B - 1) * a.ldxb + d) * 4);
  const rsrc_t rZ = make_rsrc(ws + int64_t(agent) * B * h, int64_t(B) * h * 4);
  const int col = 32 * dt + li;
  const bool cok = col < d;
  float xv[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int b = 2 * s + hh;
    xv[s] = bload(rX, (b < B && cok) ? uint32_t((b * a.ldxb + col) * 4) : kOOB, 0);
  }
  for (int ht = wave; ht < h / 32; ht += kWaves) {
    float av[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int b = 2 * s + hh;
      av[s] = bload(rZ, b < B ? uint32_t((b * h + 32 * ht + li) * 4) : kOOB, 0);
    }
    const uint32_t pv = cok ? uint32_t(((32 * ht + 4 * hh) * d + col) * 4) : kOOB;
    auto so = [&](int r) { return uint32_t(((r & 3) + 8 * (r >> 2)) * d * 4); };
    float w[16], m[16], th[16], al[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if constexpr (UPD > 0 || TH) w[r] = bload(rW, pv, so(r));
      if constexpr (UPD == 3) m[r] = bload(rM, pv, so(r));
      if constexpr (TH) th[r] = bload(rT, pv, so(r));
      if constexpr (AL) al[r] = bload(rA, pv, so(r));
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    if constexpr (CH == 2) {  // two independent k-chains (even / odd k-steps), summed at the end
      f32x16 acc1 = acc;
#pragma unroll
      for (int s = 0; s < KS; s += 2) {
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], xv[s], acc, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s + 1], xv[s + 1], acc1, 0, 0, 0);
      }
      acc += acc1;
    } else {
#pragma unroll
      for (int s = 0; s < KS; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], xv[s], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float gg = acc[r];
      if constexpr (TH) {
        float t = a.rho * (w[r] - th[r]);
        if constexpr (AL) t = al[r] + t;
        gg = gg + t;
      }
      float dd = gg;
      if constexpr (UPD == 2) {
        m[r] = gg;
      } else if constexpr (UPD == 3) {
        m[r] = m[r] * a.mom + gg;
        dd = m[r];
      }
      if (a.G) bstore_nt(rG, pv, so(r), gg);
      if constexpr (UPD > 0) bstore_nt(rW, pv, so(r), __builtin_fmaf(a.neg_lr, dd, w[r]));
      if constexpr (UPD >= 2) bstore_nt(rM, pv, so(r), m[r]);
    }
  }
}

template <int KS, int UPD, bool TH, bool AL, int CH = 1, int XG = 0>
__global__ __launch_bounds__(kThreads) void mlp_dw1_kernel(MlpArgs a, const float* __restrict__ ws, int n_agents) {
  mlp_dw1_body<KS, UPD, TH, AL, CH, XG>(a, ws, n_agents);
}

// dW1 compiled for four waves per SIMD (<= 128 VGPRs + AGPRs; DOL_MLP_DW1_OCC=4):
// the two-chain kernel needs 98 + 32 and runs three
template <int KS, int UPD, bool TH, bool AL, int CH, int XG>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void mlp_dw1_occ4_kernel(
    MlpArgs a, const float* __restrict__ ws, int n_agents) {
  mlp_dw1_body<KS, UPD, TH, AL, CH, XG>(a, ws, n_agents);
}

}  // namespace

extern "C" int64_t dol_mlp_step_workspace_bytes(int32_t n_agents, int32_t B, int32_t h) {
  if (n_agents <= 0 || B <= 0 || h <= 0 || B > kMaxB || h > kMaxH) return 0;  // outside the step's limits
  return int64_t(n_agents) * B * h * int64_t(sizeof(float));
}

extern "C" int64_t dol_mlp_step_lds_bytes(int32_t B, int32_t h, int32_t c) {
  if (B <= 0 || h <= 0 || c <= 0 || B > kMaxB || h > kMaxH || c > kMaxC) return 0;  // outside the step's limits
  return sizeof(float) * (fwd_union_floats(B, h, c) + h + c + B) + sizeof(int) * int64_t(B);
}

extern "C" int dol_mlp_step_f32(float* w, int64_t ldw, float* grad, int64_t ldg, float* mom, int64_t ldm,
                                const float* theta, const float* alpha, int64_t lda, const float* X,
                                int64_t ldx_agent, int64_t ldx_row, const int64_t* labels, int64_t ldy_agent,
                                float* loss, int32_t n_agents, int32_t B, int32_t d, int32_t h, int32_t c,
                                float lr, float momentum, float rho, int first_step, int update,
                                void* work, hipStream_t s) {
  DOL_DIMS_OK("dol_mlp_step_f32", ldw, ldg, ldm, lda, ldx_agent, ldx_row, ldy_agent);
  using dol::fail;
  if (n_agents < 0) return fail(DOL_EINVAL, "dol_mlp_step_f32: negative agent count");
  if (n_agents == 0) { dol::g_err[0] = '\0'; return DOL_OK; }
  if (B < 1 || B > kMaxB) return fail(DOL_EINVAL, "dol_mlp_step_f32: batch %d outside [1, %d]", B, kMaxB);
  if (h < 32 || h > kMaxH || h % 32) return fail(DOL_EINVAL, "dol_mlp_step_f32: hidden %d must be a multiple of 32 in [32, %d]", h, kMaxH);
  if (c < 1 || c > kMaxC) return fail(DOL_EINVAL, "dol_mlp_step_f32: classes %d outside [1, %d]", c, kMaxC);
  if (d < 4 || d % 4) return fail(DOL_EINVAL, "dol_mlp_step_f32: input dim %d must be a positive multiple of 4", d);
  if (!w || !X || !labels || !work) return fail(DOL_EINVAL, "dol_mlp_step_f32: null w / X / labels / work");
  const int64_t P = int64_t(h) * d + h + int64_t(c) * h + c;
  if (ldw < P || (grad && ldg < P) || (mom && ldm < P) || (alpha && lda < P))
    return fail(DOL_EINVAL, "dol_mlp_step_f32: ld < P (%lld)", (long long)P);
  if (ldx_row < d || ldx_agent < int64_t(B - 1) * ldx_row + d || ldy_agent < B)
    return fail(DOL_EINVAL, "dol_mlp_step_f32: X / labels strides too small");
  if ((reinterpret_cast<uintptr_t>(w) & 15) || ldw % 4 || (reinterpret_cast<uintptr_t>(X) & 15) || ldx_row % 4 ||
      ldx_agent % 4)
    return fail(DOL_EINVAL, "dol_mlp_step_f32: w and X rows must be 16-byte aligned");
  if (alpha && !theta) return fail(DOL_EINVAL, "dol_mlp_step_f32: alpha without theta");
  const int mode = (momentum == 0.0f) ? 0 : (first_step ? 1 : 2);
  if (update && mode != 0 && !mom) return fail(DOL_EINVAL, "dol_mlp_step_f32: momentum needs the mom buffer");
  if (!update && !grad) return fail(DOL_EINVAL, "dol_mlp_step_f32: update=0 needs a grad buffer to write");
  MlpArgs a{w, ldw, grad, ldg, mom, ldm, theta, alpha, lda, X, ldx_agent, ldx_row, labels, ldy_agent, loss,
            B, d, h, c, -lr, momentum, rho, update ? mode : 0, update ? 1 : 0};
  // r06: the forward walks the agents first to last and, with dW1 walking them
  // last to first, every launch starts on the rows the launch before it wrote
  // last -- still in L2 / the Infinity Cache when F1 stages them with the
  // default policy (the r05 nontemporal staging gave that up).  Config-5 round
  // (fused step + exact mix, 1024 agents): 1.378 vs 1.400 ms, the local step
  // 0.457-0.462 vs 0.477-0.479 ms, three alternating trials; the step alone
  // 0.475-0.480 vs 0.490-0.494 (profiles/r06m_mlp_order.jsonl).  Same bits.
  static const int f1_keep = [] { const char* e = getenv("DOL_MLP_F1_KEEP"); return e ? atoi(e) : 1; }();
  static const int dw1_rev = [] { const char* e = getenv("DOL_MLP_DW1_REVERSE"); return e ? atoi(e) : 1; }();
  a.f1_keep = f1_keep;
  a.dw1_reverse = dw1_rev;
  // r06: the forward's second workgroup slot of every CU (blocks [n_cu, 2 n_cu))
  // starts ~20 us late, so the two workgroups of a CU run F1 (HBM) and the
  // HBM-idle tail out of step for the rest of the launch: local step 0.4686-
  // 0.4696 vs 0.4743-0.4836 ms, three alternating trials, same bits
  // (tools/mlp_stagger_ab.py, profiles/r06u_mlp_stagger_ab.jsonl); only with
  // >= 4 n_cu agents (two full rounds of workgroups).  DOL_MLP_FWD_STAGGER =
  // "count,mode" overrides (read per call; "0" = off; mode 2 = the odd blocks of
  // [0, 2 n_cu), measured slower)
  {
    static const int n_cu = [] {
      int dev = 0, cu = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cu = 0;
      return cu;
    }();
    const char* e = getenv("DOL_MLP_FWD_STAGGER");  // read per call (A/B in one process)
    int cnt = (n_cu > 0 && n_agents >= 4 * n_cu) ? 6 : 0, mode = 1;
    if (e && sscanf(e, "%d,%d", &cnt, &mode) < 1) cnt = 0;
    if (cnt > 0 && n_cu > 0) {
      a.stagger = cnt;
      a.stagger_lo = mode == 2 ? 1 : n_cu;
      a.stagger_hi = 2 * n_cu;
      a.stagger_step = mode == 2 ? 2 : 1;
    }
  }
  const size_t lds = static_cast<size_t>(dol_mlp_step_lds_bytes(B, h, c));
  if (lds > 160 * 1024) return fail(DOL_EINVAL, "dol_mlp_step_f32: %zu B of LDS per agent exceeds 160 KiB", lds);
  const dim3 grid(static_cast<unsigned>(n_agents)), block(kThreads);
  // F1 pipeline depth (DOL_MLP_STAGES = 2 / 3 / 4; diagnostics, default 3)
  static const int stages = [] { const char* e = getenv("DOL_MLP_STAGES"); return e ? atoi(e) : kStages; }();
  // forward as two kernels (F1 / the per-agent tail; bit-identical), opt-in with
  // DOL_MLP_SPLIT_FWD=1: measured 0.518-0.524 (F1 depth 3 / 4) and 0.509-0.511
  // (depth 2) vs 0.509-0.513 ms fused (profiles/r03_mlp_split_fwd.txt)
  static const int split_fwd = [] { const char* e = getenv("DOL_MLP_SPLIT_FWD"); return e ? atoi(e) : 0; }();
  // F1 as single-wave (agent, h-tile) workgroups with NS-deep rings (mlp_f1_tile_kernel;
  // DOL_MLP_F1_TILES = NS in {3, 4, 5, 6, 8}, 0 = off), B <= 32
  static const int f1_tile_ns = [] { const char* e = getenv("DOL_MLP_F1_TILES"); return e ? atoi(e) : 0; }();
  // its k chunk width (DOL_MLP_F1_KW = 32 / 64; 64 takes NS 3 or 4) and the
  // tail's occupancy (DOL_MLP_TAIL_OCC = 4: mlp_tail_kernel, <= 128 VGPRs)
  static const int f1_kw = [] { const char* e = getenv("DOL_MLP_F1_KW"); return e ? atoi(e) : 32; }();
  static const int tail_occ4 = [] { const char* e = getenv("DOL_MLP_TAIL_OCC"); return e ? atoi(e) == 4 : 0; }();
  const int upd = update ? mode + 1 : 0;
  float* ws = static_cast<float*>(work);
  // dW1 tile order (DOL_MLP_DW1_XCD: 1 = an agent's tiles on one XCD, 0 = agent-major)
  static const int dw1_xcd = [] { const char* e = getenv("DOL_MLP_DW1_XCD"); return e ? atoi(e) : 1; }();
  const int64_t n_blk2 = int64_t((d + 31) / 32) * (dw1_xcd ? (int64_t(n_agents) + 7) / 8 * 8 : n_agents);
  if (n_blk2 > (int64_t(1) << 31) - 1) return fail(DOL_EINVAL, "dol_mlp_step_f32: too many W1 tiles for one launch");
  const dim3 grid2(static_cast<unsigned>(n_blk2));
  // dW1's k-chain as two interleaved accumulators summed at the end (VERDICT r02
  // item 4): local step 0.5036-0.5046 vs 0.5074-0.5079 ms with one chain, three
  // alternating pairs on one box (profiles/r03_mlp_dw1_chains.txt) -- the step
  // is not chain-latency bound; DOL_MLP_DW1_CHAINS=1 restores one chain
  static const int dw1_chains = [] { const char* e = getenv("DOL_MLP_DW1_CHAINS"); return e ? atoi(e) : 2; }();
  static const int dw1_occ4 = [] { const char* e = getenv("DOL_MLP_DW1_OCC"); return e ? atoi(e) == 4 : 0; }();
  // diagnostics: unused dynamic LDS per dW1 workgroup, to cap its occupancy (DOL_MLP_DW1_LDS bytes, <= 64 KiB)
  static const size_t dw1_lds = [] {
    const char* e = getenv("DOL_MLP_DW1_LDS");
    const long v = e ? atol(e) : 0;
    return static_cast<size_t>(v < 0 ? 0 : v > 65536 ? 65536 : v);
  }();
  // the one-kernel step with W1 resident in registers (mlp_fwd_kernel PH 3;
  // DOL_MLP_FUSED=1).  It reads W1 once (1.75 instead of 2.16 GB per step at 1024
  // agents) but its 400 resident floats per lane leave one workgroup per CU:
  // per agent F1 27-42 us (latency-bound at 4 chunks in flight), F2 + CE 6 and
  // B2 20 (HBM nearly idle) and B1 66-74 us, 0.588 ms in all vs 0.56 for the two
  // kernels in the same tool (tools/mlp_phase.hip, profiles/r03_mlp_fused.txt):
  // kept opt-in.
  static const int fused = [] { const char* e = getenv("DOL_MLP_FUSED"); return e ? atoi(e) : 0; }();
  const bool a16 = !(reinterpret_cast<uintptr_t>(mom) & 15) && ldm % 4 == 0 && !(reinterpret_cast<uintptr_t>(grad) & 15) &&
                   ldg % 4 == 0;
  const int nkc = (d + 31) / 32;
  const bool fusable = fused && h == 128 && B <= 32 && a16 && (nkc == 25 || nkc == 4);
  auto go = [&](auto ks, auto upd_c, auto th, auto al) {
    constexpr int KS = decltype(ks)::value, U = decltype(upd_c)::value;
    constexpr bool TH = decltype(th)::value, AL = decltype(al)::value;
    auto fwd = [&](auto kern, size_t lds_ns) {
      if (lds_ns > 65536)  // above the default dynamic-LDS cap (gfx950 has 160 KiB per CU)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(lds_ns));
      hipLaunchKernelGGL(kern, grid, block, lds_ns, s, a, ws);
    };
    auto lds_for = [&](int ns) {
      return sizeof(float) * (fwd_union_floats(B, h, c, ns) + h + c + B) + sizeof(int) * size_t(B);
    };
    const bool nt1 = h * ((B + 31) / 32) <= 128;
    if constexpr (!TH && !AL && U >= 1 && KS == 16) {
      if (fusable) {
        auto fz = [&](auto nk_c, auto ns_c) {
          constexpr int NK = decltype(nk_c)::value, NS = decltype(ns_c)::value;
          fwd(mlp_fwd_kernel<1, U, false, false, NS, 3, NK>,
              sizeof(float) * (fwd_union_floats(B, h, c, NS, true, fused_park_chunks(NK, NS)) + h + c + B) +
                  sizeof(int) * size_t(B));
        };
        if (nkc == 25) fz(std::integral_constant<int, 25>{}, std::integral_constant<int, 5>{});
        else fz(std::integral_constant<int, 4>{}, std::integral_constant<int, 5>{});
        return;
      }
    }
    // the per-agent tail (PH 2) needs no F1 staging: LDS = its post-F1 arrays alone
    auto tail = [&] {
      if (tail_occ4) {
        if (nt1) fwd(mlp_tail_kernel<1, U, TH, AL>, lds_for(1));
        else fwd(mlp_tail_kernel<4, U, TH, AL>, lds_for(1));
      } else if (nt1) {
        fwd(mlp_fwd_kernel<1, U, TH, AL, 1, 2>, lds_for(1));
      } else {
        fwd(mlp_fwd_kernel<4, U, TH, AL, 1, 2>, lds_for(1));
      }
    };
    if (f1_tile_ns && B <= 32 && P * 4 < (int64_t(1) << 31)) {  // F1 per (agent, h-tile), then the tail
      const dim3 gt(static_cast<unsigned>(int64_t(h / 32) * ((int64_t(n_agents) + 7) / 8 * 8))), bt(64);
      if (f1_kw == 64) {
        if (f1_tile_ns == 4) hipLaunchKernelGGL((mlp_f1_tile_kernel<4, 64>), gt, bt, 0, s, a, ws, n_agents);
        else hipLaunchKernelGGL((mlp_f1_tile_kernel<3, 64>), gt, bt, 0, s, a, ws, n_agents);
      } else if (f1_tile_ns == 3) hipLaunchKernelGGL(mlp_f1_tile_kernel<3>, gt, bt, 0, s, a, ws, n_agents);
      else if (f1_tile_ns == 4) hipLaunchKernelGGL(mlp_f1_tile_kernel<4>, gt, bt, 0, s, a, ws, n_agents);
      else if (f1_tile_ns == 6) hipLaunchKernelGGL(mlp_f1_tile_kernel<6>, gt, bt, 0, s, a, ws, n_agents);
      else if (f1_tile_ns == 8) hipLaunchKernelGGL(mlp_f1_tile_kernel<8>, gt, bt, 0, s, a, ws, n_agents);
      else hipLaunchKernelGGL(mlp_f1_tile_kernel<5>, gt, bt, 0, s, a, ws, n_agents);
      tail();
    } else if (split_fwd) {  // F1 kernel (staging only in LDS), then the per-agent tail kernel
      auto f1 = [&](auto ns_c) {
        constexpr int NS = decltype(ns_c)::value;
        const size_t l1 = sizeof(float) * size_t(NS) * (h + 32 * ((B + 31) / 32)) * 32;
        if (nt1) fwd(mlp_fwd_kernel<1, U, TH, AL, NS, 1>, l1);
        else fwd(mlp_fwd_kernel<4, U, TH, AL, NS, 1>, l1);
      };
      if (stages == 2) f1(std::integral_constant<int, 2>{});
      else if (stages == 4) f1(std::integral_constant<int, 4>{});
      else if (stages == 5) f1(std::integral_constant<int, 5>{});
      else f1(std::integral_constant<int, 3>{});
      tail();
    } else if (stages == 2) {
      if (nt1) fwd(mlp_fwd_kernel<1, U, TH, AL, 2>, lds_for(2));
      else fwd(mlp_fwd_kernel<4, U, TH, AL, 2>, lds_for(2));
    } else if (stages == 4 && lds_for(4) <= 160 * 1024) {
      if (nt1) fwd(mlp_fwd_kernel<1, U, TH, AL, 4>, lds_for(4));
      else fwd(mlp_fwd_kernel<4, U, TH, AL, 4>, lds_for(4));
    } else {
      if (nt1) fwd(mlp_fwd_kernel<1, U, TH, AL>, lds);
      else fwd(mlp_fwd_kernel<4, U, TH, AL>, lds);
    }
    if (dw1_xcd && dw1_occ4 && dw1_chains == 1)
      hipLaunchKernelGGL((mlp_dw1_occ4_kernel<KS, U, TH, AL, 1, 1>), grid2, block, 0, s, a, ws, n_agents);
    else if (dw1_xcd && dw1_occ4)
      hipLaunchKernelGGL((mlp_dw1_occ4_kernel<KS, U, TH, AL, 2, 1>), grid2, block, 0, s, a, ws, n_agents);
    else if (dw1_xcd && dw1_chains == 1)
      hipLaunchKernelGGL((mlp_dw1_kernel<KS, U, TH, AL, 1, 1>), grid2, block, 0, s, a, ws, n_agents);
    else if (dw1_xcd)
      hipLaunchKernelGGL((mlp_dw1_kernel<KS, U, TH, AL, 2, 1>), grid2, block, dw1_lds, s, a, ws, n_agents);
    else if (dw1_chains == 2)
      hipLaunchKernelGGL((mlp_dw1_kernel<KS, U, TH, AL, 2>), grid2, block, 0, s, a, ws, n_agents);
    else
      hipLaunchKernelGGL((mlp_dw1_kernel<KS, U, TH, AL>), grid2, block, 0, s, a, ws, n_agents);
  };
  auto by_upd = [&](auto ks, auto th, auto al) {
    using std::integral_constant;
    switch (upd) {
      case 0: go(ks, integral_constant<int, 0>{}, th, al); break;
      case 1: go(ks, integral_constant<int, 1>{}, th, al); break;
      case 2: go(ks, integral_constant<int, 2>{}, th, al); break;
      default: go(ks, integral_constant<int, 3>{}, th, al); break;
    }
  };
  using K16 = std::integral_constant<int, 16>;
  using K32 = std::integral_constant<int, 32>;
  using T = std::true_type;
  using F = std::false_type;
  if (B <= 32) {
    if (!theta) by_upd(K16{}, F{}, F{});
    else if (!alpha) by_upd(K16{}, T{}, F{});
    else by_upd(K16{}, T{}, T{});
  } else {
    if (!theta) by_upd(K32{}, F{}, F{});
    else if (!alpha) by_upd(K32{}, T{}, F{});
    else by_upd(K32{}, T{}, T{});
  }
  return dol::check_launch("dol_mlp_step_f32");
}
