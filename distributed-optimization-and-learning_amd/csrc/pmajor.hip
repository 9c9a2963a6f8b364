// pmajor.hip — the sparse gossip mix on the PARAMETER-MAJOR ("transposed")
// bank layout, and the layout conversion.  Part of libdol_hip.so.
//
// Layout.  The agent-major bank (row k = agent k's P parameters, dol_hip.hip)
// is what the notebooks' nn.Module views need.  For synthetic many-agent
// workloads whose local steps are per coordinate (BASELINE config 3: 1024-8192
// agents x 2^20 on a random-regular W) the engine can hold the bank
// transposed instead: XT[p][j] = agent j's parameter p, p-row stride ldx >= N.
// One p-row is then the whole mixing problem for one coordinate,
// Y[:, p] = W X[:, p], and it is CONTIGUOUS (N floats: 4 KiB at 1024 agents,
// 32 KiB at 8192): every byte of X and Y streams once, sequentially, whatever
// the graph — where the agent-major CSR kernel re-reads each row deg times
// through L2 (47-53 % of HBM on random-regular W).
//
// csr_pm_kernel: one persistent 1024-thread workgroup per CU walks 32 KiB
// stages (sr consecutive p-rows, each padded to xw floats in LDS); stages come
// in by LDS-DMA (global_load_lds_dwordx4) into a ring of NBUF buffers with
// NBUF - 1 stages in flight, retired by a counted s_waitcnt vmcnt and a raw
// s_barrier (no __syncthreads(): its fence would drain the ring).  Each thread
// owns QPT "quads" (4 consecutive output agents) for the whole kernel, with
// their first four (column, weight) pairs in registers (columns as u16), so the
// CSR index is read once per kernel, not once per tile; the gathers are LDS
// reads.  Sums: +0 start, ascending CSR order, separately rounded mul and add
// (-ffp-contract=off), entries past a row's degree skipped by a select (no
// 0 * Inf) — bit-identical to dol_mix_csr_f32 and the reference's consensus
// (DIST/clients.py:61-69).  Stores are buffer stores with dropped
// out-of-range lanes, so every thread issues the same number of VMEM ops per
// stage and the counted wait is exact.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <type_traits>

#include "../../include/dol_hip.h"
#include "dol_common.h"

#define DOL_GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define DOL_LPTR(p) ((__attribute__((address_space(3))) void*)(p))

namespace {
using dol::check_launch;
using dol::fail;

typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
using rsrc_t = __amdgpu_buffer_rsrc_t;

constexpr int kMaxAgents = 8192;          // one p-row image fits a 32 KiB stage
constexpr int kT1 = 1024;                 // threads per workgroup (16 waves, one workgroup per CU)
constexpr uint32_t kOOB = 0x80000000u;    // a buffer offset past every range: the store is dropped

__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
#define DOL_VMC(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
#define DOL_VMC8(N) DOL_VMC(N) DOL_VMC(N + 1) DOL_VMC(N + 2) DOL_VMC(N + 3) DOL_VMC(N + 4) DOL_VMC(N + 5) DOL_VMC(N + 6) DOL_VMC(N + 7)
    DOL_VMC(1) DOL_VMC(2) DOL_VMC(3) DOL_VMC(4) DOL_VMC(5) DOL_VMC(6) DOL_VMC(7)
    DOL_VMC8(8) DOL_VMC8(16) DOL_VMC8(24) DOL_VMC8(32) DOL_VMC8(40) DOL_VMC8(48) DOL_VMC8(56)
#undef DOL_VMC8
#undef DOL_VMC
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

__device__ __forceinline__ rsrc_t make_rsrc(const float* p, uint32_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, static_cast<int>(nbytes), 0x00020000);
}

// one output quad: agents 4q .. 4q+3, their first four neighbours (u16 columns,
// two per register), weights and degrees (4 bits each, min(degree, 15))
struct Quad {
  uint32_t c[4][2];
  float w[4][4];
  uint32_t deg;
};

__device__ __forceinline__ void load_quad(Quad& Q, int q, int n_rows, int nnz, const int32_t* __restrict__ rowptr,
                                          const int32_t* __restrict__ col, const float* __restrict__ val) {
  // unconditional loads from clamped addresses, all issued before any use (a
  // predicated load compiles to a branch + vmcnt(0) per element)
  int e0[4], d[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int i = min(4 * q + a, n_rows - 1);
    e0[a] = rowptr[i];
    d[a] = rowptr[i + 1];
  }
  int cj[4][4];
  float wj[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    d[a] = 4 * q + a < n_rows ? d[a] - e0[a] : 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ee = min(e0[a] + e, nnz - 1);
      cj[a][e] = col[ee];
      wj[a][e] = val[ee];
    }
  }
  Q.deg = 0;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    Q.deg |= uint32_t(d[a] < 15 ? d[a] : 15) << (4 * a);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool in = e < d[a];
      const uint32_t c = in ? static_cast<uint32_t>(cj[a][e]) : 0u;
      if (e % 2 == 0) Q.c[a][e / 2] = c;
      else Q.c[a][e / 2] |= c << 16;
      Q.w[a][e] = in ? wj[a][e] : 0.0f;
    }
  }
}

// y[a] = sum_e w[a][e] * im[col[a][e]]  (+0 start, ascending e)
__device__ __forceinline__ f4 mix_quad(const Quad& Q, const float* __restrict__ im, int q,
                                       const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                       const float* __restrict__ val) {
  f4 y;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int d = static_cast<int>((Q.deg >> (4 * a)) & 15u);
    float acc = 0.0f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t cj = (Q.c[a][e / 2] >> (16 * (e % 2))) & 0xffffu;
      const float t = Q.w[a][e] * im[cj];
      acc = e < d ? acc + t : acc;
    }
    if (d > 4) {  // a long row: the rest of its list from memory (rare; correct, not fast)
      const int i = 4 * q + a;
      const int e1 = rowptr[i + 1];
      for (int e = rowptr[i] + 4; e < e1; ++e) acc = acc + val[e] * im[col[e]];
    }
    y[a] = acc;
  }
  return y;
}

// Config-3 epilogue on the parameter-major bank (the DGD round of
// dol_dgd_csr_f32, transposed): after the mix, `steps` local momentum-SGD
// iterations on the separable loss, per coordinate (OBJ 0 least squares
// g = x - t, 1 logistic g = -t / (1 + exp(t x)); MODE 0 plain SGD, 1 first
// momentum step, 2 momentum), x = fma(-lr, d, x) — the arithmetic of DgdEpi /
// oracle_dgd_local_f32.  The target (and momentum) p-rows of a stage come in
// by the same LDS-DMA as X, behind the X image.
struct PmDgd {
  const float* T; int64_t ldt;
  float* M; int64_t ldm;
  float neg_lr, mom;
  int steps;
};

template <int OBJ, int MODE>
__device__ __forceinline__ float dgd_local(float x, float t, float& b, const PmDgd& e) {
  for (int s = 0; s < e.steps; ++s) {
    float g;
    if constexpr (OBJ == 0) g = x - t;
    else g = -t / (1.0f + expf(t * x));
    float d = g;
    if constexpr (MODE != 0) {
      if (MODE == 1 && s == 0) b = g;
      else b = b * e.mom + g;
      d = b;
    }
    x = __builtin_fmaf(e.neg_lr, d, x);
  }
  return x;
}

// Mix one stage image (sr p-rows of xw floats at im0, p-rows p0 ..) and store
// its rows of YT (and, OBJ >= 0, run the local steps first: target / momentum
// images of nw floats per p-row follow the X image): spt (x2 with a momentum
// store) buffer stores per thread, out-of-range ones dropped.
template <int T, int QPT, int SAUX, bool COPY, int OBJ = -1, int MODE = 0>
__device__ __forceinline__ void mix_stage(const Quad (&Q)[QPT], const float* __restrict__ im0, float* __restrict__ YT,
                                          int64_t ldy, int n_rows, int64_t P, int64_t p0, int xw, int sr, int spt,
                                          int q0, int g, int GR, const int32_t* __restrict__ rowptr,
                                          const int32_t* __restrict__ col, const float* __restrict__ val,
                                          const PmDgd& e, int nw) {
  const int nq = (n_rows + 3) / 4;
  const int xq = xw / 4;
  const int64_t rows_here = std::min<int64_t>(sr, P - p0);
  const rsrc_t ry = make_rsrc(YT + p0 * ldy, static_cast<uint32_t>(rows_here * ldy * 4));
  rsrc_t rm = ry;
  if constexpr (OBJ >= 0 && MODE != 0) rm = make_rsrc(e.M + p0 * e.ldm, static_cast<uint32_t>(rows_here * e.ldm * 4));
  const float* tim0 = im0 + sr * xw;      // target images
  const float* mim0 = tim0 + sr * nw;     // momentum images (MODE 2)
  for (int u = 0; u < spt / QPT; ++u) {
    const int pr = g + u * GR;
    const bool prow_ok = pr < rows_here;
    const int prc = pr < sr ? pr : 0;
    const float* im = im0 + prc * xw;
#pragma unroll
    for (int j = 0; j < QPT; ++j) {
      const int q = q0 + j * T;
      f4 y = COPY ? *reinterpret_cast<const f4*>(im + 4 * (q % xq)) : mix_quad(Q[j], im, q, rowptr, col, val);
      f4 bv = f4{0.f, 0.f, 0.f, 0.f};
      if constexpr (OBJ >= 0) {
        const int qc = q < nq ? q : 0;
        const f4 tv = *reinterpret_cast<const f4*>(tim0 + prc * nw + 4 * qc);
        if constexpr (MODE == 2) bv = *reinterpret_cast<const f4*>(mim0 + prc * nw + 4 * qc);
        float b0 = bv.x, b1 = bv.y, b2 = bv.z, b3 = bv.w;
        y = f4{dgd_local<OBJ, MODE>(y.x, tv.x, b0, e), dgd_local<OBJ, MODE>(y.y, tv.y, b1, e),
               dgd_local<OBJ, MODE>(y.z, tv.z, b2, e), dgd_local<OBJ, MODE>(y.w, tv.w, b3, e)};
        bv = f4{b0, b1, b2, b3};
      }
      const uint32_t off = static_cast<uint32_t>((pr * ldy + 4 * q) * 4);
      const uint32_t offm = static_cast<uint32_t>((pr * (OBJ >= 0 && MODE != 0 ? e.ldm : 0) + 4 * q) * 4);
      constexpr bool kMom = OBJ >= 0 && MODE != 0;
      if (4 * q + 3 < n_rows || q >= nq) {  // whole quad, or none (dropped)
        const bool ok = prow_ok && q < nq;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, y), ry, ok ? off : kOOB, 0, SAUX);
        if constexpr (kMom)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, bv), rm, ok ? offm : kOOB, 0, SAUX);
      } else {  // the ragged last quad (elements named one by one: hipcc 7.2 stored
                // element 0 four times from a loop over y[a] here)
        const float ye[4] = {y.x, y.y, y.z, y.w};
        const int left = n_rows - 4 * q;  // 1..3
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ye[0]), ry, prow_ok ? off : kOOB, 0, SAUX);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ye[1]), ry, prow_ok && left > 1 ? off + 4 : kOOB, 0,
                                              SAUX);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ye[2]), ry, prow_ok && left > 2 ? off + 8 : kOOB, 0,
                                              SAUX);
        if constexpr (kMom) {
          const float be[4] = {bv.x, bv.y, bv.z, bv.w};
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(be[0]), rm, prow_ok ? offm : kOOB, 0, SAUX);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(be[1]), rm, prow_ok && left > 1 ? offm + 4 : kOOB, 0,
                                                SAUX);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(be[2]), rm, prow_ok && left > 2 ? offm + 8 : kOOB, 0,
                                                SAUX);
        }
      }
    }
  }
}

// T threads per workgroup, SF floats per stage buffer, NBUF buffers, QPT
// quads per thread.  LAUX / SAUX: cache-policy bits of the LDS-DMA loads / the
// stores (0 default, 2 nontemporal); COPY: y = x of the same agent (a copy in
// the same geometry: the structure's own ceiling, measurement only).
// OBJ >= 0: the config-3 epilogue (PmDgd), its target (+ momentum) p-rows
// staged behind X's in every stage (nw floats each).
template <int T, int SF, int NBUF, int QPT, int LAUX, int SAUX, bool COPY = false, int OBJ = -1, int MODE = 0>
__global__ __launch_bounds__(T) void csr_pm_kernel(const float* __restrict__ XT, int64_t ldx, int x_rows,
                                                   float* __restrict__ YT, int64_t ldy, int n_rows, int64_t P,
                                                   int xw, int sr, int qp_log2, int spt, int64_t n_stages, int nseg,
                                                   const int32_t* __restrict__ rowptr,
                                                   const int32_t* __restrict__ col,
                                                   const float* __restrict__ val, PmDgd e, int nw, int wait_all_stores) {
  constexpr int kDma = SF / 4 / T;  // LDS-DMA instructions per thread per stage
  static_assert(kDma * 4 * T == SF, "a stage is a whole number of DMA rounds");
  extern __shared__ __attribute__((aligned(16))) float img[];  // NBUF x SF
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // thread -> (quad, p-row group): QPT == 1: QP = 2^qp_log2 quads per p-row,
  // GR = T / QP p-rows side by side; QPT > 1: quads tid + j*T of one p-row
  const int q0 = QPT == 1 ? (tid & ((1 << qp_log2) - 1)) : tid;
  const int g = QPT == 1 ? (tid >> qp_log2) : 0;
  const int GR = QPT == 1 ? (T >> qp_log2) : 1;
  const int nnz = rowptr[n_rows];
  Quad Q[QPT];
  if (nnz > 0) {
#pragma unroll
    for (int j = 0; j < QPT; ++j) load_quad(Q[j], q0 + j * T, n_rows, nnz, rowptr, col, val);
  } else {
#pragma unroll
    for (int j = 0; j < QPT; ++j) Q[j] = Quad{};
  }

  // stage order: the P range is cut into nseg contiguous segments; workgroup b
  // walks segment b % nseg with stride gridDim / nseg, so the chip streams
  // nseg separate regions at once (nseg = 8: +4-5 % over one sweep)
  const int64_t W = gridDim.x / nseg, seg = blockIdx.x % nseg, wl = blockIdx.x / nseg;
  const int64_t seg_len = (n_stages + nseg - 1) / nseg;
  const int64_t seg_n = std::max<int64_t>(0, std::min<int64_t>(seg_len, n_stages - seg * seg_len));
  const int64_t nk = wl < seg_n ? (seg_n - wl + W - 1) / W : 0;
  auto stage_of = [&](int64_t k) { return seg * seg_len + wl + k * W; };
  const int xq = xw / 4;             // 16-B pieces per p-row image
  const int xr4 = (x_rows + 3) / 4;  // pieces holding data
  const int nq4 = nw / 4, nr4 = (n_rows + 3) / 4;
  const int nX = sr * xq, nTM = sr * nq4;  // pieces of the X images, of one epilogue operand's images
  auto issue = [&](int64_t k) {      // stage k of this workgroup -> buffer k % NBUF
    const int64_t p0 = stage_of(k) * sr;
    float* dst = img + (k % NBUF) * SF;
#pragma unroll
    for (int d = 0; d < kDma; ++d) {
      const int pc = d * T + tid;
      const float* src = XT;  // dead pieces re-read XT[0..3]
      if (pc < nX) {
        const int pr = pc / xq, j4 = pc - pr * xq;
        if (p0 + pr < P && j4 < xr4) src = XT + (p0 + pr) * ldx + 4 * j4;
      } else if (OBJ >= 0) {
        const int pt = pc - nX, op = pt / nTM, r = pt - op * nTM;  // op 0: target, 1: momentum
        const int pr = r / nq4, j4 = r - pr * nq4;
        if ((op == 0 || (MODE == 2 && op == 1)) && p0 + pr < P && j4 < nr4)
          src = op == 0 ? e.T + (p0 + pr) * e.ldt + 4 * j4 : e.M + (p0 + pr) * e.ldm + 4 * j4;
      }
      __builtin_amdgcn_global_load_lds(DOL_GPTR(src), DOL_LPTR(dst + (d * T + wave * 64) * 4), 16, 0, LAUX);
    }
  };
  constexpr int kStores = (OBJ >= 0 && MODE != 0) ? 2 : 1;  // buffer stores per (p-row, quad)
#pragma unroll
  for (int k = 0; k < NBUF - 1; ++k)
    if (k < nk) issue(k);
  for (int64_t k = 0; k < nk; ++k) {
    // retire stage k: the ops younger than its DMA are the stages issued after
    // it and the stores of every stage mixed since it was issued -- min(k,
    // NBUF - 1) of them (vmcnt retires loads and stores in issue order).  r04:
    // the count before held one stage's stores, so with NBUF > 2 each stage
    // also waited for the write acknowledgements of the stores NBUF - 2 stages
    // back (DOL_PM_WAIT=0 restores it, for measurement).
    const int64_t ahead = std::min<int64_t>(nk - 1, k + NBUF - 2) - k;
    const int64_t st_groups = wait_all_stores ? std::min<int64_t>(k, NBUF - 1) : (k >= 1 ? 1 : 0);
    wait_vmcnt(static_cast<int>(std::min<int64_t>(63, kStores * spt * st_groups + kDma * ahead)));
    __builtin_amdgcn_s_barrier();  // every wave's share landed; buffer (k-1) % NBUF is free
    if (k + NBUF - 1 < nk) issue(k + NBUF - 1);
    const int64_t p0 = stage_of(k) * sr;
    const float* im0 = img + (k % NBUF) * SF;
    mix_stage<T, QPT, SAUX, COPY, OBJ, MODE>(Q, im0, YT, ldy, n_rows, P, p0, xw, sr, spt, q0, g, GR, rowptr, col, val,
                                            e, nw);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this stage's LDS reads are done before the next barrier
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ----------------------------------------------------------------------------
// Tiled transpose B[c][r] = A[r][c] (fp32, 64 x 64 tiles through LDS, rows
// padded by one float against bank conflicts): converts the agent-major bank
// to the parameter-major one and back (setup / checkpoint time, not per round).
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ A, int64_t lda,
                                                        float* __restrict__ B, int64_t ldb, int64_t rows,
                                                        int64_t cols, int64_t tiles_c) {
  __shared__ float t[64][65];
  const int64_t tr = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int lx = threadIdx.x & 63, ly = threadIdx.x >> 6;
  const int64_t r0 = tr * 64, c0 = tc * 64;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t r = r0 + ly + 4 * i, c = c0 + lx;
    if (r < rows && c < cols) t[ly + 4 * i][lx] = A[r * lda + c];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t c = c0 + ly + 4 * i, r = r0 + lx;
    if (r < rows && c < cols) B[c * ldb + r] = t[lx][ly + 4 * i];
  }
}

// stage order set by dol_pm_set_stage_order (0: DOL_PM_NSEG, else 8); atomic,
// and the _ex entry points take the order per call
std::atomic<int> g_pm_nseg{0};

int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}

int n_cus() {
  static const int n = [] {
    int dev = 0, cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cu = 0;
    return cu;
  }();
  return n;
}

}  // namespace

extern "C" {

// The best stage order depends on where the bank's pages landed: on one box,
// process to process, the same mix took 13.35 ms at 8 segments and 12.94 at 32
// in one process and 11.79 / 12.31 in the next (tools/pm_nseg_sweep.py,
// profiles/r03_pm_stage_order.txt); dolhip.ops.tune_pm_stage_order picks it per
// process for the buffers at hand.
int dol_pm_set_stage_order(int32_t nseg) {
  if (nseg < 0 || nseg > 256) return fail(DOL_EINVAL, "dol_pm_set_stage_order: segments %d outside [0, 256]", nseg);
  const int prev = g_pm_nseg.exchange(nseg, std::memory_order_relaxed);
  dol::g_err[0] = '\0';
  return prev;
}

}  // extern "C"

namespace {

// obj < 0: the plain mix; else the config-3 round (epilogue e, momentum mode)
int mix_csr_pm_impl(const char* nm, const float* XT, int64_t ldx, int32_t x_rows, float* YT, int64_t ldy,
                    int32_t n_rows, int64_t P, const int32_t* rowptr, const int32_t* col, const float* val, int obj,
                    int mode, const PmDgd& e, int32_t nseg_req, hipStream_t s) {
  if (nseg_req < 0 || nseg_req > 256) return fail(DOL_EINVAL, "%s: stage order %d outside [0, 256]", nm, nseg_req);
  if (n_rows < 0 || x_rows < 0 || P < 0) return fail(DOL_EINVAL, "%s: negative size", nm);
  if (n_rows == 0 || P == 0) { dol::g_err[0] = '\0'; return DOL_OK; }
  if (!XT || !YT || !rowptr || (x_rows > 0 && (!col || !val))) return fail(DOL_EINVAL, "%s: null pointer", nm);
  if (x_rows < 1) return fail(DOL_EINVAL, "%s: x_rows must be >= 1", nm);
  if (x_rows > kMaxAgents || n_rows > kMaxAgents)
    return fail(DOL_EINVAL, "%s: at most %d agents (x_rows %d, n_rows %d)", nm, kMaxAgents, x_rows, n_rows);
  if (ldx % 4 || ldx < (x_rows + 3) / 4 * 4 || ldy % 4 || ldy < (n_rows + 3) / 4 * 4)
    return fail(DOL_EINVAL, "%s: ldx / ldy must be multiples of 4 covering the rounded-up agent counts", nm);
  if ((reinterpret_cast<uintptr_t>(XT) | reinterpret_cast<uintptr_t>(YT)) & 15u)
    return fail(DOL_EINVAL, "%s: XT and YT must be 16-B aligned", nm);
  if (XT == YT) return fail(DOL_EINVAL, "%s: XT and YT alias (Jacobi mix needs two buffers)", nm);
  const int xw = (x_rows + 255) / 256 * 256;
  const int nq = (n_rows + 3) / 4;
  const int nw = 4 * nq;                                  // epilogue image width (floats)
  const int ne = obj < 0 ? 0 : (mode == 2 ? 2 : 1);       // epilogue operands staged per p-row
  if (obj >= 0) {
    if (!e.T || (mode != 0 && !e.M)) return fail(DOL_EINVAL, "%s: null target / momentum", nm);
    if (e.ldt % 4 || e.ldt < nw || (mode != 0 && (e.ldm % 4 || e.ldm < nw)))
      return fail(DOL_EINVAL, "%s: ldt / ldm must be multiples of 4 covering the rounded-up agent count", nm);
    if ((reinterpret_cast<uintptr_t>(e.T) | (mode ? reinterpret_cast<uintptr_t>(e.M) : 0)) & 15u)
      return fail(DOL_EINVAL, "%s: target / momentum must be 16-B aligned", nm);
    if (nq > kT1 || xw > 4096) return fail(DOL_EINVAL, "%s: the fused round takes at most 4096 agents", nm);
  }
  // geometry: 1024-thread workgroups, one per CU.  Up to 4096 agents (one quad
  // per thread): 64 KiB stages, 2 buffers; beyond (two quads per thread, a
  // p-row up to 32 KiB): 32 KiB stages, 5 buffers (r02; 4 in r01).  Measured at 1024 x 2^20
  // (one box): 64 KiB x 2 1.511 ms, 32 KiB x 4 1.533, 48 KiB x 3 1.541;
  // 256- / 512-thread workgroups (8 / 16 KiB stages, 2-4 per CU) 1.82 / 1.64;
  // one stage per short-lived workgroup 4.4; a per-wave ring (no workgroup
  // barrier, 4 KiB p-rows, 176 VGPRs) 1.64.
  const bool big = nq > kT1 || xw > 4096;
  // fused round: 64 KiB x 2 stages, or 80 KiB x 2 with the momentum read (1024
  // x 2^20 rr4, one box, twice: least squares + momentum 3.45 ms vs 3.56 with
  // 64 KiB x 2 and 3.49 with 48 KiB x 3; logistic, no momentum, 2.25 vs 2.43 /
  // 2.55).  DOL_PM_DGD_GEOM (0 / 1 / 2) overrides, for measurement.
  const int dgeo = obj >= 0 ? env_int("DOL_PM_DGD_GEOM", ne == 2 ? 2 : 0) : 0;
  const int SF = big ? 8192 : (dgeo == 1 ? 12288 : dgeo == 2 ? 20480 : 16384);
  // beyond 4096 agents: five 32-KiB buffers (all 160 KiB, four p-rows in flight)
  // (profiles/r02_pm_nbuf.txt); DOL_PM_BIG_NB=4 keeps four.  At <= 4096 agents
  // 5 x 32 KiB ran level with 2 x 64 KiB (1.56-1.59 ms at 1024 x 2^20)
  static const int big_nb = env_int("DOL_PM_BIG_NB", 5) == 4 ? 4 : 5;
  const int NB = big ? big_nb : (dgeo == 1 ? 3 : 2);  // must match the kernel's NBUF (LDS size)
  int sr = SF / (xw + ne * nw);
  int qp_log2 = 0, spt;
  if (!big) {
    while ((1 << qp_log2) < nq) ++qp_log2;
    const int gr = kT1 >> qp_log2;
    if (sr >= gr) sr = std::min(sr / gr * gr, 4 * gr);
    spt = (sr + gr - 1) / gr;
  } else {
    sr = 1;
    spt = 2;
  }
  if (sr < 1) return fail(DOL_EINVAL, "%s: a p-row and its epilogue operands exceed a stage", nm);
  if (int64_t(sr) * std::max(ldy, std::max(e.ldt, e.ldm)) * 4 >= (int64_t(1) << 31))
    return fail(DOL_EINVAL, "%s: leading dimension too large", nm);
  const int64_t n_stages = (P + sr - 1) / sr;
  const int ncu = n_cus();
  if (ncu <= 0) return fail(DOL_EINVAL, "%s: no device", nm);
  // measurement knobs: DOL_PM_VARIANT 1 = default-policy DMA loads, 4 = copy in
  // this geometry (the structure's ceiling); DOL_PM_NSEG = stage-order segments
  const int var = obj < 0 ? env_int("DOL_PM_VARIANT", 0) : 0;
  auto go = [&](auto kern) {
    const int lds = NB * SF * 4;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    const int64_t grid = std::min<int64_t>(ncu, n_stages);
    const int proc = g_pm_nseg.load(std::memory_order_relaxed);
    int nseg = nseg_req > 0 ? nseg_req : proc > 0 ? proc : env_int("DOL_PM_NSEG", 8);
    if (nseg < 1 || grid % nseg) nseg = 1;
    static const int wait_mode = env_int("DOL_PM_WAIT", 1);
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(grid)), dim3(kT1), lds, s, XT, ldx, x_rows, YT, ldy, n_rows, P,
                       xw, sr, qp_log2, spt, n_stages, nseg, rowptr, col, val, e, nw, wait_mode);
  };
  using std::integral_constant;
  if (obj >= 0) {  // small geometry only
    auto ge = [&](auto oc, auto mc) {
      constexpr int Oc = decltype(oc)::value, Mc = decltype(mc)::value;
      if (dgeo == 1) go(csr_pm_kernel<kT1, 12288, 3, 1, 2, 2, false, Oc, Mc>);
      else if (dgeo == 2) go(csr_pm_kernel<kT1, 20480, 2, 1, 2, 2, false, Oc, Mc>);
      else go(csr_pm_kernel<kT1, 16384, 2, 1, 2, 2, false, Oc, Mc>);
    };
    using O0 = integral_constant<int, 0>;
    using O1 = integral_constant<int, 1>;
    using M0 = integral_constant<int, 0>;
    using M1 = integral_constant<int, 1>;
    using M2 = integral_constant<int, 2>;
    if (obj == 0) { if (mode == 0) ge(O0{}, M0{}); else if (mode == 1) ge(O0{}, M1{}); else ge(O0{}, M2{}); }
    else { if (mode == 0) ge(O1{}, M0{}); else if (mode == 1) ge(O1{}, M1{}); else ge(O1{}, M2{}); }
    return check_launch(nm);
  }
  auto pick = [&](auto sfc, auto nbc, auto qc) {
    constexpr int SFc = decltype(sfc)::value, NBc = decltype(nbc)::value, Qc = decltype(qc)::value;
    if (var == 1) go(csr_pm_kernel<kT1, SFc, NBc, Qc, 0, 2>);
    else if (var == 4) go(csr_pm_kernel<kT1, SFc, NBc, Qc, 2, 2, true>);
    else go(csr_pm_kernel<kT1, SFc, NBc, Qc, 2, 2>);
  };
  if (big && big_nb == 5) pick(integral_constant<int, 8192>{}, integral_constant<int, 5>{}, integral_constant<int, 2>{});
  else if (big) pick(integral_constant<int, 8192>{}, integral_constant<int, 4>{}, integral_constant<int, 2>{});
  else pick(integral_constant<int, 16384>{}, integral_constant<int, 2>{}, integral_constant<int, 1>{});
  return check_launch(nm);
}

}  // namespace

extern "C" {

int dol_mix_csr_pm_f32(const float* XT, int64_t ldx, int32_t x_rows, float* YT, int64_t ldy, int32_t n_rows,
                       int64_t P, const int32_t* rowptr, const int32_t* col, const float* val, hipStream_t s) {
  return dol_mix_csr_pm_ex_f32(XT, ldx, x_rows, YT, ldy, n_rows, P, rowptr, col, val, 0, s);
}

int dol_mix_csr_pm_ex_f32(const float* XT, int64_t ldx, int32_t x_rows, float* YT, int64_t ldy, int32_t n_rows,
                          int64_t P, const int32_t* rowptr, const int32_t* col, const float* val, int32_t nseg,
                          hipStream_t s) {
  DOL_DIMS_OK("dol_mix_csr_pm_f32", ldx, ldy, P);
  return mix_csr_pm_impl("dol_mix_csr_pm_f32", XT, ldx, x_rows, YT, ldy, n_rows, P, rowptr, col, val, -1, 0, PmDgd{},
                         nseg, s);
}

int dol_dgd_csr_pm_f32(const float* XT, int64_t ldx, int32_t x_rows, float* YT, int64_t ldy, int32_t n_rows,
                       int64_t P, const int32_t* rowptr, const int32_t* col, const float* val, const float* TT,
                       int64_t ldt, float* MT, int64_t ldm, int32_t objective, int32_t local_steps, float lr,
                       float momentum, int first_step, hipStream_t s) {
  return dol_dgd_csr_pm_ex_f32(XT, ldx, x_rows, YT, ldy, n_rows, P, rowptr, col, val, TT, ldt, MT, ldm, objective,
                               local_steps, lr, momentum, first_step, 0, s);
}

int dol_dgd_csr_pm_ex_f32(const float* XT, int64_t ldx, int32_t x_rows, float* YT, int64_t ldy, int32_t n_rows,
                          int64_t P, const int32_t* rowptr, const int32_t* col, const float* val, const float* TT,
                          int64_t ldt, float* MT, int64_t ldm, int32_t objective, int32_t local_steps, float lr,
                          float momentum, int first_step, int32_t nseg, hipStream_t s) {
  DOL_DIMS_OK("dol_dgd_csr_pm_f32", ldx, ldy, P, ldt, ldm);
  const char* nm = "dol_dgd_csr_pm_f32";
  if (objective != 0 && objective != 1) return fail(DOL_EINVAL, "%s: objective must be 0 or 1", nm);
  if (local_steps < 1) return fail(DOL_EINVAL, "%s: local_steps must be >= 1", nm);
  const int mode = momentum == 0.0f ? 0 : (first_step ? 1 : 2);
  const PmDgd e{TT, ldt, mode ? MT : nullptr, mode ? ldm : 0, -lr, momentum, local_steps};
  return mix_csr_pm_impl(nm, XT, ldx, x_rows, YT, ldy, n_rows, P, rowptr, col, val, objective, mode, e, nseg, s);
}

int dol_transpose_f32(const float* A, int64_t lda, float* B, int64_t ldb, int64_t rows, int64_t cols, hipStream_t s) {
  DOL_DIMS_OK("dol_transpose_f32", lda, ldb, rows, cols);
  const char* nm = "dol_transpose_f32";
  if (rows < 0 || cols < 0) return fail(DOL_EINVAL, "%s: negative size", nm);
  if (rows == 0 || cols == 0) { dol::g_err[0] = '\0'; return DOL_OK; }
  if (!A || !B) return fail(DOL_EINVAL, "%s: null pointer", nm);
  if (lda < cols || ldb < rows) return fail(DOL_EINVAL, "%s: lda < cols or ldb < rows", nm);
  if (A == B) return fail(DOL_EINVAL, "%s: in-place transpose is not supported", nm);
  const int64_t tr = (rows + 63) / 64, tc = (cols + 63) / 64;
  if (tr * tc >= (int64_t(1) << 31)) return fail(DOL_EINVAL, "%s: too large", nm);
  hipLaunchKernelGGL(transpose_kernel, dim3(static_cast<unsigned>(tr * tc)), dim3(256), 0, s, A, lda, B, ldb, rows,
                     cols, tc);
  return check_launch(nm);
}

}  // extern "C"
