/*
 * dol_hip.h — C-ABI of the MI355X (gfx950) consensus / primal-dual engine.
 *
 * Every entry point replaces one per-agent Python loop of the reference
 * (AlirezaMoseni/Distributed-Optimization-and-Learning); the reference symbol
 * each one stands in for is cited on its declaration.  Path shorthand:
 *   DIST/ = "Distributed Optimization/src/"   (gossip, "Weighted Average")
 *   DEC/  = "Decentralized Optimization/src/" (FedAvg/FedProx/FedADMM server)
 *
 * Conventions (all entry points):
 *   - Stacked state: agent k's flattened parameter vector is row k of a
 *     row-major fp32 matrix with leading dimension `ld*` (elements, >= P).
 *     Flattening order = the model's state_dict() key order.
 *   - All pointers are caller-owned DEVICE memory (hipMalloc / torch CUDA
 *     tensors) unless stated; nothing here allocates, frees or synchronises,
 *     so every call may be captured into a hipGraph.
 *   - Work is enqueued on the caller's stream `s` (NULL = legacy default).
 *   - Return 0 on success; DOL_EINVAL (-1) for a bad argument; otherwise
 *     -(hipError_t) of the failing launch.  dol_last_error() returns a
 *     thread-local message describing the last failure on this thread.
 *   - Arithmetic is fp32 with the reference's rounding sequence (documented
 *     per call); the library is compiled with -ffp-contract=off and uses an
 *     explicit fused multiply-add only where the reference's CPU path does.
 */
#ifndef DOL_HIP_H_
#define DOL_HIP_H_

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DOL_OK 0
#define DOL_EINVAL (-1)
/* dol_bank_alloc only: the retired-address-space cap would be exceeded (outside
 * the -(hipError_t) range). */
#define DOL_ECAP (-100000)

/* Library version, e.g. 100 for 0.1.0. */
int dol_version(void);

/* Thread-local description of the last error on this thread ("" if none). */
const char* dol_last_error(void);

/*
 * Generic sparse gossip mix  Y[i,:] = sum_{e in rowptr[i]..rowptr[i+1]} val[e] * X[col[e],:]
 *
 * Replaces Simulator.Neighbors + Client.consensus + the Jacobi write-back:
 *   DIST/simulators.py:91-97  (Neighbors: j ascending, keep W[i][j] > 0)
 *   DIST/clients.py:61-69     (consensus: w_avg = 0; w_avg += x_j * a_ij)
 *   DIST/simulators.py:148-152 (all rows mixed from the old X, then loaded)
 * Rounding: acc = +0.0f; for e ascending: acc = fl(acc + fl(val[e]*x)).
 * The caller builds the CSR with the reference's selection rule (ascending
 * column, entries with W_ij <= 0 or NaN dropped); an empty row yields zeros.
 * X and Y must not alias.  col[] indexes rows of X (0 <= col < x_rows).
 */
int dol_mix_csr_f32(const float* X, int64_t ldx, int32_t x_rows,
                    float* Y, int64_t ldy, int32_t n_rows, int64_t P,
                    const int32_t* rowptr, const int32_t* col, const float* val,
                    hipStream_t s);

/*
 * dol_mix_csr_f32 on the PARAMETER-MAJOR bank (the agent-major one
 * transposed): XT[p * ldx + j] = agent j's parameter p, for p < P.
 *   YT[p][i] = sum_{e in rowptr[i]..rowptr[i+1]} val[e] * XT[p][col[e]]
 * Same reference code and the same rounding as dol_mix_csr_f32 (bit-identical
 * results, transposed): DIST/simulators.py:91-97 + DIST/clients.py:61-69.
 * Each p-row is one contiguous mixing problem, so X and Y stream from HBM once
 * in order for any graph (the agent-major CSR kernel re-reads each row deg
 * times).  Limits: x_rows, n_rows <= 8192; ldx, ldy multiples of 4 with
 * ldx >= round_up(x_rows, 4), ldy >= round_up(n_rows, 4); XT, YT 16-B aligned,
 * not aliased; 0 <= col < x_rows.
 */
int dol_mix_csr_pm_f32(const float* XT, int64_t ldx, int32_t x_rows, float* YT, int64_t ldy, int32_t n_rows,
                       int64_t P, const int32_t* rowptr, const int32_t* col, const float* val, hipStream_t s);
/* The same call with the stage order given per call (nseg as
 * dol_pm_set_stage_order; 0 = the process setting).  Same bits for every order. */
int dol_mix_csr_pm_ex_f32(const float* XT, int64_t ldx, int32_t x_rows, float* YT, int64_t ldy, int32_t n_rows,
                          int64_t P, const int32_t* rowptr, const int32_t* col, const float* val, int32_t nseg,
                          hipStream_t s);

/*
 * Stage order of the parameter-major kernels (dol_mix_csr_pm_f32,
 * dol_dgd_csr_pm_f32) for this process: the P range is streamed as `nseg`
 * separate regions at once (a divisor of the CU count; others fall back to 1).
 * 0 restores the default (DOL_PM_NSEG, else 8).  Results are the same bits for
 * every order; only the HBM channel balance changes, and with it the speed,
 * which depends on where the buffers' pages landed.  Returns the previous
 * setting, or DOL_EINVAL for nseg outside [0, 256].  No reference counterpart
 * (a launch parameter of this implementation).  The setting is atomic (a call
 * on another thread sees the old or the new order, never a torn one); callers
 * that share the library between threads pass the order per call instead
 * (dol_mix_csr_pm_ex_f32 / dol_dgd_csr_pm_ex_f32).
 */
int dol_pm_set_stage_order(int32_t nseg);

/*
 * Kernel of dol_mix_ring_steps_f32 for this process: 1 = register tiles
 * (ring_steps_kernel), 2 = streaming (ring_stream_kernel), 3 / 4 / 5 =
 * streaming with the rows arriving by LDS-DMA (ring_stream_dma_kernel: plain,
 * block-synchronised once per 8 rows, 64-row tiles in column-tile-fastest
 * order); the streaming kernels need n_rows >= 2 * steps + 17 (else tiles).
 * 0 = the default (DOL_RING_STREAM, else tiles).  Same bits for every
 * variant.  Returns the previous setting, or DOL_EINVAL outside [0, 5].
 * No reference counterpart (a launch choice of this implementation).  Atomic,
 * like dol_pm_set_stage_order; dol_mix_ring_steps_ex_f32 takes it per call.
 */
int dol_ring_steps_set_variant(int32_t variant);

/*
 * dol_mix_csr_f32 for HIGH-DEGREE graphs (tens to thousands of neighbours per
 * row: Erdos-Renyi, dense-ish time-varying W; BASELINE config 5), same
 * reference code (DIST/simulators.py:91-97 + DIST/clients.py:61-69), same
 * rounding, bit-identical results.  X's columns stream through LDS in chunks
 * of DOL_SLAB_CHUNK agents; each row's neighbour sum is gathered from LDS in
 * ascending column order.  The CSR comes re-packed chunk-major by
 * dol_csr_slab_pack (rows in groups of DOL_SLAB_ROWS, each row dealt to a
 * SLOT of its group so the kernel's 16 waves get even per-chunk loads; for
 * group g and chunk k the entries of the group's slots with columns in the
 * chunk are contiguous, in slot order):
 *   ent  int32 [dol_csr_slab_ent_len(nnz, n_rows, x_rows)]: (weight bits, LDS
 *        byte offset) entries stored in pairs as (weight 0, offset 0, weight 1,
 *        offset 1); every (slot, chunk) segment padded to an even number of
 *        entries with a (0, 65536) entry, which the kernel reads from a zero
 *        piece in LDS (its +0 product leaves every sum's bits unchanged)
 *   hdr  int32 [dol_csr_slab_hdr_len(n_rows, x_rows)]: hdr[g][k][s] = ent
 *        index of slot s's first entry in chunk k (s <= ROWS; even), bit 0 set
 *        when that segment ends in a pad entry; then perm[g][s] = the row in
 *        slot s of group g (-1: none) and inv[row] = its slot
 * A row's entries keep their ascending column order whatever its slot, so the
 * sums (and bits) do not depend on the dealing.
 * Limits: ldx, ldy multiples of 4, ldx >= round_up(P, 4) (X rows readable in
 * whole 16-B pieces), X, Y and ent 16-B aligned, X and Y not aliased.
 */
#define DOL_SLAB_CHUNK 64
#define DOL_SLAB_ROWS 128
int dol_csr_slab_nk(int32_t x_rows);
int64_t dol_csr_slab_hdr_len(int32_t n_rows, int32_t x_rows);
int64_t dol_csr_slab_ent_len(int64_t nnz_capacity, int32_t n_rows, int32_t x_rows);
int dol_mix_csr_slab_f32(const float* X, int64_t ldx, int32_t x_rows, float* Y, int64_t ldy, int32_t n_rows,
                         int64_t P, const int32_t* ent, const int32_t* hdr, hipStream_t s);
/* ent and hdr (above) of a device CSR (rowptr / col / val as dol_mix_csr_f32,
 * 0 <= col < x_rows); ent sized for the CSR's nnz (or a capacity >= nnz).
 * balance = 0: slots in row order; 1: rows dealt to the 16 waves by greedy
 * vector packing of their per-chunk entry counts (x_rows <= 32768; measured
 * 0.5-1 % off the mix at 1024 x 101,770 ER p = 0.1 for 0.13 ms of packing, so
 * worth it only when one W is mixed many times). */
int dol_csr_slab_pack(const int32_t* rowptr, const int32_t* col, const float* val, int32_t n_rows,
                      int32_t x_rows, int32_t balance, int32_t* ent, int32_t* hdr, hipStream_t s);
/* Kernel of dol_mix_csr_slab_f32 for this process: 0 = default (DOL_SLAB_KERNEL,
 * else 3), 1 = a loop per (row, chunk) segment (r03), 2 = each wave's pairs as
 * one software-pipelined stream (r06), 3 = that stream hand-scheduled in
 * assembly (r06; P >= 2^30 runs 2).  Same bits for every variant.  Returns the
 * previous setting, or DOL_EINVAL outside [0, 3].  No reference counterpart (a
 * launch choice). */
int dol_slab_set_variant(int32_t variant);
/*
 * Neighbors (DIST/simulators.py:91-97) of every row of a dense device W, on
 * the device: rowptr[n_rows + 1] and col / val (capacity cap >= n_rows *
 * n_cols entries; nnz = rowptr[n_rows]) with the reference's selection
 * (W_ij > 0, NaN and <= 0 dropped, j ascending): a W drawn every round
 * (dol_er_stochastic_f32) becomes a CSR without a host round trip.
 * n_rows * n_cols < 2^31.
 */
int dol_dense_to_csr_f32(const float* W, int64_t ldw, int32_t n_rows, int32_t n_cols, int32_t* rowptr,
                         int32_t* col, float* val, int64_t cap, hipStream_t s);

/*
 * B[c * ldb + r] = A[r * lda + c] for r < rows, c < cols (fp32, tiled through
 * LDS): converts the agent-major bank to the parameter-major one and back
 * (setup and checkpoint time, not on the round path).  A and B must not alias.
 */
int dol_transpose_f32(const float* A, int64_t lda, float* B, int64_t ldb, int64_t rows, int64_t cols,
                      hipStream_t s);

/*
 * Ring (circle topology) specialisation of dol_mix_csr_f32:
 *   Y[i,:] = fl(fl(+0 + fl(w_prev[i]*X[i-1,:])) + fl(w_next[i]*X[i+1,:]))
 * Replaces the same reference code as dol_mix_csr_f32 for
 * communication_graph("circle", ...) (DIST/simulators.py:42-47), where every
 * row has exactly the two neighbours i-1 and i+1 (mod n) with W > 0.  Two
 * addends commute exactly, so this equals the ascending-column order.
 * Row -1 is `halo_prev` and row n_rows is `halo_next` (each a P-vector);
 * pass NULL for both to wrap around inside X (single-shard ring, n_rows>=3).
 * w_prev/w_next: device arrays [n_rows].  X and Y must not alias.
 */
int dol_mix_ring_f32(const float* X, int64_t ldx, float* Y, int64_t ldy,
                     int32_t n_rows, int64_t P,
                     const float* halo_prev, const float* halo_next,
                     const float* w_prev, const float* w_next,
                     hipStream_t s);
/*
 * Only the two BOUNDARY rows (0 and n_rows - 1) of dol_mix_ring_f32 with halos,
 * in one launch: the second half of a sharded ring round (the interior rows
 * 1..n-2 are mixed while the halo rows travel between ranks, the reference's
 * neighbour read DIST/simulators.py:96 become RCCL send/recv).  Same
 * arithmetic as dol_mix_ring_f32; n_rows == 1 mixes its one row from both
 * halos.  halo_prev / halo_next must be non-NULL.
 */
int dol_mix_ring_edges_f32(const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t n_rows, int64_t P,
                           const float* halo_prev, const float* halo_next, const float* w_prev,
                           const float* w_next, hipStream_t s);

/*
 * `steps` synchronous ring rounds in ONE pass over HBM (temporal blocking):
 * Y = W^steps X for the wrap-around ring of dol_mix_ring_f32, replacing the
 * eps consensus steps of FedLCon.run (DIST/simulators.py:190-196; the
 * reference applies Neighbors + consensus + load_state_dict eps times).
 * Each intermediate value is computed with the single-round formula, so Y is
 * bit-identical to `steps` calls of dol_mix_ring_f32 (ping-ponging buffers).
 * Requires 16-B aligned rows, P % 4 == 0, n_rows >= 3, 1 <= steps <= 8.
 */
int dol_mix_ring_steps_f32(const float* X, int64_t ldx, float* Y, int64_t ldy,
                           int32_t n_rows, int64_t P, int32_t steps,
                           const float* w_prev, const float* w_next, hipStream_t s);
/* The same call with the kernel given per call (variant as
 * dol_ring_steps_set_variant; 0 = the process setting).  Same bits. */
int dol_mix_ring_steps_ex_f32(const float* X, int64_t ldx, float* Y, int64_t ldy,
                              int32_t n_rows, int64_t P, int32_t steps,
                              const float* w_prev, const float* w_next, int32_t variant, hipStream_t s);

/*
 * Dense mix on the matrix cores:  Y[M,P] = W[M,K] . X[K,P]   (fp32 MFMA)
 * For dense mixing matrices (communication_graph("compelete", ...), Erdos-
 * Renyi, time-varying W; DIST/simulators.py:54-58 and :59-64 with stochastic
 * weights), replacing the same Neighbors + consensus loop as dol_mix_csr_f32.
 * Numerics: per output an fma chain over k ascending (v_mfma_f32_32x32x2_f32),
 * not the reference's separately rounded mul-then-add with W_ij <= 0 skipped:
 * results differ from the reference by at most ~K ulp-scaled sum|W||X|
 * (error bound gamma_K); use dol_mix_csr_f32 when bit-exactness is required.
 * W row-major with ldw >= K; X, Y row stride ldx, ldy >= P; X, Y must not alias.
 */
int dol_mix_dense_f32(const float* W, int64_t ldw, const float* X, int64_t ldx,
                      float* Y, int64_t ldy, int32_t M, int32_t K, int64_t P,
                      hipStream_t s);

/*
 * Dense mix on the bf16 matrix cores at fp32 accuracy ("split3"): the same
 * Y[M,P] = W[M,K] . X[K,P] and the same reference call sites as
 * dol_mix_dense_f32 (DIST/simulators.py:54-70 + DIST/clients.py:61-69), with
 * every operand split into three bf16 pieces (exact) and the six leading
 * piece products summed on v_mfma_f32_32x32x16_bf16 in fp32: 2.67x the
 * exact-f32 MFMA rate.  Error: |Y - W.X| <= (gamma_{6K'} + 2^-23) sum|W||X|
 * with gamma in units of 2^-23 (K' = K rounded up to 16); tests state the
 * observed maximum.  Finite inputs (0 * Inf of a dense GEMM gives NaN).
 * A split pass writes X's pieces to `work`, then the GEMM runs.  With
 * DOL_SPLIT3_FUSE_X (memory-lean, slower) X is instead split in registers
 * inside the GEMM when its rows are 16-B aligned with ldx % 4 == 0 and readable
 * in whole 16-B pieces (P % 4 == 0, or DOL_SPLIT3_X_ROWS_PADDED: every row
 * readable up to round_up(P, 4) floats); both give the same bits.  `work`
 * (>= dol_mix_dense_split3_workspace_bytes(M, K, P, flags), 256-B aligned)
 * receives the split W (and X); flags & DOL_SPLIT3_W_READY reuses the split W
 * a previous call left in `work` (same W, M, K).  Y must not alias W or X.
 */
#define DOL_SPLIT3_W_READY 1
#define DOL_SPLIT3_X_ROWS_PADDED 2
#define DOL_SPLIT3_FUSE_X 4
int dol_mix_dense_split3_f32(const float* W, int64_t ldw, const float* X, int64_t ldx,
                             float* Y, int64_t ldy, int32_t M, int32_t K, int64_t P,
                             void* work, int64_t work_bytes, int flags, hipStream_t s);
/* Workspace bytes for dol_mix_dense_split3_f32 with these flags: the split W
 * only when FUSE_X | X_ROWS_PADDED promise the fused path, else W + X. */
int64_t dol_mix_dense_split3_workspace_bytes(int32_t M, int32_t K, int64_t P, int flags);

/*
 * One round of decentralised gradient descent on a separable synthetic loss
 * (BASELINE config 3), fused: the gossip mix of dol_mix_ring_f32 /
 * dol_mix_csr_f32 (same arguments, same bit-exact mix), then `local_steps`
 * momentum-SGD iterations per agent in the reference's round order
 * (DIST/simulators.py:147-162: consensus, then local_update with
 * torch.optim.SGD(lr, momentum), DIST/clients.py:17,43-49):
 *   objective 0, least squares f_i(x) = 1/2 ||x - t_i||^2:     g = fl(x - t)
 *   objective 1, logistic (diagonal features, t = label*feature):
 *                f_i(x) = sum_p log(1 + exp(-t_p x_p)):         g = -t / (1 + exp(t x))
 *   buf = (first_step && s == 0) ? g : fl(fl(buf*momentum) + g);  x = fma(-lr, buf or g, x)
 * target: rows aligned with Y (ldt); mom: momentum rows (ldm), NULL iff momentum == 0.
 * One pass streams X (and the neighbours), the targets and the momentum once.
 */
int dol_dgd_ring_f32(const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t n_rows, int64_t P,
                     const float* halo_prev, const float* halo_next, const float* w_prev, const float* w_next,
                     const float* target, int64_t ldt, float* mom, int64_t ldm, int32_t objective,
                     int32_t local_steps, float lr, float momentum, int first_step, hipStream_t s);
int dol_dgd_csr_f32(const float* X, int64_t ldx, int32_t x_rows, float* Y, int64_t ldy, int32_t n_rows, int64_t P,
                    const int32_t* rowptr, const int32_t* col, const float* val, const float* target, int64_t ldt,
                    float* mom, int64_t ldm, int32_t objective, int32_t local_steps, float lr, float momentum,
                    int first_step, hipStream_t s);
/* the boundary rows of dol_dgd_ring_f32 in one launch (see dol_mix_ring_edges_f32) */
int dol_dgd_ring_edges_f32(const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t n_rows, int64_t P,
                           const float* halo_prev, const float* halo_next, const float* w_prev, const float* w_next,
                           const float* target, int64_t ldt, float* mom, int64_t ldm, int32_t objective,
                           int32_t local_steps, float lr, float momentum, int first_step, hipStream_t s);
/*
 * dol_dgd_csr_f32 on the parameter-major bank (XT, YT as dol_mix_csr_pm_f32;
 * TT [P][ldt] the targets and MT [P][ldm] the momentum, transposed the same
 * way): the same mix, the same local steps, bit-identical results, one pass.
 * Target and momentum p-rows ride the mix's LDS stages.  Limits: x_rows,
 * n_rows <= 4096; ldt, ldm multiples of 4 >= round_up(n_rows, 4); TT, MT 16-B
 * aligned; MT NULL iff momentum == 0 (then ldm is ignored).
 */
int dol_dgd_csr_pm_f32(const float* XT, int64_t ldx, int32_t x_rows, float* YT, int64_t ldy, int32_t n_rows,
                       int64_t P, const int32_t* rowptr, const int32_t* col, const float* val, const float* TT,
                       int64_t ldt, float* MT, int64_t ldm, int32_t objective, int32_t local_steps, float lr,
                       float momentum, int first_step, hipStream_t s);
/* dol_dgd_csr_pm_f32 with the stage order per call (see dol_mix_csr_pm_ex_f32). */
int dol_dgd_csr_pm_ex_f32(const float* XT, int64_t ldx, int32_t x_rows, float* YT, int64_t ldy, int32_t n_rows,
                          int64_t P, const int32_t* rowptr, const int32_t* col, const float* val, const float* TT,
                          int64_t ldt, float* MT, int64_t ldm, int32_t objective, int32_t local_steps, float lr,
                          float momentum, int first_step, int32_t nseg, hipStream_t s);

/*
 * Fused local step of n_agents agents (rows of w/buf/g), replacing:
 *   FedProx_Client.update_model  DEC/clients.py:101-115  g' = fl(g + fl(rho*fl(w-theta)))
 *   FedAdmm_Client.update_model  DEC/clients.py:125-139  g' = fl(g + fl(alpha + fl(rho*fl(w-theta))))
 *   FedAvg / gossip local step   DEC/clients.py:85-95, DIST/clients.py:43-49  g' = g
 * followed by torch.optim.SGD(lr, momentum).step()  (DIST/clients.py:17,49; DEC/clients.py:14,44):
 *   momentum != 0: buf = first_step ? g' : fl(fl(buf*momentum) + g');  d = buf
 *   momentum == 0: d = g'
 *   w = fma(-lr, d, w)            (ATen's vectorised add_(d, alpha=-lr))
 * theta: [P] (shared by all agents) or NULL (no proximal/ADMM term).
 * alpha: stacked duals (lda) or NULL (FedProx when theta != NULL).
 * write_grad != 0 stores g' back into g (the reference mutates param.grad).
 * buf may be NULL only when momentum == 0.
 */
int dol_prox_admm_sgd_f32(float* w, int64_t ldw, float* buf, int64_t ldb,
                          float* g, int64_t ldg,
                          const float* theta, const float* alpha, int64_t lda,
                          float rho, float lr, float momentum,
                          int first_step, int write_grad,
                          int32_t n_agents, int64_t P, hipStream_t s);

/*
 * The LAST local FedADMM step of a round fused with the dual ascent, one pass:
 *   dol_prox_admm_sgd_f32(theta, alpha)  then  alpha = fl(alpha + fl(rho*fl(w' - theta)))
 * on the updated w' (DEC/clients.py:125-139, SGD.step, then update_duals
 * :141-144 called at :52).  Bit-identical to the two calls in sequence; reads
 * w, g, buf, alpha once and writes w, buf, alpha (and g if write_grad).
 */
int dol_admm_step_dual_f32(float* w, int64_t ldw, float* buf, int64_t ldb,
                           float* g, int64_t ldg, const float* theta,
                           float* alpha, int64_t lda, float rho, float lr,
                           float momentum, int first_step, int write_grad,
                           int32_t n_agents, int64_t P, hipStream_t s);

/*
 * The proximal / ADMM gradient term alone, in place (no optimizer step):
 *   FedProx_Client.update_model  DEC/clients.py:108-111  g = fl(g + fl(rho*fl(w-theta)))
 *   FedAdmm_Client.update_model  DEC/clients.py:132-135  g = fl(g + fl(alpha + fl(rho*fl(w-theta))))
 * Used when a client's update_model is called on its own (the reference runs
 * optimizer.step() separately, DEC/clients.py:44); the default local step
 * fuses both into dol_prox_admm_sgd_f32.  alpha NULL = FedProx.
 */
int dol_prox_grad_f32(float* g, int64_t ldg, const float* w, int64_t ldw,
                      const float* theta, const float* alpha, int64_t lda,
                      float rho, int32_t n_agents, int64_t P, hipStream_t s);

/*
 * ADMM dual ascent for n_agents agents, replacing
 *   FedAdmm_Client.update_duals  DEC/clients.py:141-144 (called at :52)
 *   alpha = fl(alpha + fl(rho * fl(w - theta)))       (theta: [P], pre-round)
 * resid_sq (nullable, [n_agents] fp64): receives ||w_k - theta||^2 summed in
 * a fixed order (deterministic).  It needs `work` (nullable iff resid_sq is
 * NULL) of dol_admm_dual_workspace_bytes(n_agents, P) bytes.
 */
int dol_admm_dual_f32(float* alpha, int64_t lda, const float* w, int64_t ldw,
                      const float* theta, float rho,
                      int32_t n_agents, int64_t P,
                      double* resid_sq, void* work, hipStream_t s);
int64_t dol_admm_dual_workspace_bytes(int32_t n_agents, int64_t P);

/*
 * One FedADMM client round for m sampled agents on the separable least-squares
 * objective f_k(w) = 1/2 ||w - t_k||^2 (BASELINE config 4's primal/dual side),
 * fused into one pass per agent.  Replaces FedAdmm_Client.update_weights
 * (DEC/clients.py:36-53) with the CNN gradient swapped for the exact
 * least-squares one, for agent row a = agents[k] (agents NULL: a = k):
 *   w = theta                                                    (:37)
 *   local_steps times:  g = fl(w - t_a)
 *     g' = fl(g + fl(alpha + fl(rho * fl(w - theta))))           (:132-135)
 *     momentum != 0: buf = (first[k] && step 0) ? g' : fl(fl(buf*momentum) + g'); d = buf
 *     momentum == 0: d = g'
 *     w = fma(-lr, d, w)                                         (SGD.step, :44)
 *   alpha = fl(alpha + fl(rho * fl(w - theta)))                  (update_duals, :141-144)
 * first: [m] nonzero where agent k takes its first momentum step ever (the
 * reference's optimizer state is never reset), or NULL for none.  w is only
 * written.  resid_sq / alpha_sq (both or neither, fp64 [m]) receive
 * ||w_k - theta||^2 and ||alpha_k||^2 after the round, summed in a fixed order;
 * they need `work` of dol_admm_ls_round_workspace_bytes(m, P) bytes.  The
 * server's average of the new w rows is dol_ordered_mean_f32 (DEC/servers.py:42-48).
 */
int dol_admm_ls_round_f32(float* w, int64_t ldw, float* buf, int64_t ldb, float* alpha, int64_t lda,
                          const float* target, int64_t ldt, const float* theta, const int32_t* agents,
                          const int32_t* first, int32_t m, int64_t P, float rho, float lr, float momentum,
                          int32_t local_steps, double* resid_sq, double* alpha_sq, void* work, hipStream_t s);
int64_t dol_admm_ls_round_workspace_bytes(int32_t m, int64_t P);

/*
 * dol_admm_ls_round_f32 fused with the server's ordered average: the whole
 * round of DEC/servers.py:50-81 (every sampled client's update_weights,
 * DEC/clients.py:36-53, then average_weights, DEC/servers.py:42-48) in one
 * pass.  w / buf / alpha rows come out bit-identical to dol_admm_ls_round_f32,
 * and theta_out to dol_ordered_sum_f32(w, agents, m, P, NULL, theta_out,
 * scale) on them (acc = w[agents[0]]; acc = fl(acc + w[agents[k]]); theta_out
 * = fl(acc / scale) when scale != 1; scale = m is the mean, scale = 1 the raw
 * sum that a multi-rank 'fast' mean all-reduces) — without reading the new w
 * rows back.  agents: [m] DISTINCT rows in the sampled order (NULL: 0..m-1),
 * m >= 1.  theta_out may alias theta (each column is read before it is
 * written); it must not alias the rows.  resid_total (nullable, fp64 [2])
 * receives the round's sums over the agents of ||w_k - theta||^2 and
 * ||alpha_k||^2 (a fixed reduction order, deterministic, not per agent); it
 * needs `work` of dol_admm_ls_round_mean_workspace_bytes(P) bytes.  P < 2^29.
 */
int dol_admm_ls_round_mean_f32(float* w, int64_t ldw, float* buf, int64_t ldb, float* alpha, int64_t lda,
                               const float* target, int64_t ldt, const float* theta, const int32_t* agents,
                               const int32_t* first, int32_t m, int64_t P, float rho, float lr, float momentum,
                               int32_t local_steps, float* theta_out, float scale, double* resid_total, void* work,
                               hipStream_t s);
int64_t dol_admm_ls_round_mean_workspace_bytes(int64_t P);

/*
 * Ordered uniform average, replacing Server.average_weights
 *   DEC/servers.py:42-48:  acc = w[order[0]]; acc = fl(acc + w[order[k]]) k=1..m-1;
 *                          theta = fl(acc / (float)m)
 * order: device int32 [m] of row indices into W (the sampled-client order of
 * DEC/servers.py:57).  theta: [P], must not alias W.
 */
int dol_ordered_mean_f32(const float* W, int64_t ldw, const int32_t* order,
                         int32_t m, int64_t P, float* theta, hipStream_t s);

/*
 * Ordered partial sum without the division (building block for the
 * multi-GPU chain reduce):  acc_out = fl(...fl(acc_in + w[order[0]]) ...)
 * acc_in NULL: start from w[order[0]] exactly (as DEC/servers.py:43).
 * acc_out may alias acc_in.  scale != 1 divides the final result:
 * acc_out = fl(acc / scale) when scale != 1.0f.
 */
int dol_ordered_sum_f32(const float* W, int64_t ldw, const int32_t* order,
                        int32_t m, int64_t P, const float* acc_in,
                        float* acc_out, float scale, hipStream_t s);

/*
 * One fused local step of n_agents per-agent MLPs  Linear(d,h) -> ReLU -> Linear(h,c)
 * with CrossEntropyLoss (mean over the batch), parameters = rows of w in
 * state_dict order [W1 (h x d), b1 (h), W2 (c x h), b2 (c)], P = h*d + h + c*h + c.
 * Replaces, for every agent at once, one iteration of the reference's local loop
 *   DIST/clients.py:34-59   forward, loss, backward, optimizer.step()
 *   DEC/clients.py:101-139  (FedProx / FedADMM gradient terms, theta / alpha)
 * i.e. forward + backward on fp32 MFMA (v_mfma_f32_32x32x2_f32) and the update of
 * dol_prox_admm_sgd_f32 (same rounding) applied to each gradient tile in registers.
 * X: agent k's batch at X + k*ldx_agent, sample b at + b*ldx_row (d floats, 16-B
 * aligned); labels: int64 [k*ldy_agent + b] in [0, c) (out of range -> NaN loss).
 * update == 0: only write the raw gradients to grad (forward_backward); otherwise
 * update w (and mom), and store g' into grad when grad != NULL.  loss: [n_agents]
 * per-agent mean CE, or NULL.  work: device scratch of
 * dol_mlp_step_workspace_bytes(n_agents, B, h) bytes (holds dZ1 between the two
 * launches the step enqueues).  Limits: 1 <= B <= 64, h % 32 == 0 and h <= 256,
 * c <= 32, d % 4 == 0.  GEMM numerics are fp32 fma chains (tolerance, not
 * bit-exact vs torch CPU).
 */
int dol_mlp_step_f32(float* w, int64_t ldw, float* grad, int64_t ldg, float* mom, int64_t ldm,
                     const float* theta, const float* alpha, int64_t lda,
                     const float* X, int64_t ldx_agent, int64_t ldx_row,
                     const int64_t* labels, int64_t ldy_agent, float* loss,
                     int32_t n_agents, int32_t B, int32_t d, int32_t h, int32_t c,
                     float lr, float momentum, float rho, int first_step, int update,
                     void* work, hipStream_t s);
/* Scratch bytes dol_mlp_step_f32 needs (n_agents * B * h floats). */
int64_t dol_mlp_step_workspace_bytes(int32_t n_agents, int32_t B, int32_t h);
/* Dynamic LDS bytes the MLP step uses per workgroup (one agent). */
int64_t dol_mlp_step_lds_bytes(int32_t B, int32_t h, int32_t c);

/*
 * A fresh Erdos-Renyi G(n, p) mixing matrix under the reference's 'stochastic'
 * weighting (DIST/simulators.py:65-70: G = R o A, G /= colsum(G), W = G^T), A
 * undirected with a zero diagonal, for BASELINE config 5's time-varying dense
 * W — one kernel, W written once (rows sum to 1; entries the reference's
 * Neighbors would drop, incl. empty columns, are 0).  Seeded and
 * deterministic (counter-based hash; not torch's generator stream).
 * W row-major [n][ldw], ldw >= n, n <= 65535, 0 <= p <= 1.
 */
int dol_er_stochastic_f32(float* W, int64_t ldw, int32_t n, float p, uint64_t seed, hipStream_t s);

/*
 * Device memory for a bank buffer as ONE physical allocation (hipMemCreate)
 * mapped into a reserved virtual range (hipMemAddressReserve + hipMemMap),
 * rounded up to the allocation granularity (*mapped_bytes).  Free with
 * dol_bank_free(ptr, *mapped_bytes), with the size recorded at allocation: it
 * unmaps the range and releases the physical allocation, and RETIRES the
 * virtual range (keeps it reserved, never reused: on this ROCm stack a range
 * re-mapped after a free was read through stale translations)
 * unless DOL_BANK_FREE_VA=1 (diagnostics: the range is freed).  Retired bytes
 * are counted (dol_bank_retired_bytes / _blocks); dol_bank_alloc returns
 * DOL_ECAP when retired + live mapped + the new block would pass
 * dol_bank_retired_cap_bytes() (DOL_BANK_RETIRED_VA_CAP_GIB, default 4096).
 * dol_bank_free refuses a pointer this library did not hand out or a size
 * other than *mapped_bytes (DOL_EINVAL, before any HIP call) and accepts NULL.
 * A failed step leaves the block registered: calling dol_bank_free again
 * resumes at that step.  Host-side, synchronous, thread-safe, not
 * graph-capturable.  The default for bank matrices of >= 1 GiB
 * (bank.device_matrix); DOL_BANK_ALLOC=torch or mapped=False opts out.  No
 * reference counterpart (the reference keeps one nn.Module per agent in host
 * memory).
 */
int dol_bank_alloc(int64_t bytes, void** ptr, int64_t* mapped_bytes);
int dol_bank_free(void* ptr, int64_t mapped_bytes);
int64_t dol_bank_retired_bytes(void);
int64_t dol_bank_retired_blocks(void);
int64_t dol_bank_retired_cap_bytes(void);

/* Streaming copy dst = src (n floats): HBM calibration kernel for roofline. */
int dol_stream_copy_f32(const float* src, float* dst, int64_t n, hipStream_t s);

/* Y[:, :P] = X[:, :P] by the ring mix's own kernel with the stencil replaced by
 * the tile's row (same launch, loads incl. halo rows, cache policies and
 * stores): the HBM ceiling of exactly that access pattern, the roofline's
 * second calibration (bytes = 2 * n_rows * P * 4, as the mix).  >= 3 rows,
 * 16-B aligned rows, P % 4 == 0. */
int dol_stream_copy_rows_f32(const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t n_rows, int64_t P,
                             hipStream_t s);

#ifdef __cplusplus
}
#endif
#endif /* DOL_HIP_H_ */
