// csr_slab.hip — high-degree sparse mix on the agent-major bank, gathered from LDS.
//
// Same operation, same reference code and the same bits as dol_mix_csr_f32
// (DIST/simulators.py:91-97 Neighbors: j ascending, W_ij > 0 kept;
// DIST/clients.py:61-69 consensus: acc = +0; acc = fl(acc + fl(x_j * a_ij))),
// for graphs whose rows have tens to thousands of neighbours: the Erdos-Renyi
// p = 0.1 W of BASELINE config 5 (about 100 neighbours per row at 1024 agents,
// 820 at 8192), drawn anew every round.  The agent-major CSR kernel fetches
// every neighbour row from L2 (deg L2 reads per output element); the dense
// split3 GEMM runs six bf16 MFMAs per W entry, 90 % of which are zeros, and is
// not bit-exact.  Here each X value is read from HBM once per row group and
// from LDS once per (output row, neighbour):
//
//   * a work item is one SLAB = 256 columns of P and a ROW GROUP of 16 * RW
//     output rows, RW per wave, held in registers (f4 per row per lane: lane l
//     owns columns 4l .. 4l+3 of the slab); a workgroup (16 waves, one per CU)
//     walks its items with the chunk stream running on across them;
//   * the slab's X columns stream through LDS in CHUNKS of 64 agents (64 x 1 KiB,
//     LDS-DMA global_load_lds_dwordx4: each agent's 1 KiB piece is contiguous
//     in HBM and lands contiguous in LDS), double-buffered;
//   * the CSR is re-packed chunk-major (dol_csr_slab_pack): for row group g
//     and chunk k, the entries of the group's rows whose columns fall in the
//     chunk form one contiguous block, (LDS byte offset of the agent's piece,
//     weight bits) pairs in (row, column) order; hdr[g][k][i] = the block's
//     first entry of row i.  Each block rides the chunk's LDS-DMA into LDS
//     beside the X chunk, so the gather loop reads its indices from LDS
//     (in-order, ~120-cycle reads, prefetched a step ahead) instead of scalar
//     loads from L2 (out-of-order returns force a full drain per use: measured
//     2.1 ms vs 0.24 ms of staging at 1024 x 101,770);
//   * each wave walks its 8 rows' chunk segments as one contiguous run of
//     entry PAIRS (pads included: a pad reads a zero piece and adds +0), the
//     next two pairs always in flight behind the current pairs' gathers: per
//     entry one conflict-free ds_read_b128 gather (1 KiB: the wave reads one
//     agent's whole piece) + 4 separately rounded mul / add, per pair one
//     uniform ds_read_b128 of the index.  Chunks are visited in ascending agent
//     order, so each row's sum runs over its CSR entries in exactly the
//     reference's order.
//
// Bounds: LDS bytes = nnz * 1 KiB per slab (256 B/clk/CU), VALU = 5 wave
// instructions per (neighbour, slab) (address add, 2 packed mul, 2 packed
// add).  The row groups of one slab sit on one XCD at the same time
// (blockIdx % 8 = XCD), so the slab's chunks come from HBM once and from that
// XCD's L2 for the others.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/dol_hip.h"
#include "dol_common.h"
#include "csr_slab_stream.inc"

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kCols = 256;                 // slab width (floats): one f4 per lane
constexpr int kChunk = DOL_SLAB_CHUNK;     // agents per LDS chunk
constexpr int kWaves = 16;
constexpr int kThreads = 64 * kWaves;
constexpr int kXBytes = kChunk * kCols * 4;  // 64 KiB of X per chunk
// LDS: stage b = X chunk (64 KiB) + one zero piece (1 KiB) at b * kStage; the
// two index stages (15 KiB each) after them: 2 * 65 + 2 * 15 = 160 KiB.  A pad
// entry's offset is kZeroRel, i.e. the zero piece of whichever stage it is read
// against, with weight 0: its product is +0 and acc + (+0) == acc for every
// acc the sum can hold (+0 start, round-to-nearest never yields -0 from +0),
// so pads are gathered like real entries and leave the bits unchanged.
constexpr int kStage = kXBytes + 1024;
constexpr int kZeroRel = kXBytes;
constexpr int kIdxBytes = 15 * 1024;          // index block capacity per chunk (1920 entries)
constexpr int kIdxBase = 2 * kStage;
constexpr int kLds = 2 * kStage + 2 * kIdxBytes;
// index bytes a stream variant reads past a wave's run (variant 2: two pairs;
// variant 3: DOL_SLAB_STREAM_AHEAD pairs)
constexpr int kAhead = 16 * (DOL_SLAB_STREAM_AHEAD > 2 ? DOL_SLAB_STREAM_AHEAD : 2);
constexpr int kRW = 8;                        // rows per wave
constexpr int kRows = kWaves * kRW;           // rows per row group
constexpr int kEntPad = 160;                  // ent pad entries (the block DMA may read 1 KiB + 8 B past a block)
constexpr int kPerWave = kChunk / kWaves;  // DMA pieces per wave per chunk
static_assert(kChunk % kWaves == 0, "chunk must split evenly over the waves");
static_assert(kLds <= 160 * 1024, "LDS budget");

#define DOL_GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define DOL_LPTR(p) ((__attribute__((address_space(3))) void*)(p))

struct alignas(16) I4 {
  // a PAIR of entries: (weight bits 0, offset 0, weight bits 1, offset 1) -- each
  // weight in an even register of the loaded quad, so v_pk_mul_f32 broadcasts it
  // straight from there (op_sel_hi), no copy into an aligned pair
  int32_t w0, o0, w1, o1;
};

// LDS-DMA of 16 B per lane (1 KiB per wave) from `gptr` to the wave-uniform LDS
// address of `ldst` (the hardware adds lane * 16), written as inline asm: the
// compiler's waitcnt model treats a pending global_load_lds as making LGKM
// returns unordered and then waits lgkmcnt(0) before every LDS read result is
// used, which serialises the gather pipeline below; hidden from it, the gathers
// get counted lgkmcnt waits.  The kernel orders the DMA itself (s_waitcnt
// vmcnt(0) + barrier before a stage is read); any compiler-counted vmcnt wait
// issued later only waits for more, never fewer, loads.
__device__ __forceinline__ void dma16(const void* gptr, void* ldst) {
  const uint32_t la = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(DOL_LPTR(ldst)));
  asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(gptr), "{m0}"(__builtin_amdgcn_readfirstlane(la)) : "memory");
}

// separately rounded mul, then add (v_pk_mul_f32 / v_pk_add_f32 pairs: 1.18 ms
// vs 1.33 with the per-component scalar form at 1024 x 101,770, same bits)
__device__ __forceinline__ f4 fmac(f4 acc, float w, f4 x) { return acc + x * w; }

// LDS byte address of entry word `o`'s piece for this lane (stage base + lane * 16 in `lb`)
__device__ __forceinline__ uint32_t piece_addr(uint32_t o, uint32_t lb) { return o + lb; }

// PROBE (diagnostics, DOL_SLAB_PROBE; results meaningless except 0): 1 = staging
// only (no gathers), 2 = no X staging (index blocks and gathers only), 3 = no
// workgroup barrier per chunk (waves drift; reads race the DMA), 4 = no index
// reads inside a row (every step reuses the row's first two pairs), 5 = the
// products' multiplies dropped (acc += x: half the VALU), 6 = the tails (a
// row's last np % 4 pairs) skipped.
// Each row walks its chunk segment in groups of 4 / 2 / 1 entries: the index
// pairs by uniform ds_read_b128 (segments are padded to even lengths, so two
// entries share one 16-B LDS read: 2 LDS cycles per entry; ds_read2_b64 took
// 4), then the gathers, then separately rounded packed mul / add.
// Tried and dropped (1024 x 101,770; profiles/r02_slab_probe.txt): index by
// v_readlane from a lane-distributed group index (1.17 ms vs 1.12 with
// ds_read2_b64 pairs); the wave's entries as one stream in windows of 4 / 8
// across row boundaries with the accumulator chosen by a uniform switch on a
// row tag (5.4 ms; needs 8 waves x 16 rows for registers, which slow the rest
// to 1.5 ms); row pairs in lockstep, 4 entries per row per step, clamped
// reads, branch-skipped arithmetic (1.73 ms); one stream in steps of up to 4
// entries of one row with the next step's index read across rows (1.35 ms);
// index by scalar loads (2.1 ms).  Chunk headers (row starts, the next block's
// bounds) arrive by vector loads issued with the chunk's DMA, so the chunk
// loop has no scalar-load waits (1.105-1.12 vs 1.135-1.147 ms with s_load).
// Work items: item t = (slab, row group) with t's low 3 bits = the XCD (t & 7),
// slab = ((t >> 3) / n_rg) * 8 + (t & 7), rg = (t >> 3) % n_rg.  Workgroup b
// takes items b, b + G, b + 2G, ... (G = gridDim.x, a multiple of 8, so every
// item of a workgroup is on its XCD); with G = n_items each workgroup runs one
// item.  Persistent (G < n_items): the chunk stream runs on across items — the
// next item's chunk 0 is staged during the current item's last chunk, so a new
// item does not start on an exposed DMA latency (needs nk >= 2).
// STREAM (r06, dol_slab_set_variant(2)): each wave walks its run of entry
// pairs for the chunk as ONE software-pipelined stream instead of a loop per
// row: the index pair two steps ahead and the gathers one step ahead are in
// flight while a pair is summed (registers rotate through a 6-step unrolled
// body, so no copies), and the running sum `a` moves between the wave's 8 row
// accumulators -- one 32-register tuple -- only at a row boundary, by
// dynamically indexed register moves (s_set_gpr_idx_on: 4 moves out, 4 in).
// Per pair: one uniform compare for the boundary; the r03 loop paid a loop
// entry, tail cases and a prefetch per (row, chunk) segment (~30 instructions
// per 6.4-entry segment).  Same entries, same order, same bits.  Reads run at
// most two pairs past the wave's run (kAhead): the index DMA covers them and
// the packer pads past the last block (slab_tail_kernel).
template <int PROBE = 0, bool A4 = false, int SV = 0>
__global__ __launch_bounds__(kThreads) void csr_slab_kernel(
    const float* __restrict__ X, int64_t ldx, int x_rows, float* __restrict__ Y, int64_t ldy, int n_rows, int64_t P,
    const int32_t* __restrict__ ent, const int32_t* __restrict__ hdr, int nk, int n_rg, int64_t n_slabs,
    int64_t n_items) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int64_t G = gridDim.x;
  const int64_t p4 = (P + 3) / 4 * 4;  // X rows are readable up to here (dol_hip.h)
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // SA (the asm stream, SV 2): DMA addresses as a uniform row base plus this
  // lane's 32-bit column byte offset (the host keeps round_up(P, 4) * 4 < 2^32),
  // so an item is uniform state only -- the stream's registers come from here
  constexpr bool SA = SV == 2;
  struct Item {
    int rg;
    int64_t slab;            // uniform
    int64_t p;               // this lane's first column
    const float* xsrc;       // X + the in-bounds DMA column of this lane
    const int32_t* H;        // the row group's chunk blocks
  };
  auto item_at = [&](int64_t t, Item& it) -> bool {  // false: no such item (and none later for this workgroup)
    if (t >= n_items) return false;
    const uint32_t local = uint32_t(t >> 3);
    const int64_t slab = int64_t(local / uint32_t(n_rg)) * 8 + (t & 7);
    if (slab >= n_slabs) return false;
    it.rg = int(local % uint32_t(n_rg));
    it.slab = slab;
    if constexpr (!SA) {
      it.p = slab * kCols + lane * 4;
      const int64_t pl = it.p + 4 <= p4 ? it.p : p4 - 4;  // lanes past P: values unused, reads kept inside round_up(P, 4)
      it.xsrc = X + pl;
    }
    it.H = hdr + int64_t(it.rg) * nk * (kRows + 1);
    return true;
  };
  // SA: this lane's in-bounds DMA column of slab `slab`, in bytes
  auto col_bytes = [&](int64_t slab) -> uint32_t {
    const int64_t p = slab * kCols + lane * 4;
    return uint32_t((p + 4 <= p4 ? p : p4 - 4) * 4);
  };
  const int32_t* perm = hdr + int64_t(n_rg) * nk * (kRows + 1);  // slot -> output row (dol_csr_slab_pack)
  int64_t t = blockIdx.x;
  Item cur, nxt;
  if (!item_at(t, cur)) return;
  bool has_next = item_at(t + G, nxt);
  const uint8_t* entb = reinterpret_cast<const uint8_t*>(ent);

  const int row0 = wave * kRW;  // within the group
  int blk0 = cur.H[0], blk1 = cur.H[kRows];  // the next chunk to stage: its index block [blk0, blk1)
  int hv = 0;                                 // header lanes, see issue()
  // stage chunk k of item `it` into buffer `buf`; `after` = the item whose chunk 0
  // follows it when k is the last chunk (nullptr: none)
  // LDS byte address of the dynamic LDS (hoisted: the generic -> local cast
  // costs a null check per use)
  const uint32_t lds_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(DOL_LPTR(lds)));
  auto issue = [&](const Item& it, int k, int buf, const Item* after) {
    if constexpr (PROBE != 2) {
      // this wave's kPerWave agent pieces of the chunk: one 64-bit product per
      // chunk, then a row stride per piece (agents past x_rows: the last row
      // again, never referenced)
      const int a0w = k * kChunk + wave * kPerWave;
      const uint32_t la = lds_base + uint32_t(buf * kStage + wave * kPerWave * 1024);
      if constexpr (SA) {
        const uint32_t cb = col_bytes(it.slab);
#pragma unroll
        for (int i = 0; i < kPerWave; ++i) {
          const float* row = X + int64_t(min(a0w + i, x_rows - 1)) * ldx;  // uniform
          asm volatile("global_load_lds_dwordx4 %0, %1" ::"v"(cb), "s"(row), "{m0}"(la + i * 1024) : "memory");
        }
      } else if (a0w + kPerWave <= x_rows) {
        const float* src = it.xsrc + int64_t(a0w) * ldx;
#pragma unroll
        for (int i = 0; i < kPerWave; ++i)
          asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(src + i * ldx), "{m0}"(la + i * 1024) : "memory");
      } else {
#pragma unroll
        for (int i = 0; i < kPerWave; ++i) {
          const float* src = it.xsrc + int64_t(min(a0w + i, x_rows - 1)) * ldx;
          asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(la + i * 1024) : "memory");
        }
      }
    }
    // the chunk's index block (16-B aligned start, whole 1 KiB pieces; ent is padded)
    const int64_t a0 = int64_t(blk0 & ~1) * 8;  // even: 16-B aligned
    const int64_t nbytes = int64_t(blk1 & ~1) * 8 - a0;
    if (nbytes <= kIdxBytes - kAhead)
      for (int pc = wave; pc * 1024 < nbytes + (SV ? kAhead : 0); pc += kWaves) {
        if constexpr (SA) {
          const uint32_t la = lds_base + uint32_t(kIdxBase + buf * kIdxBytes + pc * 1024);
          asm volatile("global_load_lds_dwordx4 %0, %1" ::"v"(uint32_t(lane) * 16), "s"(entb + a0 + pc * 1024), "{m0}"(la)
                       : "memory");
        } else {
          dma16(entb + a0 + pc * 1024 + lane * 16, lds + kIdxBase + buf * kIdxBytes + pc * 1024);
        }
      }
    // headers ride the same vmcnt wait: lanes 0..kRW hold chunk k's row starts of
    // this wave's rows, lanes kRW+1 / kRW+2 the block bounds of the chunk after it
    const int32_t* hb = it.H + int64_t(k + 1) * (kRows + 1);   // (it, k + 1)
    if (k + 1 >= nk) hb = after ? after->H : it.H + int64_t(k) * (kRows + 1);  // (after, 0), or unused
    if (lane <= kRW) hv = it.H[int64_t(k) * (kRows + 1) + row0 + lane];
    else if (lane == kRW + 1) hv = hb[0];
    else if (lane == kRW + 2) hv = hb[kRows];
  };

  f4 acc[kRW];
#pragma unroll
  for (int r = 0; r < kRW; ++r) acc[r] = f4{0.f, 0.f, 0.f, 0.f};
  // STREAM: the row accumulators as one register tuple (dynamic row index ->
  // s_set_gpr_idx_on moves; a static index is a plain register)
  typedef float v32 __attribute__((ext_vector_type(32)));
  static_assert(kRW * 4 == 32, "the accumulator tuple holds kRW f4 rows");
  v32 accv = 0.f;
  auto vget = [&](int r) -> f4 { return f4{accv[4 * r], accv[4 * r + 1], accv[4 * r + 2], accv[4 * r + 3]}; };
  auto vset = [&](int r, f4 a) {
    accv[4 * r] = a.x;
    accv[4 * r + 1] = a.y;
    accv[4 * r + 2] = a.z;
    accv[4 * r + 3] = a.w;
  };
  const uint32_t lane16 = uint32_t(lane) * 16;
  if (threadIdx.x < 128)  // the two stages' zero pieces (pads read them); visible after the first barrier
    *reinterpret_cast<f4*>(lds + (threadIdx.x >> 6) * kStage + kZeroRel + lane16) = f4{0.f, 0.f, 0.f, 0.f};

  int g = 0;  // chunks consumed by this workgroup: buffer g & 1
  issue(cur, 0, 0, has_next ? &nxt : nullptr);
  for (;;) {
    Item nn;  // the item after nxt (header bounds of nxt's last chunk)
    const bool has_nn = has_next && item_at(t + 2 * G, nn);
    for (int k = 0; k < nk; ++k, ++g) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // my pieces (and header lanes) of chunk k landed
      if constexpr (PROBE != 3) __syncthreads();         // ... and every wave's; the other buffer is free
      int bnd[kRW + 1];  // header words: (even) first entry | 1 if the row's segment ends in a pad entry
#pragma unroll
      for (int i = 0; i <= kRW; ++i) bnd[i] = __builtin_amdgcn_readlane(hv, i) & ~1;
      const int hcur = hv;  // this chunk's header lanes (issue() below loads the next chunk's into hv)
      const int e0 = blk0 & ~1;
      const bool fits = int64_t((blk1 & ~1) - e0) * 8 <= kIdxBytes - kAhead;
      blk0 = __builtin_amdgcn_readlane(hv, kRW + 1);  // the next chunk's block, for the issue below
      blk1 = __builtin_amdgcn_readlane(hv, kRW + 2);
      if (k + 1 < nk) issue(cur, k + 1, (g + 1) & 1, has_next ? &nxt : nullptr);
      else if (has_next) issue(nxt, 0, (g + 1) & 1, has_nn ? &nn : nullptr);
      if constexpr (PROBE == 1) continue;
      const uint32_t lb = uint32_t((g & 1) * kStage) + lane16;  // stage base + my lane's 16 B
      auto gather = [&](int32_t o) { return *reinterpret_cast<const f4*>(lds + piece_addr(uint32_t(o), lb)); };
      if (!fits) {  // an over-full block (denser graphs): indices from global memory, same order
#pragma unroll
        for (int r = 0; r < kRW; ++r) {
          f4 a = SV ? vget(r) : acc[r];
          for (int e = bnd[r]; e < bnd[r + 1]; ++e) {
            const int64_t q = int64_t(e >> 1) * 4 + 2 * (e & 1);  // (weight, offset)
            a = fmac(a, __int_as_float(ent[q]), gather(ent[q + 1]));
          }
          if constexpr (SV != 0) vset(r, a);
          else acc[r] = a;
        }
        if constexpr (SV != 2) continue;  // SV 2: on into the stream with no pairs (one exit for the tuple)
      }
      // This wave's rows' segments are one contiguous run of entry pairs in the
      // block (row order; every segment an even number of entries, pads
      // included).  Row r's first two pairs are read while row r - 1 is being
      // summed (fa / fb), so a row never starts on an index round trip; inside
      // a row the pairs go two at a time with the next two pairs' index read
      // behind the current gathers, the loop unrolled twice so the prefetched
      // index lands in the registers the next step reads (no copies).  Reads
      // run at most kAhead bytes past the wave's run (inside the stage:
      // `fits` leaves the room).
      const uint32_t ibase = uint32_t(kIdxBase + (g & 1) * kIdxBytes) - uint32_t(e0) * 8;
      auto pair_at = [&](uint32_t a) { return *static_cast<const I4*>(__builtin_assume_aligned(lds + a, 16)); };
      if constexpr (SV == 2) {  // variant 3: the same stream, hand-scheduled (csr_slab_stream.inc)
        const int b0 = bnd[0];
        const int n = fits ? (bnd[kRW] - b0) >> 1 : 0;  // the stream returns at once on n == 0
        uint32_t pbv = ibase + uint32_t(b0) * 8;  // LDS address of the run's pair 0 (advanced by the loop)
        int hb = hcur;  // the header lanes, turned into row-start pair indices by the stream
        asm volatile(DOL_SLAB_STREAM_ASM
                     : [acc] DOL_SLAB_STREAM_ACC(accv), [pb] "+v"(pbv), [hc] "+v"(hb)
                     : [lb] "v"(lb), [n] "s"(n), [b0] "s"(b0)
                     : DOL_SLAB_STREAM_CLOBBERS, "scc", "memory");
        continue;
      }
      if constexpr (SV == 1) {
        const int b0 = bnd[0];
        const int n = (bnd[kRW] - b0) >> 1;  // the wave's pairs in this chunk (all rows, pads included)
        if (n == 0) continue;
        // B(r): pair index where row r starts (B(kRW) = n)
        auto B = [&](int r) { return ((__builtin_amdgcn_readlane(hcur, r) & ~1) - b0) >> 1; };
        const uint32_t pa0 = ibase + uint32_t(b0) * 8;  // LDS address of the run's pair 0
        int r = 0, jb = 0;  // the current row; pair index of this 6-step block's first step
        int nb = B(1);      // pair index where the next row starts
        int nbr = nb;       // ... relative to jb
        uint32_t pb = pa0;  // LDS address of pair jb
        f4 a = vget(0);
        I4 I0 = pair_at(pa0), I1 = pair_at(pa0 + 16), I2;
        f4 G0a = gather(I0.o0), G0b = gather(I0.o1), G1a, G1b;
        // step K of the block (pair jb + K): at a row boundary move the running
        // sum (and skip empty rows; the run's end is the last boundary); then
        // the index two pairs ahead, the gathers one pair ahead, this pair's sum
#define DOL_SLAB_STEP(K, IC, IN, INN, GCA, GCB, GNA, GNB)                      \
        if (nbr == K) {                                                          \
          if (jb + K == n) goto stream_done;                                     \
          vset(r, a);                                                            \
          do { /* rows empty in this chunk keep their sums */                    \
            r = __builtin_amdgcn_readfirstlane(r + 1);                           \
            nb = B(r + 1);                                                       \
          } while (nb == jb + K);                                                \
          a = vget(r);                                                           \
          nbr = nb - jb;                                                         \
        }                                                                        \
        INN = pair_at(pb + 16 * (K + 2));                                        \
        GNA = gather(IN.o0);                                                     \
        GNB = gather(IN.o1);                                                     \
        a = fmac(a, __int_as_float(IC.w0), GCA);                                 \
        a = fmac(a, __int_as_float(IC.w1), GCB);
        for (;;) {
          DOL_SLAB_STEP(0, I0, I1, I2, G0a, G0b, G1a, G1b)
          DOL_SLAB_STEP(1, I1, I2, I0, G1a, G1b, G0a, G0b)
          DOL_SLAB_STEP(2, I2, I0, I1, G0a, G0b, G1a, G1b)
          DOL_SLAB_STEP(3, I0, I1, I2, G1a, G1b, G0a, G0b)
          DOL_SLAB_STEP(4, I1, I2, I0, G0a, G0b, G1a, G1b)
          DOL_SLAB_STEP(5, I2, I0, I1, G1a, G1b, G0a, G0b)
          jb += 6;
          nbr -= 6;
          pb += 96;
        }
#undef DOL_SLAB_STEP
      stream_done:
        vset(r, a);
        continue;
      }
      auto step2 = [&](f4 a, const I4& p, const I4& q) {  // four entries: p's pair, then q's
        const f4 x0 = gather(p.o0), x1 = gather(p.o1), x2 = gather(q.o0), x3 = gather(q.o1);
        if constexpr (PROBE == 5) return a + x0 + x1 + x2 + x3;
        a = fmac(a, __int_as_float(p.w0), x0);
        a = fmac(a, __int_as_float(p.w1), x1);
        a = fmac(a, __int_as_float(q.w0), x2);
        return fmac(a, __int_as_float(q.w1), x3);
      };
      I4 fa = pair_at(ibase + uint32_t(bnd[0]) * 8), fb = pair_at(ibase + uint32_t(bnd[0]) * 8 + 16);
#pragma unroll
      for (int r = 0; r < kRW; ++r) {
        int np = (bnd[r + 1] - bnd[r]) >> 1;  // pairs of row r in this chunk
        I4 qa = fa, qb = fb;
        if (r + 1 < kRW) {  // the next row's first two pairs
          const uint32_t nx = ibase + uint32_t(bnd[r + 1]) * 8;
          fa = pair_at(nx);
          fb = pair_at(nx + 16);
        }
        uint32_t ip = ibase + uint32_t(bnd[r]) * 8 + 32;  // the pair after qb
        f4 a = acc[r];
        while (np >= 4) {
          const I4 na = PROBE == 4 ? qb : pair_at(ip), nb = PROBE == 4 ? qa : pair_at(ip + 16);
          a = step2(a, qa, qb);
          // qa / qb are free once this step's products are summed: reload them
          // only then, into the same registers (a hoisted reload needs fresh
          // registers and a copy back at the loop end)
          asm volatile("" : "+v"(a)::"memory");
          if constexpr (PROBE != 4) {
            qa = pair_at(ip + 32);
            qb = pair_at(ip + 48);
          }
          ip += 64;
          a = step2(a, na, nb);
          asm volatile("" : "+v"(a)::"memory");
          np -= 4;
        }
        if constexpr (PROBE == 6) {  // diagnostics: a row's np % 4 tail pairs skipped
          acc[r] = a;
          continue;
        }
        if constexpr (A4) {  // np % 4 is 0 or 2 (segments of whole pairs of pairs)
          if (np >= 2) a = step2(a, qa, qb);
          acc[r] = a;
          continue;
        }
        if (np >= 2) {
          I4 na;
          if (np == 3) na = pair_at(ip);
          a = step2(a, qa, qb);
          if (np == 3) {
            a = fmac(a, __int_as_float(na.w0), gather(na.o0));
            a = fmac(a, __int_as_float(na.w1), gather(na.o1));
          }
        } else if (np == 1) {
          a = fmac(a, __int_as_float(qa.w0), gather(qa.o0));
          a = fmac(a, __int_as_float(qa.w1), gather(qa.o1));
        }
        acc[r] = a;
      }
    }
    const int64_t p = SA ? cur.slab * kCols + lane * 4 : cur.p;
    if (p < P) {
      const int32_t* pr = perm + int64_t(cur.rg) * kRows + row0;
#pragma unroll
      for (int r = 0; r < kRW; ++r) {
        const int row = pr[r];  // this wave's slot r holds output row `row` (-1: none)
        const f4 v = SV ? vget(r) : acc[r];
        if (row >= 0) {
          float* y = Y + int64_t(row) * ldy + p;
          if (p + 4 <= P) {
            __builtin_nontemporal_store(v, reinterpret_cast<f4*>(y));
          } else {
            for (int c = 0; c < int(P - p); ++c) y[c] = v[c];
          }
        }
      }
    }
    if (!has_next) break;
#pragma unroll
    for (int r = 0; r < kRW; ++r) acc[r] = f4{0.f, 0.f, 0.f, 0.f};
    accv = 0.f;
    t += G;
    cur = nxt;
    nxt = nn;
    has_next = has_nn;
  }
}

// ---------------------------------------------------------------------------
// Dense W -> CSR (+ chunk starts) on the device, for a W drawn every round.
// Selection rule of Neighbors (DIST/simulators.py:91-97): W_ij > 0 (NaN and
// <= 0 dropped), j ascending.
// ---------------------------------------------------------------------------
constexpr int kRowThreads = 256;

__global__ __launch_bounds__(kRowThreads) void dense_count_kernel(const float* __restrict__ W, int64_t ldw, int n_cols,
                                                                  int32_t* __restrict__ rowptr) {
  __shared__ int part[kRowThreads / 64];
  const float* row = W + int64_t(blockIdx.x) * ldw;
  int c = 0;
  for (int j = threadIdx.x; j < n_cols; j += kRowThreads) c += row[j] > 0.f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < kRowThreads / 64; ++w) t += part[w];
    rowptr[blockIdx.x + 1] = t;
  }
}

// in-place inclusive scan of rowptr[1..n] (one workgroup), rowptr[0] = 0
__global__ __launch_bounds__(1024) void rowptr_scan_kernel(int32_t* __restrict__ rowptr, int n) {
  __shared__ int wsum[16];
  __shared__ int carry;
  if (threadIdx.x == 0) {
    carry = 0;
    rowptr[0] = 0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int base = 0; base < n; base += 1024) {
    const int i = base + int(threadIdx.x);
    int v = i < n ? rowptr[i + 1] : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {  // inclusive wave scan
      const int t = __shfl_up(v, o);
      if (lane >= o) v += t;
    }
    if (lane == 63) wsum[w] = v;
    __syncthreads();
    int off = carry;
    for (int q = 0; q < w; ++q) off += wsum[q];
    if (i < n) rowptr[i + 1] = v + off;
    __syncthreads();
    if (threadIdx.x == 1023) carry = v + off;
    __syncthreads();
  }
}

__global__ __launch_bounds__(kRowThreads) void dense_fill_kernel(const float* __restrict__ W, int64_t ldw, int n_cols,
                                                                 const int32_t* __restrict__ rowptr,
                                                                 int32_t* __restrict__ col, float* __restrict__ val) {
  __shared__ int wcnt[kRowThreads / 64];
  const int r = blockIdx.x;
  const float* row = W + int64_t(r) * ldw;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int run = rowptr[r];
  for (int t0 = 0; t0 < n_cols; t0 += kRowThreads) {
    const int j = t0 + int(threadIdx.x);
    const float v = j < n_cols ? row[j] : 0.f;
    const bool keep = v > 0.f;
    const uint64_t m = __ballot(keep);
    const int below = __popcll(m & ((uint64_t(1) << lane) - 1));
    if (lane == 0) wcnt[w] = __popcll(m);
    __syncthreads();
    int off = run;
    for (int q = 0; q < w; ++q) off += wcnt[q];
    if (keep) {
      col[off + below] = j;
      val[off + below] = v;
    }
    for (int q = w; q < kRowThreads / 64; ++q) off += wcnt[q];
    run = off;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Chunk-major packing of a device CSR (dol_csr_slab_pack).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lower_bound_col(const int32_t* __restrict__ col, int lo, int hi, int key) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (col[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// hdr[g][k][i] <- number of row (g R + i)'s entries in chunk k (0 for i == R and rows past n_rows)
__global__ __launch_bounds__(256) void slab_count_kernel(const int32_t* __restrict__ rowptr,
                                                         const int32_t* __restrict__ col, int n_rows, int nk,
                                                         int64_t len, int32_t* __restrict__ hdr, int align) {
  const int64_t idx = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (idx >= len) return;
  const int i = int(idx % (kRows + 1));
  const int64_t gk = idx / (kRows + 1);
  const int k = int(gk % nk), g = int(gk / nk);
  const int r = g * kRows + i;
  int c = 0;
  if (i < kRows && r < n_rows) {
    const int e0 = rowptr[r], e1 = rowptr[r + 1];
    const int lo = lower_bound_col(col, e0, e1, k * kChunk);
    c = lower_bound_col(col, lo, e1, (k + 1) * kChunk) - lo;
  }
  hdr[idx] = (c + align - 1) / align * align;  // segments padded to a multiple of `align` (2 or 4)
}

// in-place exclusive scan of hdr[0..len) (one workgroup: a contiguous segment per thread)
__global__ __launch_bounds__(1024) void slab_scan_kernel(int32_t* __restrict__ hdr, int64_t len) {
  __shared__ int wsum[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t seg = (len + 1023) / 1024;
  const int64_t b0 = min(len, int64_t(t) * seg), b1 = min(len, b0 + seg);
  int s = 0;
  int64_t j = b0;
  for (; j + 8 <= b1; j += 8) {  // eight independent loads per round trip
    int v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = hdr[j + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; j < b1; ++j) s += hdr[j];
  int v = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  if (lane == 63) wsum[w] = v;
  __syncthreads();
  int off = v - s;
  for (int q = 0; q < w; ++q) off += wsum[q];
  j = b0;
  for (; j + 8 <= b1; j += 8) {
    int v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = hdr[j + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      hdr[j + u] = off;
      off += v[u];
    }
  }
  for (; j < b1; ++j) {
    const int c = hdr[j];
    hdr[j] = off;
    off += c;
  }
}

// Row balancing (one wave per row group).  The mix kernel syncs its 16 waves
// once per chunk, so a chunk costs the wave with the most entries in it; with
// rows dealt to waves in index order the per-chunk maxima run ~22 % above the
// mean at p = 0.1.  Greedy vector packing: rows by total entries (descending,
// ties by index), each to the wave with < kRW rows whose chunk loads grow the
// least in sum of squares, sum_k c_k (2 L_wk + c_k) (ties: lowest wave).  A
// row's sum order is untouched (its entries keep their ascending-column
// order), so the output bits are the same for any assignment.  In: hdr[g][k][i]
// = padded entry count of row g R + i in chunk k (natural order).  Out: the
// same counts in slot order (slot = wave * kRW + position), perm[g][slot] =
// output row (-1: none), inv[g R + i] = slot.  nk > kBalMaxNk (x_rows > 32768)
// or DOL_SLAB_BALANCE = 0: slots in row order.
constexpr int kBalMaxNk = 512;
__global__ __launch_bounds__(64) void slab_balance_kernel(int32_t* __restrict__ hdr, int n_rows, int nk,
                                                          int32_t* __restrict__ perm, int32_t* __restrict__ inv,
                                                          int balance) {
  extern __shared__ __attribute__((aligned(16))) uint8_t bl[];
  int* L = reinterpret_cast<int*>(bl);                  // [kWaves][nk] wave loads
  int* tot = L + kWaves * nk;                           // [kRows] row totals, then order
  int* slot_of = tot + kRows;                           // [kRows]
  uint8_t* c = reinterpret_cast<uint8_t*>(slot_of + kRows);  // [kRows][nk] counts (<= kChunk)
  const int g = blockIdx.x, lane = threadIdx.x;
  if (!balance) {  // slots in row order: the counts are already in slot order
    for (int i = lane; i < kRows; i += 64) {
      const int r = g * kRows + i;
      perm[int64_t(g) * kRows + i] = r < n_rows ? r : -1;
      if (r < n_rows) inv[r] = i;
    }
    return;
  }
  int32_t* H = hdr + int64_t(g) * nk * (kRows + 1);
  // counts of rows lane and lane + 64, eight chunks' loads in flight at a time
  // (one dependent global load per element cost ~0.1 ms per pack)
  static_assert(kRows == 128, "two rows per lane");
  int t0 = 0, t1 = 0;
  for (int k0 = 0; k0 < nk; k0 += 8) {
    int v0[8], v1[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int32_t* h = H + int64_t(min(k0 + u, nk - 1)) * (kRows + 1);
      v0[u] = h[lane];
      v1[u] = h[lane + 64];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (k0 + u < nk) {
        c[lane * nk + k0 + u] = uint8_t(v0[u]);
        c[(lane + 64) * nk + k0 + u] = uint8_t(v1[u]);
        t0 += v0[u];
        t1 += v1[u];
      }
  }
  tot[lane] = t0;
  tot[lane + 64] = t1;
  for (int j = lane; j < kWaves * nk; j += 64) L[j] = 0;
  __syncthreads();
  {
    int rk[2];
    for (int h = 0; h < 2; ++h) {
      const int i = lane + 64 * h, ti = tot[i];
      int r = 0;
      for (int j = 0; j < kRows; ++j) {
        const int tj = tot[j];
        r += (tj > ti) | ((tj == ti) & (j < i));
      }
      rk[h] = r;
    }
    __syncthreads();
    tot[rk[0]] = lane;  // tot becomes order[]: rows by rank
    tot[rk[1]] = lane + 64;
    __syncthreads();
    const int w = lane & (kWaves - 1), q = lane >> 4;  // this lane: wave w, chunks k = q mod 4
    int filled = 0;                                    // rows dealt to wave w
    for (int s = 0; s < kRows; ++s) {
      const int i = tot[s];
      const uint8_t* ci = c + i * nk;
      int part = 0;
      for (int k = q; k < nk; k += 4) {
        const int ck = ci[k];
        part += ck * (2 * L[w * nk + k] + ck);
      }
      part += __shfl_xor(part, 16);
      part += __shfl_xor(part, 32);
      int64_t key = filled < kRW ? (int64_t(part) << 4) | w : INT64_MAX;
#pragma unroll
      for (int o = 1; o < kWaves; o <<= 1) {
        const int64_t other = __shfl_xor(key, o);
        key = other < key ? other : key;
      }
      const int wb = int(key & (kWaves - 1));
      if (w == wb) {
        for (int k = q; k < nk; k += 4) L[w * nk + k] += ci[k];
      }
      if (lane == wb) slot_of[i] = wb * kRW + filled;
      filled += (w == wb);
      __syncthreads();
    }
  }
  __syncthreads();
  for (int i = lane; i < kRows; i += 64) {
    const int r = g * kRows + i, sl = slot_of[i];
    perm[int64_t(g) * kRows + sl] = r < n_rows ? r : -1;
    if (r < n_rows) inv[r] = sl;
  }
  for (int h = 0; h < 2; ++h) {
    const int i = lane + 64 * h, sl = slot_of[i];
    for (int k = 0; k < nk; ++k) H[int64_t(k) * (kRows + 1) + sl] = c[i * nk + k];
  }
}

// The same greedy packing for nk <= NKM (x_rows <= 64 NKM) with the wave loads
// in registers: lanes 0..15 are the 16 waves, each holding its NKM chunk loads,
// so a step is one LDS read of the row's counts (four per word), the sums of
// squares in registers, a DPP min over the 16 lanes and one update -- no
// barrier, no LDS round trip for the loads.  The row order and the keys
// ((part << 4) | wave, smallest wins) are slab_balance_kernel's: same slots.
template <int NKM>
__global__ __launch_bounds__(64) void slab_balance_reg_kernel(int32_t* __restrict__ hdr, int n_rows, int nk,
                                                              int32_t* __restrict__ perm, int32_t* __restrict__ inv) {
  static_assert(NKM % 4 == 0 && kRows == 128 && kWaves == 16, "layout");
  __shared__ __attribute__((aligned(16))) uint8_t c[kRows * NKM];  // counts, row-major, zero past nk
  __shared__ int tot[kRows];                                      // row totals, then the order
  __shared__ int slot_of[kRows];
  const int g = blockIdx.x, lane = threadIdx.x;
  int32_t* H = hdr + int64_t(g) * nk * (kRows + 1);
  int t0 = 0, t1 = 0;
#pragma unroll
  for (int k0 = 0; k0 < NKM; k0 += 8) {
    int v0[8], v1[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int32_t* h = H + int64_t(min(k0 + u, nk - 1)) * (kRows + 1);
      v0[u] = k0 + u < nk ? h[lane] : 0;
      v1[u] = k0 + u < nk ? h[lane + 64] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      c[lane * NKM + k0 + u] = uint8_t(v0[u]);
      c[(lane + 64) * NKM + k0 + u] = uint8_t(v1[u]);
      t0 += v0[u];
      t1 += v1[u];
    }
  }
  tot[lane] = t0;
  tot[lane + 64] = t1;
  __syncthreads();
  int rk0 = 0, rk1 = 0;
  for (int j = 0; j < kRows; ++j) {
    const int tj = tot[j];
    rk0 += (tj > t0) | ((tj == t0) & (j < lane));
    rk1 += (tj > t1) | ((tj == t1) & (j < lane + 64));
  }
  __syncthreads();
  tot[rk0] = lane;  // tot becomes order[]: rows by rank
  tot[rk1] = lane + 64;
  __syncthreads();
  const int w = lane & (kWaves - 1);
  const int ord0 = tot[lane], ord1 = tot[lane + 64];  // the order in registers (lane s % 64)
  int L[NKM];
#pragma unroll
  for (int k = 0; k < NKM; ++k) L[k] = 0;
  int filled = 0;
  // the counts of step s + 1's row are read while step s decides (the order
  // does not depend on the decisions)
  auto row_words = [&](int s, uint32_t (&wd)[NKM / 4]) {
    const int i = __builtin_amdgcn_readlane(s < 64 ? ord0 : ord1, s & 63);
    const uint32_t* cw = reinterpret_cast<const uint32_t*>(c + i * NKM);
#pragma unroll
    for (int q = 0; q < NKM / 4; ++q) wd[q] = cw[q];
    return i;
  };
  uint32_t wnext[NKM / 4];
  int inext = row_words(0, wnext);
  for (int s = 0; s < kRows; ++s) {
    const int i = inext;
    uint32_t words[NKM / 4];
#pragma unroll
    for (int q = 0; q < NKM / 4; ++q) words[q] = wnext[q];
    if (s + 1 < kRows) inext = row_words(s + 1, wnext);
    int part = 0;
#pragma unroll
    for (int k = 0; k < NKM; ++k) {
      const int ck = int((words[k >> 2] >> (8 * (k & 3))) & 255u);
      part += ck * (2 * L[k] + ck);
    }
    int key = (lane < kWaves && filled < kRW) ? (part << 4) | w : INT32_MAX;
    // min over lanes 0..15 (one DPP row): shifts in from outside the row read INT32_MAX
    key = min(key, __builtin_amdgcn_update_dpp(INT32_MAX, key, 0x111, 0xf, 0xf, false));  // row_shr:1
    key = min(key, __builtin_amdgcn_update_dpp(INT32_MAX, key, 0x112, 0xf, 0xf, false));  // row_shr:2
    key = min(key, __builtin_amdgcn_update_dpp(INT32_MAX, key, 0x114, 0xf, 0xf, false));  // row_shr:4
    key = min(key, __builtin_amdgcn_update_dpp(INT32_MAX, key, 0x118, 0xf, 0xf, false));  // row_shr:8
    const int wb = __builtin_amdgcn_readlane(key, kWaves - 1) & (kWaves - 1);
    if (lane == wb) {
#pragma unroll
      for (int k = 0; k < NKM; ++k) L[k] += int((words[k >> 2] >> (8 * (k & 3))) & 255u);
      slot_of[i] = wb * kRW + filled;
      ++filled;
    }
  }
  __syncthreads();
  for (int h = 0; h < 2; ++h) {
    const int i = lane + 64 * h, r = g * kRows + i, sl = slot_of[i];
    perm[int64_t(g) * kRows + sl] = r < n_rows ? r : -1;
    if (r < n_rows) inv[r] = sl;
    for (int k = 0; k < nk; ++k) H[int64_t(k) * (kRows + 1) + sl] = c[i * NKM + k];
  }
}

// one wave per row: entries to their chunk-major slots as (LDS byte offset,
// weight bits); then, per chunk with an odd count, a (0, 0) pad entry closes the
// segment and bit 0 of the segment's header word is set
__global__ __launch_bounds__(64) void slab_scatter_kernel(const int32_t* __restrict__ rowptr,
                                                          const int32_t* __restrict__ col,
                                                          const float* __restrict__ val, int nk,
                                                          const int32_t* __restrict__ inv,
                                                          int32_t* __restrict__ hdr, int32_t* __restrict__ ent,
                                                          int align) {
  const int r = blockIdx.x, g = r / kRows, i = inv[r];
  const int e0 = rowptr[r], e1 = rowptr[r + 1];
  for (int e = e0 + int(threadIdx.x); e < e1; e += 64) {
    const int c = col[e], k = c / kChunk;
    const int first = lower_bound_col(col, e0, e1, k * kChunk);
    const int64_t dst = hdr[(int64_t(g) * nk + k) * (kRows + 1) + i] + (e - first);
    const int64_t q = (dst >> 1) * 4 + 2 * (dst & 1);  // pair layout (w0, off0, w1, off1)
    ent[q] = __float_as_int(val[e]);
    ent[q + 1] = (c % kChunk) * (kCols * 4);
  }
  __syncthreads();  // every header read above is done before the pad bits change them
  for (int k = int(threadIdx.x); k < nk; k += 64) {
    const int lo = lower_bound_col(col, e0, e1, k * kChunk);
    const int n = lower_bound_col(col, lo, e1, (k + 1) * kChunk) - lo;
    const int np = (n + align - 1) / align * align;
    if (np > n) {
      int32_t* h = hdr + (int64_t(g) * nk + k) * (kRows + 1) + i;
      for (int64_t pad = *h + n; pad < *h + np; ++pad) {  // (0, zero piece) entries up to the alignment
        const int64_t q = (pad >> 1) * 4 + 2 * (pad & 1);
        ent[q] = 0;
        ent[q + 1] = kZeroRel;
      }
      *h |= 1;
    }
  }
}

// kTailPad pad entries (weight 0, the zero piece) right after the last block:
// the stream kernel reads up to two pairs past a wave's run, and past the last
// block ent is otherwise unwritten.  hdr[blocks - 1] (the last group's
// terminator slot, count 0) holds the total after the exclusive scan.
constexpr int kTailPad = 8;
__global__ void slab_tail_kernel(const int32_t* __restrict__ hdr, int64_t blocks, int32_t* __restrict__ ent) {
  const int64_t total = hdr[blocks - 1];
  const int t = threadIdx.x;
  if (t < kTailPad) {
    const int64_t e = total + t;
    const int64_t q = (e >> 1) * 4 + 2 * (e & 1);
    ent[q] = 0;
    ent[q + 1] = kZeroRel;
  }
}
static_assert(kTailPad <= kEntPad, "the tail pads fit the entry slack");

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// kernel of dol_mix_csr_slab_f32 (dol_slab_set_variant): 0 = the process
// default (DOL_SLAB_KERNEL, else the asm stream), 1 = row loop (r03),
// 2 = pipelined stream (r06), 3 = the stream hand-scheduled (asm; rows of
// 2^30 floats and more run variant 2).  Atomic: thread-compatible like the
// other setters.
std::atomic<int> g_slab_variant{0};
int slab_default_variant() {
  static const int v = [] {
    const char* e = getenv("DOL_SLAB_KERNEL");
    const int x = e ? atoi(e) : 3;
    return (x == 1 || x == 2) ? x : 3;
  }();
  return v;
}

// segment alignment of the packing and the kernel variant that reads it (one
// value per process): 2 = pairs; 4 = pairs of pairs, so a row's tail is at most
// one 2-pair step (DOL_SLAB_ALIGN)
int slab_align() {
  static const int a = [] { const char* e = getenv("DOL_SLAB_ALIGN"); return (e && atoi(e) == 4) ? 4 : 2; }();
  return a;
}

}  // namespace

extern "C" int dol_slab_set_variant(int32_t variant) {
  if (variant < 0 || variant > 3)
    return dol::fail(DOL_EINVAL,
                     "dol_slab_set_variant: variant %d outside 0 (default) / 1 (row loop) / 2 (stream) / 3 (stream, asm)",
                     variant);
  const int prev = g_slab_variant.exchange(variant, std::memory_order_relaxed);
  dol::g_err[0] = '\0';
  return prev;
}

extern "C" int dol_csr_slab_nk(int32_t x_rows) { return x_rows <= 0 ? 0 : int((int64_t(x_rows) + kChunk - 1) / kChunk); }
extern "C" int64_t dol_csr_slab_hdr_len(int32_t n_rows, int32_t x_rows) {
  if (n_rows <= 0 || x_rows <= 0) return 0;
  const int64_t n_rg = cdiv(n_rows, kRows);
  return n_rg * dol_csr_slab_nk(x_rows) * (kRows + 1) + n_rg * kRows + n_rg * kRows;  // blocks, perm, inv
}
extern "C" int64_t dol_csr_slab_ent_len(int64_t nnz_cap, int32_t n_rows, int32_t x_rows) {
  if (nnz_cap < 0 || nnz_cap > dol::kMaxDim || n_rows < 0 || x_rows < 0) return 0;
  return 2 * (nnz_cap + 3 * int64_t(n_rows) * dol_csr_slab_nk(x_rows) + kEntPad);  // + <= 3 pads per (row, chunk)
}

extern "C" int dol_mix_csr_slab_f32(const float* X, int64_t ldx, int32_t x_rows, float* Y, int64_t ldy,
                                    int32_t n_rows, int64_t P, const int32_t* ent, const int32_t* hdr,
                                    hipStream_t s) {
  DOL_DIMS_OK("dol_mix_csr_slab_f32", ldx, ldy, P);
  using dol::fail;
  if (n_rows < 0 || x_rows < 0 || P < 0) return fail(DOL_EINVAL, "dol_mix_csr_slab_f32: negative size");
  if (n_rows == 0 || P == 0) return DOL_OK;
  if (x_rows == 0) return fail(DOL_EINVAL, "dol_mix_csr_slab_f32: x_rows == 0");
  if (!X || !Y || !ent || !hdr) return fail(DOL_EINVAL, "dol_mix_csr_slab_f32: null pointer");
  if (X == Y) return fail(DOL_EINVAL, "dol_mix_csr_slab_f32: X and Y alias");
  const int64_t p4 = (P + 3) / 4 * 4;
  if (ldx % 4 || ldy % 4 || ldx < p4 || ldy < P)
    return fail(DOL_EINVAL, "dol_mix_csr_slab_f32: need ldx, ldy multiples of 4, ldx >= round_up(P, 4), ldy >= P");
  if (reinterpret_cast<uintptr_t>(X) % 16 || reinterpret_cast<uintptr_t>(Y) % 16 ||
      reinterpret_cast<uintptr_t>(ent) % 16)
    return fail(DOL_EINVAL, "dol_mix_csr_slab_f32: X, Y and ent must be 16-B aligned");
  const int nk = dol_csr_slab_nk(x_rows);
  const int64_t n_rg = cdiv(n_rows, kRows);
  const int64_t n_slabs = cdiv(P, kCols);
  const int64_t n_items = 8 * cdiv(n_slabs, 8) * n_rg;
  if (n_items >= (int64_t(1) << 32)) return fail(DOL_EINVAL, "dol_mix_csr_slab_f32: too many workgroups");
  static const int probe = [] { const char* e = getenv("DOL_SLAB_PROBE"); return e ? atoi(e) : 0; }();
  // persistent grid (one workgroup per CU, a multiple of 8) unless DOL_SLAB_PERSIST=0
  // or a single chunk (x_rows <= 64: the stream needs nk >= 2)
  static const int persist = [] { const char* e = getenv("DOL_SLAB_PERSIST"); return e ? atoi(e) : 1; }();
  static const int n_cu = [] {
    int dev = 0, cu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cu = 0;
    return cu;
  }();
  const int64_t g_cap = int64_t(n_cu) / 8 * 8;
  const int64_t grid = (persist && nk >= 2 && g_cap >= 8) ? std::min<int64_t>(n_items, g_cap) : n_items;
  auto launch = [&](auto kern) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(grid)), dim3(kThreads), kLds, s, X, ldx, x_rows, Y, ldy,
                       n_rows, P, ent, hdr, nk, static_cast<int>(n_rg), n_slabs, n_items);
  };
  if (probe == 1) launch(csr_slab_kernel<1>);
  else if (probe == 2) launch(csr_slab_kernel<2>);
  else if (probe == 3) launch(csr_slab_kernel<3>);
  else if (probe == 4) launch(csr_slab_kernel<4>);
  else if (probe == 5) launch(csr_slab_kernel<5>);
  else if (probe == 6) launch(csr_slab_kernel<6>);
  else if (probe == 7) launch(csr_slab_kernel<3, false, 2>);  // the asm stream without the chunk barrier (timing bound; wrong bits)
  else if (slab_align() == 4) launch(csr_slab_kernel<0, true>);
  else {
    int v = g_slab_variant.load(std::memory_order_relaxed);
    if (v == 0) v = slab_default_variant();
    if (v == 2) launch(csr_slab_kernel<0, false, 1>);
    else if (v == 3 && p4 * 4 < (int64_t(1) << 32)) launch(csr_slab_kernel<0, false, 2>);  // 32-bit column offsets
    else if (v == 3) launch(csr_slab_kernel<0, false, 1>);
    else launch(csr_slab_kernel<0>);
  }
  return dol::check_launch("dol_mix_csr_slab_f32");
}

extern "C" int dol_csr_slab_pack(const int32_t* rowptr, const int32_t* col, const float* val, int32_t n_rows,
                                 int32_t x_rows, int32_t balance, int32_t* ent, int32_t* hdr, hipStream_t s) {
  using dol::fail;
  if (n_rows < 0 || x_rows < 0) return fail(DOL_EINVAL, "dol_csr_slab_pack: negative size");
  if (n_rows == 0 || x_rows == 0) return DOL_OK;
  if (!rowptr || !ent || !hdr) return fail(DOL_EINVAL, "dol_csr_slab_pack: null pointer");
  const int nk = dol_csr_slab_nk(x_rows);
  const int64_t len = cdiv(n_rows, kRows) * nk * (kRows + 1);  // the header blocks
  if (cdiv(len, 256) >= (int64_t(1) << 31)) return fail(DOL_EINVAL, "dol_csr_slab_pack: too many chunk blocks");
  hipLaunchKernelGGL(slab_count_kernel, dim3(static_cast<unsigned>(cdiv(len, 256))), dim3(256), 0, s, rowptr, col,
                     n_rows, nk, len, hdr, slab_align());
  const int64_t n_rg = cdiv(n_rows, kRows);
  const int64_t blocks = n_rg * nk * (kRows + 1);  // the header blocks; perm and inv follow
  int32_t* perm = hdr + blocks;
  int32_t* inv = perm + n_rg * kRows;
  const int bal = balance && nk <= kBalMaxNk;  // beyond: slots in row order
  const size_t bal_lds = bal ? size_t(kWaves) * nk * 4 + 2 * kRows * 4 + size_t(kRows) * nk : 16;
  if (bal && nk <= 16)
    hipLaunchKernelGGL(slab_balance_reg_kernel<16>, dim3(static_cast<unsigned>(n_rg)), dim3(64), 0, s, hdr, n_rows, nk,
                       perm, inv);
  else if (bal && nk <= 64)
    hipLaunchKernelGGL(slab_balance_reg_kernel<64>, dim3(static_cast<unsigned>(n_rg)), dim3(64), 0, s, hdr, n_rows, nk,
                       perm, inv);
  else {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(slab_balance_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bal_lds));
    hipLaunchKernelGGL(slab_balance_kernel, dim3(static_cast<unsigned>(n_rg)), dim3(64), bal_lds, s, hdr, n_rows, nk,
                       perm, inv, bal);
  }
  hipLaunchKernelGGL(slab_scan_kernel, dim3(1), dim3(1024), 0, s, hdr, blocks);
  hipLaunchKernelGGL(slab_scatter_kernel, dim3(static_cast<unsigned>(n_rows)), dim3(64), 0, s, rowptr, col, val, nk,
                     inv, hdr, ent, slab_align());
  hipLaunchKernelGGL(slab_tail_kernel, dim3(1), dim3(64), 0, s, hdr, blocks, ent);
  return dol::check_launch("dol_csr_slab_pack");
}

extern "C" int dol_dense_to_csr_f32(const float* W, int64_t ldw, int32_t n_rows, int32_t n_cols, int32_t* rowptr,
                                    int32_t* col, float* val, int64_t cap, hipStream_t s) {
  DOL_DIMS_OK("dol_dense_to_csr_f32", ldw, cap);
  using dol::fail;
  if (n_rows < 0 || n_cols < 0) return fail(DOL_EINVAL, "dol_dense_to_csr_f32: negative size");
  if (!rowptr) return fail(DOL_EINVAL, "dol_dense_to_csr_f32: null rowptr");
  if (int64_t(n_rows) * n_cols > int64_t(INT32_MAX)) return fail(DOL_EINVAL, "dol_dense_to_csr_f32: n_rows * n_cols >= 2^31");
  if (n_rows > 0 && n_cols > 0 && (!W || !col || !val)) return fail(DOL_EINVAL, "dol_dense_to_csr_f32: null pointer");
  if (n_rows > 0 && n_cols > 0 && ldw < n_cols) return fail(DOL_EINVAL, "dol_dense_to_csr_f32: ldw < n_cols");
  if (cap < int64_t(n_rows) * n_cols)
    return fail(DOL_EINVAL, "dol_dense_to_csr_f32: col/val capacity %lld < n_rows * n_cols", static_cast<long long>(cap));
  if (n_rows == 0) return hipMemsetAsync(rowptr, 0, 4, s) == hipSuccess ? DOL_OK : fail(DOL_EINVAL, "memset failed");
  if (n_cols == 0)
    return hipMemsetAsync(rowptr, 0, (int64_t(n_rows) + 1) * 4, s) == hipSuccess ? DOL_OK
           : fail(DOL_EINVAL, "dol_dense_to_csr_f32: memset failed");
  hipLaunchKernelGGL(dense_count_kernel, dim3(n_rows), dim3(kRowThreads), 0, s, W, ldw, n_cols, rowptr);
  hipLaunchKernelGGL(rowptr_scan_kernel, dim3(1), dim3(1024), 0, s, rowptr, n_rows);
  hipLaunchKernelGGL(dense_fill_kernel, dim3(n_rows), dim3(kRowThreads), 0, s, W, ldw, n_cols, rowptr, col, val);
  return dol::check_launch("dol_dense_to_csr_f32");
}
