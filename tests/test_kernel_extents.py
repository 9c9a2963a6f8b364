"""Host restatement of the launch geometry and indexing of the bank kernels on
the path of the r04 GPU memory fault (profiles/r04k_vmm_fault.txt: the
config-3 DGD rounds of tools/bench_configs.py on exact-size mapped blocks),
computing the lowest and highest element each launch touches in each buffer
and checking it against the buffer's extent [0, rows * ld).  With torch's
caching allocator an overrun lands in slack; with a dol_bank_alloc block
mapped to exactly rows * ld * 4 bytes (rounded to the 2 MiB granularity) it
faults, so every kernel must stay inside its rows.

Restated (csrc/dol_hip.hip, function and index expressions named per case):
  * ring_mix_dma_kernel<4, DgdEpi, NTI> -- the ring DGD round's float4 body
    (mix_ring_impl: grid nct * cdiv(n, 4)); R + 2 row loads per block at
    min(r0 - 1 + k, r1) through row() (halo pointers below 0 / from n), the
    epilogue's target / momentum loads at min(r0 + k, r1 - 1), stores r < r1;
  * ring_mix_kernel<float, 4> -- the same round's P % 4 tail columns;
  * ring_edges_kernel -- rows 0 and n - 1 of a sharded block;
  * csr_xcd_kernel<32, 2, DgdEpi> -- the random-regular DGD round (mix_csr_impl
    from 512 rows), rows clamped to n - 1 on the degree-4 fast path;
  * csr_mix_kernel<f4 / float, 16> -- the columns the XCD kernel leaves over;
  * ring_stream_dma_kernel<S, 8, 8> -- FedLCon's eps pass (variants 3-5): the
    DMA walks wrap(r0 - S ..) and stays on the tile's last input row past the
    end; its buffer stores are bounded by a per-row descriptor of ldy * 4 bytes.
Every case runs at the geometry of the fault (1024 x 2^20, ld = 2^20 + 2048,
momentum), at 8192 x 2^20 and at ragged shapes (P % 4 != 0, n not a multiple
of the tile height, fewer rows than one tile).
Reference semantics these kernels implement: DIST/clients.py:61-69
(consensus), DIST/simulators.py:147-162 (the DGD round order),
DIST/simulators.py:190-196 (FedLCon's eps rounds)."""
import numpy as np
import pytest

from dolhip import graph as G
from dolhip.bank import row_stride

KT = 256  # kThreads


def cdiv(a, b):
    return -(-a // b)


class Ext:
    """[lo, hi] element offsets touched per buffer."""

    def __init__(self):
        self.r = {}

    def add(self, buf, lo, hi):
        lo, hi = int(np.min(lo)), int(np.max(hi))
        a, b = self.r.get(buf, (lo, hi))
        self.r[buf] = (min(a, lo), max(b, hi))

    def check(self, sizes):
        for buf, (lo, hi) in self.r.items():
            assert lo >= 0, f"{buf}: touches element {lo} < 0"
            assert hi < sizes[buf], f"{buf}: touches element {hi} >= its extent {sizes[buf]}"


def split_cols(P):
    return P // 4, P % 4  # n4, tail (vec_ok: 16-B aligned rows, ld % 4 == 0)


def _row_ptr(r, n, wrap_halos):
    """row() of the ring kernels: (buffer, row) of logical row r in [-1, n]."""
    if r < 0:
        return ("X", n - 1) if wrap_halos else ("HP", 0)
    if r >= n:
        return ("X", 0) if wrap_halos else ("HN", 0)
    return ("X", r)


def _add_rows(e, r, n, ld, c_lo, c_hi, wrap_halos):
    """Loads through row(r) for arrays of logical rows r and f4 column ranges."""
    r = np.asarray(r, np.int64)
    inside = (r >= 0) & (r < n)
    if inside.any():
        e.add("X", (r[inside] * ld + 4 * c_lo[inside]), (r[inside] * ld + 4 * c_hi[inside] + 3))
    for mask, wrap_row, halo in ((r < 0, n - 1, "HP"), (r >= n, 0, "HN")):
        if mask.any():
            if wrap_halos:
                e.add("X", wrap_row * ld + 4 * c_lo[mask], wrap_row * ld + 4 * c_hi[mask] + 3)
            else:
                e.add(halo, 4 * c_lo[mask], 4 * c_hi[mask] + 3)


def ring_dma_extents(n, P, ld, mode, wrap_halos=True, R=4):
    """mix_ring_impl -> ring_mix_dma_kernel<R, DgdEpi<*, mode>, NTI> + the float tail."""
    e = Ext()
    n4, tail = split_cols(P)
    if n4:
        nct = cdiv(n4, KT)
        b = np.arange(nct * cdiv(n, R), dtype=np.int64)
        ct, r0 = b % nct, (b // nct) * R
        r1 = np.minimum(r0 + R, n)
        c_lo, c_hi = ct * KT, np.minimum(ct * KT + KT - 1, n4 - 1)  # lanes with c < ncols_v
        live = c_lo < n4
        ct, r0, r1, c_lo, c_hi = ct[live], r0[live], r1[live], c_lo[live], c_hi[live]
        for k in range(R + 2):  # DMA rows min(r0 - 1 + k, r1) through row()
            _add_rows(e, np.minimum(r0 - 1 + k, r1), n, ld, c_lo, c_hi, wrap_halos)
        for k in range(R):
            r = np.minimum(r0 + k, r1 - 1)  # epilogue operands ride with the DMA
            e.add("T", r * ld + 4 * c_lo, r * ld + 4 * c_hi + 3)
            if mode == 2:
                e.add("M", r * ld + 4 * c_lo, r * ld + 4 * c_hi + 3)
            st = r0 + k < r1  # stores (Y, and the momentum after the local steps)
            if st.any():
                rs = (r0 + k)[st]
                e.add("Y", rs * ld + 4 * c_lo[st], rs * ld + 4 * c_hi[st] + 3)
                if mode:
                    e.add("M", rs * ld + 4 * c_lo[st], rs * ld + 4 * c_hi[st] + 3)
    if tail:  # ring_mix_kernel<float, PF 4> over columns [4 n4, P), rows_per_block 4
        c_off, rpb, PF = 4 * n4, 4, 4
        for r0 in range(0, n, rpb):
            r1 = min(r0 + rpb, n)
            rows = [r0 - 1, r0] + [min(r0 + 1 + k, r1) for k in range(PF)]
            for i in range(r0, r1, PF):
                rows += [min(i + PF + 1 + k, r1) for k in range(PF)]
            for r in rows:
                buf, row = _row_ptr(r, n, wrap_halos)
                base = row * (ld if buf == "X" else 0) + c_off
                e.add(buf, base, base + tail - 1)
            for r in range(r0, r1):
                e.add("Y", r * ld + c_off, r * ld + c_off + tail - 1)
                e.add("T", r * ld + c_off, r * ld + c_off + tail - 1)
                if mode:
                    e.add("M", r * ld + c_off, r * ld + c_off + tail - 1)
    return e


def ring_edges_extents(n, P, ld, mode):
    """ring_edges_kernel: blockIdx.y 0 -> row 0, 1 -> row n - 1 (both halos when n == 1)."""
    e = Ext()
    for r in ([0] if n == 1 else [0, n - 1]):
        for buf, row in (("HP", 0) if r == 0 else ("X", r - 1), ("HN", 0) if r == n - 1 else ("X", r + 1)):
            e.add(buf, row * (ld if buf == "X" else 0), row * (ld if buf == "X" else 0) + P - 1)
        for buf in ("Y", "T") + (("M",) if mode else ()):
            e.add(buf, r * ld, r * ld + P - 1)
    return e


def csr_extents(n, P, ld, csr, mode, x_rows):
    """mix_csr_impl -> csr_xcd_kernel<32, 2, DgdEpi> (+ csr_mix_kernel for the rest)."""
    e = Ext()
    rowptr, col = np.asarray(csr.rowptr, np.int64), np.asarray(csr.col, np.int64)
    n4, tail = split_cols(P)
    XW, PS = 32, 2
    done4 = 0
    if n4 >= XW and n >= 512:
        nt = n4 // XW
        nrb = cdiv(n, (KT // XW) * PS)
        grid = cdiv(nt, 8) * 8 * nrb
        RB = (KT // XW) * PS
        b = np.arange(grid)
        xcd, local = b & 7, b >> 3
        tloc, rb = local // nrb, local % nrb
        ct = tloc * 8 + xcd
        live = ct < nt
        ct, rb = ct[live], rb[live]
        c_lo, c_hi = ct * XW, ct * XW + XW - 1  # f4 columns
        # rows of the block's passes: rb * RB + j, j < RB; the fast path reads
        # rowptr / col of min(row, n - 1) and stores only rows < n
        r_first, r_last = rb * RB, rb * RB + RB - 1
        e.add("rowptr", np.minimum(r_first, n - 1), np.minimum(r_last, n - 1) + 1)
        cols_touched = col if len(col) else np.zeros(1, np.int64)
        # X: neighbour rows (any row's columns: clamped rows read valid rows' lists)
        e.add("X", cols_touched.min() * ld + 4 * c_lo.min(), cols_touched.max() * ld + 4 * c_hi.max() + 3)
        ok = r_first < n
        lo_row, hi_row = r_first[ok], np.minimum(r_last[ok], n - 1)
        for buf in ("Y", "T") + (("M",) if mode else ()):
            e.add(buf, (lo_row * ld + 4 * c_lo[ok]).min(), (hi_row * ld + 4 * c_hi[ok] + 3).max())
        done4 = nt * XW
    for V, c_off, ncols in ((4, done4 * 4, n4 - done4), (1, n4 * 4, tail)):
        if ncols <= 0:
            continue
        # csr_mix_kernel<V, 16>: c < ncols_v; rows r0..r1-1 of each group; X rows col[e] of those rows
        c_hi = c_off + (ncols - 1) * V + V - 1
        e.add("X", col.min() * ld + c_off, col.max() * ld + c_hi)
        e.add("rowptr", 0, n)
        for buf in ("Y", "T") + (("M",) if mode else ()):
            e.add(buf, c_off, (n - 1) * ld + c_hi)
    return e


def ring_stream_dma_extents(n, P, ld, S, T=1024, D=8, PF=8):
    """ring_stream_dma_kernel<S, D, PF> (order 0 / 1 visit the same (ct, r0) set)."""
    e = Ext()
    n4 = P // 4
    nct = cdiv(n4, KT)
    for r0 in range(0, n, T):
        nT = min(T, n - r0)
        nsteps = nT + 2 * S
        ntot = cdiv(nsteps, PF) * PF
        interior = r0 - 2 * S >= 0 and r0 + nT + S + PF <= n

        def wrap(g):
            return g if interior else (g + n if g < 0 else (g - n if g >= n else g))
        # DMA rows: issue j = 0 .. ntot + D - 2; the pointer advances while issued < nsteps
        gl = wrap(r0 - S)
        rows = [gl]
        for _ in range(1, min(ntot + D - 1, nsteps)):
            gl += 1
            if not interior and gl == n:
                gl = 0
            rows.append(gl)
        rows = np.asarray(rows)
        assert rows.min() >= 0 and rows.max() < n, (r0, rows.min(), rows.max())
        e.add("X", rows.min() * ld, rows.max() * ld + 4 * (n4 - 1) + 3)
        # weights: wrap(r0 - 2S + min(i0 + j, nsteps + S - 1)), or the INTERIOR block loads
        w_lo = r0 - 2 * S if interior else 0
        w_hi = (r0 - 2 * S + ntot - PF + PF + S - 1) if interior else n - 1
        e.add("W", w_lo, w_hi)
        # live stores: rows r0 + i - 2S for 2S <= i < nsteps, descriptor = [row base, row base + ldy*4)
        e.add("Y", r0 * ld, (r0 + nT - 1) * ld + 4 * (n4 - 1) + 3)
    assert nct >= 1
    return e


GEOMETRIES = [
    (1024, 1 << 20),  # the fault's DGD round (tools/bench_configs.py dgd_round)
    (8192, 1 << 20),  # the bench's headline buffers
    (1000, 1 << 20),  # n not a multiple of the tile heights
    (515, 4099),      # P % 4 == 3: float tail columns
    (600, 101_770),   # config 5's MLP rows (P % 4 == 2)
    (3, 33),          # fewer rows than one tile
]


@pytest.mark.parametrize("n,P", GEOMETRIES)
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_ring_dgd_round_stays_in_its_rows(n, P, mode):
    ld = row_stride(P)
    e = ring_dma_extents(n, P, ld, mode)
    e.check({"X": n * ld, "Y": n * ld, "T": n * ld, "M": n * ld})
    hv = ring_dma_extents(max(n, 3), min(P, 4099), ld, mode, wrap_halos=False)  # sharded interior: halo vectors
    hv.check({"X": max(n, 3) * ld, "Y": max(n, 3) * ld, "T": max(n, 3) * ld, "M": max(n, 3) * ld, "HP": P, "HN": P})


@pytest.mark.parametrize("n", [1, 2, 1024])
def test_ring_edges_stay_in_their_rows(n):
    P = (1 << 20) + 3
    ld = row_stride(P)
    for mode in (0, 1, 2):
        ring_edges_extents(n, P, ld, mode).check({"X": n * ld, "Y": n * ld, "T": n * ld, "M": n * ld, "HP": P,
                                                  "HN": P})


@pytest.mark.parametrize("n,P", [(1024, 1 << 20), (8192, 1 << 20), (515, 4099), (700, 1 << 16 | 5)])
def test_csr_dgd_round_stays_in_its_rows(n, P):
    ld = row_stride(P)
    csr = G.random_regular_csr(n, 4, seed=2028)
    for mode in (0, 1, 2):
        e = csr_extents(n, P, ld, csr, mode, n)
        e.check({"X": n * ld, "Y": n * ld, "T": n * ld, "M": n * ld, "rowptr": n + 1})


@pytest.mark.parametrize("n,P,S", [(8192, 1 << 20, 5), (1024, 1 << 20, 8), (1000, 4096, 3), (20, 1024, 8)])
def test_ring_stream_dma_stays_in_its_rows(n, P, S):
    ld = row_stride(P)
    ring_stream_dma_extents(n, P, ld, S).check({"X": n * ld, "Y": n * ld, "W": n})


def test_mapped_size_covers_the_rows():
    """dol_bank_alloc maps round_up(rows * ld * 4, granularity): the extents
    above are checked against rows * ld, the tighter bound."""
    for n, P in GEOMETRIES:
        ld = row_stride(P)
        assert ld >= P and ld % 64 == 0
