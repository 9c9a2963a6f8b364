"""Generate distributed-optimization-and-learning_amd/csrc/csr_slab_stream.inc:
the hand-scheduled inner loop of csr_slab_kernel's variant 3 (one wave's run
of entry pairs for one chunk as one software-pipelined stream).  See the
comment at the top of the generated file; rerun after editing:
    python tools/gen_slab_stream_asm.py [--ahead G]
G = how many pairs ahead the gathers run (the index reads run G + 1 ahead)."""
import argparse
import math
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "distributed-optimization-and-learning_amd", "csrc", "csr_slab_stream.inc")

ACC = "DOL_ACCB_%="   # first register of the accumulator tuple %[acc] (row r's f4 at ACC + 4 r)
T0 = None             # pipeline registers: the top nregs VGPRs (clobbered; set by Map)
VMAX = 128            # VGPRs per lane at 16 waves per CU
S_JB, S_NBR, S_RN, S_M0, S_IDX = "s84", "s85", "s86", "s88", "s89"


def v(a, b=None):
    return f"v{a}" if b is None else f"v[{a}:{b}]"


def acc(x):
    """accumulator registers ACC + x, ACC + x + 1"""
    return f"v[{ACC}+{x}:{ACC}+{x + 1}]"


def acc_base(lines, nregs):
    """%[acc] is a compiler-allocated 32-register tuple: find its first register
    by matching the operand's text against every even base outside the pipeline
    registers (assembler directives only; nothing runs)."""
    lines += [f".set {ACC}, -1"]
    for b in range(0, VMAX - 31, 2):
        if b + 31 < T0 or b >= T0 + nregs:
            lines += [f".ifc %[acc],v[{b}:{b + 31}]", f".set {ACC}, {b}", ".endif"]
    lines += [f".if {ACC} < 0", ".error \\\"csr_slab_stream: accumulator tuple not found\\\"", ".endif"]


class Map:
    def __init__(self, g):
        global T0
        self.g = g
        self.ni, self.ng = g + 2, g + 1             # index-pair sets, gathered-piece sets
        T0 = VMAX - (4 * self.ni + 8 * self.ng + 2)
        self.unroll = self.ni * self.ng // math.gcd(self.ni, self.ng)
        self.I = [T0 + 4 * i for i in range(self.ni)]                      # (w0, o0, w1, o1)
        gb = T0 + 4 * self.ni
        self.G = [(gb + 8 * i, gb + 8 * i + 4) for i in range(self.ng)]    # (entry 0 f4, entry 1 f4)
        self.VA = gb + 8 * self.ng                                          # gather addresses
        self.nregs = self.VA + 2 - T0


def bnd_update(lines):
    """S_NBR = B(S_RN) - S_JB (%[hc] lane r holds B(r) after the prologue)."""
    lines += [f"v_readlane_b32 {S_NBR}, %[hc], {S_RN}",
              f"s_nop 0",
              f"s_sub_u32 {S_NBR}, {S_NBR}, {S_JB}"]


def gathers(m, iset, gset, lines):
    lines += [f"v_add_u32 {v(m.VA)}, %[lb], {v(iset + 1)}",
              f"v_add_u32 {v(m.VA + 1)}, %[lb], {v(iset + 3)}",
              f"ds_read_b128 {v(gset[0], gset[0] + 3)}, {v(m.VA)}",
              f"ds_read_b128 {v(gset[1], gset[1] + 3)}, {v(m.VA + 1)}"]


def step(m, k, lines, tail):
    g = m.g
    ic, inx, ird = m.I[k % m.ni], m.I[(k + g) % m.ni], m.I[(k + g + 1) % m.ni]
    gc, gn = m.G[k % m.ng], m.G[(k + g) % m.ng]
    lines += [f"s_cmp_eq_u32 {S_NBR}, {k}",        # row r + 1 starts at pair jb + k
              f"s_cbranch_scc1 .Lbnd{k}_%=",
              f".Lcont{k}_%=:",
              f"ds_read_b128 {v(ird, ird + 3)}, %[pb] offset:{16 * (k + g + 1)}",
              # LDS returns in order: <= 3 left means pair j + g's index and pair j's pieces landed
              "s_waitcnt lgkmcnt(3)"]
    gathers(m, inx, gn, lines)
    if g == 1:
        lines += ["s_waitcnt lgkmcnt(3)"]          # pair j's pieces were issued after pair j + 2's index
    lines += [  # products in place of the gathered pieces (dead after)
        f"v_pk_mul_f32 {v(gc[0], gc[0] + 1)}, {v(ic, ic + 1)}, {v(gc[0], gc[0] + 1)} op_sel_hi:[0,1]",
        f"v_pk_mul_f32 {v(gc[0] + 2, gc[0] + 3)}, {v(ic, ic + 1)}, {v(gc[0] + 2, gc[0] + 3)} op_sel_hi:[0,1]",
        f"v_pk_mul_f32 {v(gc[1], gc[1] + 1)}, {v(ic + 2, ic + 3)}, {v(gc[1], gc[1] + 1)} op_sel_hi:[0,1]",
        f"v_pk_mul_f32 {v(gc[1] + 2, gc[1] + 3)}, {v(ic + 2, ic + 3)}, {v(gc[1] + 2, gc[1] + 3)} op_sel_hi:[0,1]",
        f"s_set_gpr_idx_on {S_IDX}, gpr_idx(SRC0,DST)",
        f"v_pk_add_f32 {acc(0)}, {acc(0)}, {v(gc[0], gc[0] + 1)}",
        f"v_pk_add_f32 {acc(2)}, {acc(2)}, {v(gc[0] + 2, gc[0] + 3)}",
        f"v_pk_add_f32 {acc(0)}, {acc(0)}, {v(gc[1], gc[1] + 1)}",
        f"v_pk_add_f32 {acc(2)}, {acc(2)}, {v(gc[1] + 2, gc[1] + 3)}",
        "s_set_gpr_idx_off"]
    # out of line: the row boundary at pair jb + k -- r advances (S_RN = r + 1,
    # S_IDX = 4 r), rows empty in this chunk are skipped; the run's end is row
    # 7's boundary (B(8) = n), so r reaching 8 ends the stream
    tail += [f".Lbnd{k}_%=:",
             f"s_add_u32 {S_RN}, {S_RN}, 1",
             f"v_readlane_b32 {S_NBR}, %[hc], {S_RN}",   # B(r + 1) (lane 9 when r = 8: unused)
             f"s_add_u32 {S_IDX}, {S_IDX}, 4",
             f"s_cmp_ge_u32 {S_RN}, 9",
             "s_cbranch_scc1 .Ldone_%=",
             f"s_sub_u32 {S_NBR}, {S_NBR}, {S_JB}",
             f"s_cmp_eq_u32 {S_NBR}, {k}",
             f"s_cbranch_scc1 .Lbnd{k}_%=",
             f"s_branch .Lcont{k}_%="]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ahead", type=int, default=2)
    g = ap.parse_args().ahead
    assert g >= 1
    m = Map(g)
    lines = []
    acc_base(lines, m.nregs)
    lines += ["s_waitcnt lgkmcnt(0)",
             f"s_mov_b32 {S_M0}, m0",
             "s_cmp_eq_u32 %[n], 0",                # no pairs for this wave in this chunk
             "s_cbranch_scc1 .Ldone_%=",
             f"s_mov_b32 {S_JB}, 0",
             f"s_mov_b32 {S_RN}, 1",
             f"s_mov_b32 {S_IDX}, 0",
             # header lanes -> B(r) = (((lane r) & ~1) - b0) >> 1, the pair where row r starts
             "v_and_b32 %[hc], -2, %[hc]",
             "v_sub_u32_e64 %[hc], %[hc], %[b0]",
             "v_lshrrev_b32 %[hc], 1, %[hc]"]
    bnd_update(lines)
    # prologue: index pairs 0..g, gathers of pairs 0..g-1
    for i in range(g + 1):
        lines += [f"ds_read_b128 {v(m.I[i], m.I[i] + 3)}, %[pb]" + (f" offset:{16 * i}" if i else "")]
    for i in range(g):
        lines += [f"s_waitcnt lgkmcnt({g + i})"]  # outstanding: index pairs i..g, then 2 i pieces
        gathers(m, m.I[i], m.G[i], lines)
    lines += [".Lloop_%=:"]
    tail = []
    for k in range(m.unroll):
        step(m, k, lines, tail)
    lines += [f"v_add_u32 %[pb], {16 * m.unroll}, %[pb]",
              f"s_add_u32 {S_JB}, {S_JB}, {m.unroll}",
              f"s_sub_u32 {S_NBR}, {S_NBR}, {m.unroll}",
              "s_branch .Lloop_%="]
    lines += tail
    lines += [".Ldone_%=:", "s_waitcnt lgkmcnt(0)", f"s_mov_b32 m0, {S_M0}"]
    clob = [f'"v{r}"' for r in range(T0, T0 + m.nregs)] + [f'"{s}"' for s in (S_JB, S_NBR, S_RN, S_M0, S_IDX)]
    with open(OUT, "w") as f:
        f.write("// GENERATED by tools/gen_slab_stream_asm.py -- do not edit by hand.\n")
        f.write("// csr_slab_kernel variant 3: one wave's run of n entry pairs for one chunk as a\n")
        f.write(f"// software-pipelined stream.  Pair j: index pair j + {g + 1} read, gathers of pair j + {g}\n")
        f.write("// issued, pair j's four products added into row r's accumulator IN PLACE\n")
        f.write("// (s_set_gpr_idx_on SRC0|DST, index 4 r into the %[acc] tuple); at the pair\n")
        f.write("// where row r + 1 starts (B(r + 1)) r advances, skipping rows empty in this\n")
        f.write(f"// chunk; the run ends at B(8) = n.  Registers rotate over {m.unroll} steps ({m.ni} index\n")
        f.write(f"// pairs from v{m.I[0]}, {m.ng} gathered piece pairs from v{m.G[0][0]}, overwritten by their\n")
        f.write(f"// products; addresses v{m.VA}, v{m.VA + 1}).  Reads run up to {g + 1} pairs past the run.\n")
        f.write("// Entry order and rounding as every other variant: same bits.\n")
        f.write(f"#define DOL_SLAB_STREAM_AHEAD {g + 1}\n")
        f.write("#define DOL_SLAB_STREAM_ASM \\\n")
        for ln in lines:
            f.write(f'  "{ln}\\n\\t" \\\n')
        f.write("\n")
        f.write("#define DOL_SLAB_STREAM_ACC \"+v\"\n")
        f.write("#define DOL_SLAB_STREAM_CLOBBERS " + ", ".join(clob) + "\n")
    print(OUT, len(lines), "lines")


if __name__ == "__main__":
    main()
