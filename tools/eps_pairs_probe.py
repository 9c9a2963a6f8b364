"""Which buffer makes FedLCon's eps pass slow?  Three bank matrices of the
bench's geometry (8192 x 2^20 at ld = row_stride(P), bank.device_matrix:
mapped blocks by default) and the eps = 5 pass (variant 3, LDS-DMA stream)
plus the headline ring kernel timed for every ordered (src, dst) pair.  One
JSON line: {"pairs": {"A>B": ms, ...}, "ring": {...}}.
python tools/eps_pairs_probe.py [--variants 3 6] [--reps 5] [--torch] [--va-align 0 1073741824 ...]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip import ops  # noqa: E402
from dolhip.bank import device_matrix, row_stride  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", type=int, nargs="+", default=[3])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--torch", action="store_true", help="torch-allocated matrices instead of mapped blocks")
    ap.add_argument("--pm", action="store_true", help="also the parameter-major random 4-regular mix (config 3) per pair")
    ap.add_argument("--va-align", type=int, nargs="+", default=[0],
                    help="DOL_BANK_VA_ALIGN per block of three matrices (0: the granularity)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    N, P = 8192, 1 << 20
    ld = row_stride(P)
    wp, wn = torch.rand(N, device=dev), torch.rand(N, device=dev)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.reps

    for align in a.va_align:  # each setting: its own three matrices (the alignment is read per allocation)
        if align:
            os.environ["DOL_BANK_VA_ALIGN"] = str(align)
        else:
            os.environ.pop("DOL_BANK_VA_ALIGN", None)
        mats = {k: device_matrix(N, ld, dev, mapped=not a.torch) for k in "ABC"}
        for m in mats.values():
            m.normal_()
        eps, ring, pm = {}, {}, {}
        if a.pm:
            from dolhip import graph as G
            c = G.random_regular_csr(N, 4, seed=2028)
            rr = [torch.as_tensor(t, device=dev) for t in (c.rowptr, c.col, c.val)]
        for src in "ABC":
            for dst in "ABC":
                if src == dst:
                    continue
                X, Y = mats[src], mats[dst]
                pair = f"{src}>{dst}"
                eps[pair] = {v: timed(lambda: ops.mix_ring_steps(X, Y, wp, wn, 5, P=P, n_rows=N, variant=v))
                             for v in a.variants}
                ring[pair] = timed(lambda: ops.mix_ring(X, Y, wp, wn, P=P, n_rows=N))
                if a.pm:
                    XT, YT = X.view(-1)[:P * N].view(P, N), Y.view(-1)[:P * N].view(P, N)
                    pm.setdefault(pair, timed(lambda: ops.mix_csr_pm(XT, YT, *rr, nseg=16)))
                print(json.dumps({"va_align": align, "pair": pair, "eps_ms": {v: round(t, 3) for v, t in eps[pair].items()},
                                  "ring_ms": round(ring[pair], 3), "pm_ms": round(pm.get(pair, 0.0), 3)}),
                      file=sys.stderr, flush=True)
        print(json.dumps({"variants": a.variants, "band_r": os.environ.get("DOL_RING_BAND_R"),
                          "alloc": "torch" if a.torch else "mapped", "ld": ld, "va_align": align,
                          "bases": {k: m.data_ptr() for k, m in mats.items()}, "eps_ms": eps, "ring_ms": ring}),
              flush=True)
        del mats, X, Y
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
