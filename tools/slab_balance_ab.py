"""The LDS-gather CSR mix (variant 3, the asm stream) on a row-order pack vs
the greedy wave-balanced pack (csr_slab_pack balance=True) of the same device
ER p = 0.1 W at 1024 x 101,770 and 8192 x 1024; plus each pack's own time.
Outputs compared bit for bit.  One JSON line per (shape, balance, trial)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))
from dolhip import graph as G, ops  # noqa: E402
from dolhip.bank import row_stride  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dev = torch.device("cuda")
    for N, P in ((1024, 101770), (8192, 1024)):
        g = torch.Generator(device=dev).manual_seed(2028)
        X = torch.empty(N, row_stride(P), device=dev).normal_(generator=g)
        W = G.erdos_renyi_stochastic_hip(N, 0.1, seed=2028, device=dev)
        rowptr, col, val = ops.dense_to_csr(W)
        packs = {b: ops.csr_slab_pack(rowptr, col, val, N, balance=b) for b in (False, True)}
        outs = {b: torch.empty_like(X) for b in packs}
        for trial in range(3):
            for b, (ent, hdr) in packs.items():
                ms = timed(lambda: ops.mix_csr_slab(X, outs[b], ent, hdr, N, P=P), 20)
                pk = timed(lambda: ops.csr_slab_pack(rowptr, col, val, N, ent=ent, hdr=hdr, balance=b), 10)
                same = bool(torch.equal(outs[b][:, :P].view(torch.int32), outs[False][:, :P].view(torch.int32)))
                print(json.dumps({"agents": N, "params": P, "balance": b, "trial": trial, "mix_ms": ms,
                                  "pack_ms": pk, "bits_equal_row_order": same}), flush=True)
        del X, W, packs, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
