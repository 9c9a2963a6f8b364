"""split3 at bench.dense_mix_round's shape (1024 x 1024 x 101,770, fused X
split): the tail's quarter-tile kernel at 8 waves (4 x 2, default) vs 4 waves
(2 x 2, DOL_SPLIT3_FX8_TAIL=4) vs no tail split (DOL_SPLIT3_CUS=0: the last
partial wave runs as whole tiles), alternating in one process; outputs compared
bit for bit.  One JSON line per (rep, path)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-optimization-and-learning_amd")]
from dolhip import graph as G, ops  # noqa: E402
from dolhip.bank import row_stride  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    N, P = 1024, 101770
    gen = torch.Generator(device=dev).manual_seed(2028)
    W = G.erdos_renyi_stochastic(N, 0.1, gen)
    X = torch.empty(N, row_stride(P), device=dev).normal_(generator=gen)
    work = torch.empty(ops.dense_split3_workspace_bytes(N, N, P, 0), dtype=torch.uint8, device=dev)
    paths = (("tail8", {"DOL_SPLIT3_FX8_TAIL": "8", "DOL_SPLIT3_CUS": ""}),
             ("tail4", {"DOL_SPLIT3_FX8_TAIL": "4", "DOL_SPLIT3_CUS": ""}),
             ("no_tail", {"DOL_SPLIT3_FX8_TAIL": "8", "DOL_SPLIT3_CUS": "0"}))
    outs = {name: torch.empty_like(X) for name, _ in paths}
    for _ in range(200):  # clocks up
        ops.mix_dense_split3(W, X, outs["tail8"], P=P, work=work)
    torch.cuda.synchronize()
    for rep in range(4):
        for name, env in paths:
            os.environ.update(env)  # read per call by dol_mix_dense_split3_f32
            Y = outs[name]
            for _ in range(20):
                ops.mix_dense_split3(W, X, Y, P=P, work=work)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                ops.mix_dense_split3(W, X, Y, P=P, work=work)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / 20
            same = bool(torch.equal(Y[:, :P].view(torch.int32), outs["tail8"][:, :P].view(torch.int32)))
            print(json.dumps({"rep": rep, "path": name, "ms": ms, "bf16_mfma_util": 6 * 2.0 * N * N * P / ms / 1e9 / 2516.6,
                              "bits_equal_tail8": same}), flush=True)


if __name__ == "__main__":
    main()
