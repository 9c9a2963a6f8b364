"""Dense ER mix on the bf16 matrix cores (split3): the split pass + record-staged
GEMM vs the fused X split (dense_split3_fx8_kernel and dense_split3_fxw_kernel,
r05; DOL_SPLIT3_FXW=1 selects the latter), alternating in one
process at bench.dense_mix_round's shape (1024 agents x 101,770, ER p = 0.1,
ld = row_stride(P)); one JSON line per (rep, path) with ms and the bf16 MFMA
utilisation the bench reports (6 x 2 N^2 P flop / ms / 2516.6 TF)."""
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
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    P = 101770
    gen = torch.Generator(device=dev).manual_seed(2028)
    W = G.erdos_renyi_stochastic(N, 0.1, gen)
    X = torch.empty(N, row_stride(P), device=dev).normal_(generator=gen)
    Y = torch.empty_like(X)
    work = torch.empty(ops.dense_split3_workspace_bytes(N, N, P, 0), dtype=torch.uint8, device=dev)
    for _ in range(200):  # clocks up
        ops.mix_dense_split3(W, X, Y, P=P, work=work)
    torch.cuda.synchronize()
    for rep in range(4):
        for path, fuse, env in (("split_pass", False, {}), ("fx8", True, {"DOL_SPLIT3_FXW": "0"}),
                                ("fxw", True, {"DOL_SPLIT3_FXW": "1"})):
            os.environ.update(env)  # read per call by dol_mix_dense_split3_f32
            for _ in range(20):
                ops.mix_dense_split3(W, X, Y, P=P, work=work, fuse=fuse)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                ops.mix_dense_split3(W, X, Y, P=P, work=work, fuse=fuse)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / 20
            print(json.dumps({"rep": rep, "agents": N, "params": P, "path": path, "ms": ms,
                              "bf16_mfma_util": 6 * 2.0 * N * N * P / (ms / 1e3) / 1e12 / 2516.6}), flush=True)


if __name__ == "__main__":
    main()
