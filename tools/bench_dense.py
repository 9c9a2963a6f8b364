"""Dense-W mix (BASELINE config 5's mixing): exact-f32 MFMA kernel vs the
three-piece bf16 split kernel, TFLOP/s (2 N^2 P flop per round) from HIP
events on the launching stream, and the max deviation between the two.

  python tools/bench_dense.py [--agents 1024 2048 8192] [--params 101770 1048576] [--reps 5]
Prints one JSON line per (N, P)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip import graph as G, ops  # noqa: E402
from dolhip.bank import row_stride  # noqa: E402

F32_MFMA_PEAK = 157.3   # TFLOP/s, MI355X spec (MI355X_MICROARCH.md)
BF16_MFMA_PEAK = 2516.6  # TFLOP/s dense bf16 (= 16 x the f32 matrix rate)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, nargs="+", default=[1024, 2048, 8192])
    ap.add_argument("--params", type=int, nargs="+", default=[101770])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--p-edge", type=float, default=0.1)
    ap.add_argument("--skip-f32-above", type=int, default=8192)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for N in a.agents:
        gen = torch.Generator(device=dev).manual_seed(2028)
        W = G.erdos_renyi_stochastic(N, a.p_edge, gen)
        for P in a.params:
            ld = row_stride(P)
            X = torch.empty(N, ld, device=dev).normal_()
            Y1 = torch.empty_like(X)
            Y2 = torch.empty_like(X)
            flops = 2.0 * N * N * P
            work = torch.empty(ops.dense_split3_workspace_bytes(N, N, P, 0), dtype=torch.uint8, device=dev)
            rec = {"agents": N, "params": P, "flop_per_round": flops, "workspace_GB": work.numel() / 1e9,
                   "workspace_fused_x_GB": ops.dense_split3_workspace_bytes(N, N, P, 6) / 1e9}
            ms_u = timed(lambda: ops.mix_dense_split3(W, X, Y2, P=P, work=work, fuse=True), a.reps)
            rec.update({"fused_x_ms": ms_u, "fused_x_TFLOPs": flops / ms_u / 1e9})
            ms_s = timed(lambda: ops.mix_dense_split3(W, X, Y2, P=P, work=work), a.reps)
            ms_g = timed(lambda: ops.mix_dense_split3(W, X, Y2, P=P, work=work, w_ready=True), a.reps)
            rec.update({"split3_ms": ms_s, "split3_TFLOPs": flops / ms_s / 1e9,
                        "split3_w_ready_ms": ms_g, "split3_w_ready_TFLOPs": flops / ms_g / 1e9,
                        "split3_vs_f32_peak": flops / ms_s / 1e9 / F32_MFMA_PEAK,
                        "split3_bf16_mfma_util": 6 * flops / ms_g / 1e9 / BF16_MFMA_PEAK})
            if N <= a.skip_f32_above:
                ms_f = timed(lambda: ops.mix_dense(W, X, Y1, P=P), a.reps)
                d = (Y1[:, :P] - Y2[:, :P]).abs().max().item()
                rec.update({"f32_ms": ms_f, "f32_TFLOPs": flops / ms_f / 1e9, "speedup": ms_f / ms_s,
                            "max_abs_diff_vs_f32": d, "max_abs_y": Y1[:, :P].abs().max().item()})
            print(json.dumps(rec), flush=True)
            del X, Y1, Y2, work
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
