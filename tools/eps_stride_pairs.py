"""Is a slow destination of FedLCon's eps pass a property of the allocation
at the bank's row stride?  Three mapped matrices A, B, C with 16 rows of
slack; for each ordered pair, the eps = 5 pass (variant 3) from X = src at
ld = row_stride(P) into Y = dst viewed at other row strides ld' (Y's rows at
ld' floats, same allocation).  ms per pass, one JSON line per pair.
  python tools/eps_stride_pairs.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from dolhip import ops  # noqa: E402
from dolhip.bank import device_matrix, row_stride  # noqa: E402


def main():
    dev = torch.device("cuda")
    N, P = 8192, 1 << 20
    ld = row_stride(P)  # 2^20 + 2048
    strides = [ld, ld - 1024, ld + 64, ld + 256, ld + 1024, ld + 2048]
    wp, wn = torch.rand(N, device=dev), torch.rand(N, device=dev)
    mats = {k: device_matrix(N + 24, ld, dev) for k in "ABC"}
    for m in mats.values():
        m.normal_()

    def timed(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps

    for src in "ABC":
        for dst in "ABC":
            if src == dst:
                continue
            X = mats[src][:N]
            out = {}
            for s in strides:
                Y = mats[dst].view(-1)[: N * s].view(N, s)
                out[s - (1 << 20)] = round(timed(lambda: ops.mix_ring_steps(X, Y, wp, wn, 5, P=P, n_rows=N,
                                                                             variant=3)), 3)
            print(json.dumps({"pair": f"{src}>{dst}", "eps_ms_by_dst_ld_minus_2^20": out}), flush=True)


if __name__ == "__main__":
    main()
