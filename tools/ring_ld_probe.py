"""Ring round (the headline kernel) at several row strides over the same two
8192-row buffers, alternating strides several times in one process; one JSON
line per (rep, stride).  bank.row_stride uses P + 1024 floats for P = 2^20."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-optimization-and-learning_amd")]
from dolhip import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    N, P = 8192, 1 << 20
    pads = [int(x) for x in (sys.argv[1:] or "1024 2048 3072 4096 6144".split())]
    ldmax = P + max(pads)
    fx = torch.empty(N * ldmax, device=dev).normal_()
    fy = torch.empty(N * ldmax, device=dev)
    wp = torch.full((N,), 0.5, device=dev)
    wn = torch.full((N,), 0.5, device=dev)
    for rep in range(3):
        for pad in pads:
            ld = P + pad
            X = fx[: N * ld].view(N, ld)
            Y = fy[: N * ld].view(N, ld)
            for _ in range(5):
                ops.mix_ring(X, Y, wp, wn, P=P)
            torch.cuda.synchronize()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
            for s, e in evs:
                s.record()
                ops.mix_ring(X, Y, wp, wn, P=P)
                e.record()
            torch.cuda.synchronize()
            ms = sorted(s.elapsed_time(e) for s, e in evs)
            print(json.dumps({"rep": rep, "pad_floats": pad, "ring_ms_mean": sum(ms) / len(ms), "ring_ms_min": ms[0],
                              "TBps_mean": 2 * N * P * 4 / (sum(ms) / len(ms) / 1e3) / 1e12}), flush=True)


if __name__ == "__main__":
    main()
