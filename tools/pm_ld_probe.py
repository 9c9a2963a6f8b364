"""Parameter-major random 4-regular mix (csr_pm_kernel) at 8192 agents x 2^20
parameters: does the p-row stride (floats, >= 8192 = 32 KiB, a multiple of
8 KiB) decide its rate the way the agent-row stride decides the ring's?  Each
stride's XT / YT are views of the same two allocations; every stage order is
timed; strides alternate twice.  One JSON line per (rep, stride)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-optimization-and-learning_amd")]
from dolhip import graph as G, ops  # noqa: E402


def ev_ms(fn, reps):
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
    dev = torch.device("cuda:0")
    N, P = 8192, 1 << 20
    pads = [int(x) for x in (sys.argv[1:] or "0 64 1024 2048 4096".split())]
    ldmax = N + max(pads)
    fx = torch.empty(P * ldmax, device=dev).normal_()
    fy = torch.empty(P * ldmax, device=dev)
    c = G.random_regular_csr(N, 4, seed=2028)
    rp = torch.as_tensor(c.rowptr, dtype=torch.int32, device=dev)
    col = torch.as_tensor(c.col, dtype=torch.int32, device=dev)
    val = torch.as_tensor(c.val, dtype=torch.float32, device=dev)
    for rep in range(2):
        for pad in pads:
            ld = N + pad
            XT = fx[: P * ld].view(P, ld)
            YT = fy[: P * ld].view(P, ld)
            rec = {"rep": rep, "pad_floats": pad, "ld": ld}
            for ns in (8, 16, 32):
                rec[f"nseg{ns}_ms"] = ev_ms(lambda: ops.mix_csr_pm(XT, YT, rp, col, val, nseg=ns), 6)
            rec["best_ms"] = min(rec[f"nseg{ns}_ms"] for ns in (8, 16, 32))
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
