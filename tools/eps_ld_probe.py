"""Does the row stride decide whether the eps = 5 pass is fast on a box?  On
some boxes every column-strip kernel runs the pass at ~5.4 TB/s while the ring
round (row bands) runs 6.3; the bank's stride is P + 1024 floats
(bank.row_stride).  Times each ring-steps kernel and one ring round at several
strides over the same two 8192-row buffers (views of one allocation each);
one JSON line per stride."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-optimization-and-learning_amd")]
from dolhip import ops  # noqa: E402


def ev_ms(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dev = torch.device("cuda:0")
    N, P = 8192, 1 << 20
    pads = [int(x) for x in (sys.argv[1:] or "1024 0 64 256 512 2048 3072 5120".split())]
    ldmax = P + max(pads)
    fx = torch.empty(N * ldmax, device=dev)
    fy = torch.empty(N * ldmax, device=dev)
    wp = torch.full((N,), 0.5, device=dev)
    wn = torch.full((N,), 0.5, device=dev)
    for pad in pads:
        ld = P + pad
        X = fx[: N * ld].view(N, ld)
        Y = fy[: N * ld].view(N, ld)
        X.normal_()
        rec = {"pad_floats": pad, "ld": ld,
               "ring_ms": ev_ms(lambda: ops.mix_ring(X, Y, wp, wn, P=P), 10)}
        for v in ops.RING_STEPS_VARIANTS:
            rec[f"eps5_v{v}_ms"] = ev_ms(lambda: ops.mix_ring_steps(X, Y, wp, wn, 5, P=P, variant=v), 5)
        rec["eps5_best_ms"] = min(rec[f"eps5_v{v}_ms"] for v in ops.RING_STEPS_VARIANTS)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
