"""Is a slow (source, destination) pair of bank matrices a matter of their
relative physical offset?  Three matrices of the bench's geometry; for every
ordered pair the eps = 5 pass (variant 3) writes the destination at column
offsets delta (floats; the row padding ld - P = 2048 leaves room): one JSON
line per pair with ms per delta.  python tools/eps_offset_probe.py"""
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
    ld = row_stride(P)
    deltas = [0, 64, 256, 1024, 2048]
    mats = {k: device_matrix(N, ld, dev) for k in "ABC"}
    for m in mats.values():
        m.normal_()
    wp, wn = torch.rand(N, device=dev), torch.rand(N, device=dev)

    def timed(fn, reps=4):
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
            X = mats[src]
            out = {}
            for dl in deltas:
                assert dl + P <= ld
                Y = mats[dst].view(-1)[dl:].as_strided((N, P), (ld, 1))
                out[dl] = timed(lambda: ops.mix_ring_steps(X[:, :P], Y, wp, wn, 5, P=P, n_rows=N, variant=3))
            print(json.dumps({"pair": f"{src}>{dst}", "ms_by_dst_offset_floats": {k: round(v, 3) for k, v in out.items()}}),
                  flush=True)


if __name__ == "__main__":
    main()
