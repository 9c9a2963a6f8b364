"""BASELINE configs 1 and 2 end to end through the drop-in API on one GPU.

  config 1 (WA.ipynb cell[11]/[23]): DecFedAvg, 6 users, Model1, local_ep 4,
           local_bs 128, lr 0.01, momentum 0.5, circle/stochastic, non-IID (2 shards)
  config 2 (PD.ipynb cell[8]/[10]):  FedAdmm_Server, 100 users, frac 0.1, Model1,
           local_ep 10, local_bs 50, lr 0.1, rho 0.1, momentum 0.5, IID

Data: seeded synthetic MNIST-shaped sets of MNIST's size (60000 / 10000;
MNIST itself is not available offline).  Prints one JSON line per config with
seconds per round.  The reference's only published numbers are end-to-end
Colab wall clocks (GPU model unrecorded): 80.6 s/round
(DecFedAvg circle) and 31.2 s/round (FedADMM) — context, not a like-for-like
baseline.
usage: python tools/bench_notebooks.py [--rounds 2] [--configs 1 2]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))

import torch  # noqa: E402

from conftest import load_project  # noqa: E402


def run_wa(rounds):
    m = load_project("weighted_average", ["simulators", "utils"])
    args = m["utils"].DotDict(rounds=rounds, num_users=6, local_ep=4, local_bs=128, lr=0.01, topology="circle",
                              mode="stochastic", model="Model1", dataset="synthetic", iid=False, shards=2, seed=2028,
                              momentum=0.5, verbose=False, synthetic_train=60000, synthetic_test=10000, device="cuda")
    t0 = time.time()
    sim = m["simulators"].DecFedAvg(args)
    build = time.time() - t0
    torch.cuda.synchronize()
    t0 = time.time()
    sim.run(rounds)
    torch.cuda.synchronize()
    el = time.time() - t0
    return {"config": "WA DecFedAvg circle 6 users Model1 local_ep 4 bs 128", "rounds": rounds,
            "s_per_round": el / rounds, "setup_s": build, "history": sim.history,
            "reference_colab_s_per_round": 82.2}


def run_pd(rounds):
    m = load_project("primal_dual", ["servers", "utils"])
    args = m["utils"].DotDict(num_users=100, local_ep=10, local_bs=50, lr=0.1, model="Model1", dataset="synthetic",
                              iid=True, rho=0.1, seed=2022, momentum=0.5, verbose=False, synthetic_train=60000,
                              synthetic_test=10000, device="cuda")
    t0 = time.time()
    s = m["servers"].FedAdmm_Server(args)
    build = time.time() - t0
    torch.cuda.synchronize()
    t0 = time.time()
    s.run(0.1, rounds)
    torch.cuda.synchronize()
    el = time.time() - t0
    return {"config": "PD FedAdmm_Server 100 users frac 0.1 Model1 local_ep 10 bs 50", "rounds": rounds,
            "s_per_round": el / rounds, "setup_s": build,
            "history": [{k: float(v) for k, v in h.items()} for h in s.history],
            "reference_colab_s_per_round": 31.2}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--configs", type=int, nargs="+", default=[1, 2])
    a = ap.parse_args()
    import contextlib
    import io
    for c in a.configs:
        with contextlib.redirect_stdout(io.StringIO()):
            res = run_wa(a.rounds) if c == 1 else run_pd(a.rounds)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
