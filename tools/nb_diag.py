"""Diagnostic: drop-in FedAvg/FedAdmm at the PD notebook shape vs the reference's
CPU trajectory (tests/golden/trajectories.json 'notebook'): per-round history
and the relative parameter differences, to size the GPU-vs-CPU drift."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "distributed-optimization-and-learning_amd")]
from conftest import GOLDEN, load_project  # noqa: E402

TRAJ = json.load(open(os.path.join(GOLDEN, "trajectories.json")))
NB = TRAJ["notebook"]
det = len(sys.argv) > 1 and sys.argv[1] == "det"
if det:
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
for server in ("FedAvg_Server", "FedAdmm_Server"):
    m = load_project("primal_dual", ["servers", "utils"])
    args = m["utils"].DotDict(dict(TRAJ["dec_args"], **NB["dec_args"], device="cuda", verbose=False))
    s = getattr(m["servers"], server)(args)
    s.run(NB["frac"], 2)
    ref = NB[server]
    print(server, "deterministic" if det else "")
    for h, r in zip(s.history, ref["history"]):
        print("  got", {k: round(float(v), 6) for k, v in h.items()})
        print("  ref", {k: round(float(v), 6) for k, v in r.items()})
    g = torch.cat([v.detach().reshape(-1).float().cpu() for v in s.global_client.model.state_dict().values()]).numpy()
    rs = np.array(ref["global"]["sample"], np.float32)
    d = np.abs(g[::NB["stride"]] - rs)
    print("  global: max|d| %.3e  max|x| %.3e  l2 got %.6f ref %.6f" % (d.max(), np.abs(rs).max(),
          np.linalg.norm(g.astype(np.float64)), ref["global"]["l2"]))
