"""Golden digests at Model1's real 8-key layout (P = 1,663,370) from the
REFERENCE (build container only; needs /root/reference):
    python tests/golden/make_golden_model1.py

For N = 6 and 16 agents whose state dicts have Model1's keys and shapes
(DIST/models.py:8-30, read from the reference class itself), with parameter
values drawn from numpy's default_rng(seed).standard_normal(float32):
  * one mixing round through Simulator.Neighbors + Client.consensus
    (DIST/simulators.py:91-97, DIST/clients.py:61-69) for circle/stochastic,
    compelete/stochastic and circle/double_stochastic W (communication_graph,
    seeded 2028);
  * FedAdmm_Client.update_duals (DEC/clients.py:141-144), rho = 0.1;
  * Server.average_weights (DEC/servers.py:42-48) over all N in a shuffled order.
The outputs are far too large to commit (up to 106 MB each), so the fixture
holds the inputs' seeds and, per output, the SHA-256 of its flattened fp32
bytes plus a strided sample (for diagnosis).  Tests regenerate the inputs
from the seeds and compare digests: bit-exactness at full Model1 size."""
import contextlib
import hashlib
import io
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import (DEC_SRC, DIST_SRC, GRAPH_SEED, _import_project, _Model, _Obj,  # noqa: E402
                         _placeholder_torchvision, rows_to_state_dicts, state_dict_to_row)

STRIDE = 99991


def model1_layout(models_mod):
    return [(k, tuple(v.shape)) for k, v in models_mod.Model1().state_dict().items()]


def inputs(seed, n, P):
    return np.random.default_rng(seed).standard_normal((n, P), dtype=np.float32)


def digest(a):
    a = np.ascontiguousarray(a, np.float32)
    return {"sha256": hashlib.sha256(a.tobytes()).hexdigest(), "sample": a.reshape(-1)[::STRIDE].tolist()}


def main():
    _placeholder_torchvision()
    dist = _import_project(DIST_SRC, ["simulators", "clients", "models"])
    layout = model1_layout(dist["models"])
    P = int(sum(np.prod(s) for _, s in layout))
    out = {"layout": [[k, list(s)] for k, s in layout], "P": P, "stride": STRIDE, "graph_seed": GRAPH_SEED,
           "mix": {}, "duals": {}, "average": {}}
    for n in (6, 16):
        for topo, mode in (("circle", "stochastic"), ("compelete", "stochastic"), ("circle", "double_stochastic")):
            seed = 1000 + n
            X = inputs(seed, n, P)
            torch.manual_seed(GRAPH_SEED)
            with contextlib.redirect_stdout(io.StringIO()):
                W = dist["simulators"].Simulator.communication_graph(None, topo, mode, n)[0]
            sds = rows_to_state_dicts(X, layout)
            fake = _Obj(args=_Obj(num_users=n), clients=[_Obj(model=_Model(sd)) for sd in sds])
            Y = np.empty_like(X)
            for i in range(n):
                Ni = dist["simulators"].Simulator.Neighbors(fake, i, W)
                Y[i] = state_dict_to_row(dist["clients"].Client.consensus(_Obj(model=_Model(sds[i])), Ni))
            out["mix"][f"{topo}_{mode}_{n}"] = {"seed": seed, "n": n, "topology": topo, "mode": mode,
                                               "Y": digest(Y)}
            print("mix", topo, mode, n, flush=True)
    dec = _import_project(DEC_SRC, ["clients", "servers"])
    for n in (6, 16):
        seeds = {"alpha": 2000 + n, "w": 3000 + n, "theta": 4000 + n}
        A = inputs(seeds["alpha"], n, P)
        Wt = inputs(seeds["w"], n, P)
        th = inputs(seeds["theta"], 1, P)[0]
        theta_sd = rows_to_state_dicts(th[None], layout)[0]
        A1 = np.empty_like(A)
        for k in range(n):
            c = _Obj(args=_Obj(rho=0.1), model=_Model(rows_to_state_dicts(Wt[k:k + 1], layout)[0]),
                     alpha=rows_to_state_dicts(A[k:k + 1], layout)[0])
            dec["clients"].FedAdmm_Client.update_duals(c, theta_sd)
            A1[k] = state_dict_to_row(c.alpha)
        out["duals"][str(n)] = {"seeds": seeds, "n": n, "rho": 0.1, "alpha1": digest(A1)}
        order = np.random.default_rng(5000 + n).permutation(n)
        theta = dec["servers"].Server.average_weights(None, [rows_to_state_dicts(Wt[o:o + 1], layout)[0]
                                                             for o in order])
        out["average"][str(n)] = {"seed_w": seeds["w"], "n": n, "order": order.tolist(),
                                  "theta": digest(state_dict_to_row(theta))}
        print("duals/average", n, flush=True)
    out["versions"] = {"torch": torch.__version__, "numpy": np.__version__}
    with open(os.path.join(HERE, "model1.json"), "w") as f:
        json.dump(out, f)
    print("wrote model1.json")


if __name__ == "__main__":
    main()
