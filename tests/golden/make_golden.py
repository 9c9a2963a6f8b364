"""Generate the golden vectors in tests/golden/*.npz by running the REFERENCE.

Run in the build container only (needs /root/reference, which never travels
to the GPU box):   python tests/golden/make_golden.py

It imports the shipped reference modules
  /root/reference/Distributed Optimization/src/{simulators,clients}.py
  /root/reference/Decentralized Optimization/src/{servers,clients}.py
and calls the hot-path functions directly on seeded synthetic inputs:
  communication_graph (DIST/simulators.py:40-86), Neighbors (:91-97),
  Client.consensus (DIST/clients.py:61-69), FedAvg/FedProx/FedAdmm
  update_model + torch.optim.SGD.step (DEC/clients.py:85-139, :44),
  FedAdmm_Client.update_duals (DEC/clients.py:141-144),
  Server.average_weights (DEC/servers.py:42-48).

torchvision is not installed here.  The reference's utils.py imports it at
module level but none of the functions called above touch it (datasets are
never loaded), so a bare placeholder module is registered in sys.modules
purely to satisfy that import.  Nothing else of the reference is altered.
The arrays are written with numpy (no pickles): inputs AND reference outputs.
"""
from __future__ import annotations

import contextlib
import copy
import importlib
import io
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
DIST_SRC = os.path.join(REF, "Distributed Optimization", "src")
DEC_SRC = os.path.join(REF, "Decentralized Optimization", "src")
OUT = os.path.dirname(os.path.abspath(__file__))


def _placeholder_torchvision():
    tv = types.ModuleType("torchvision")
    tv.datasets = types.ModuleType("torchvision.datasets")
    tv.transforms = types.ModuleType("torchvision.transforms")
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.datasets", tv.datasets)
    sys.modules.setdefault("torchvision.transforms", tv.transforms)


def _import_project(src_dir, names):
    """Import the reference's flat modules from one project directory."""
    for n in ("models", "utils", "sampling", "clients", "simulators", "servers"):
        sys.modules.pop(n, None)
    sys.path.insert(0, src_dir)
    try:
        return {n: importlib.import_module(n) for n in names}
    finally:
        sys.path.remove(src_dir)


class _Obj:
    """Attribute bag used as `self` for unbound reference methods."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


class _Model:
    def __init__(self, sd):
        self._sd = sd

    def state_dict(self):
        return self._sd


# "mini" layout: several keys with odd sizes, exercising multi-key flattening.
MINI = [("a.weight", (5, 3)), ("a.bias", (7,)), ("b.weight", (33, 4))]
FLAT_1031 = [("w", (1031,))]
FLAT_4097 = [("w", (4097,))]


def layout_size(layout):
    return int(sum(int(np.prod(s)) for _, s in layout))


def random_rows(rng, n, P, special=False):
    X = rng.standard_normal((n, P)).astype(np.float32)
    if special:
        flat = X.reshape(-1)
        k = flat.size
        idx = rng.choice(k, size=min(k, 64), replace=False)
        vals = np.array([-0.0, 0.0, 1e-40, -1e-40, 3e38, -3e38, 1e-30, 7.0],
                        dtype=np.float32)
        flat[idx] = vals[np.arange(idx.size) % vals.size]
    return X


def rows_to_state_dicts(X, layout):
    out = []
    for row in X:
        sd, off = {}, 0
        for k, shape in layout:
            n = int(np.prod(shape))
            sd[k] = torch.from_numpy(row[off:off + n].copy()).reshape(shape)
            off += n
        out.append(sd)
    return out


def state_dict_to_row(sd):
    return np.concatenate([v.detach().cpu().numpy().reshape(-1) for v in sd.values()]).astype(
        np.float32)


GRAPH_CASES = [
    ("circle", "stochastic", 3), ("circle", "stochastic", 5), ("circle", "stochastic", 6),
    ("circle", "stochastic", 16), ("circle", "stochastic", 64), ("circle", "stochastic", 1),
    ("circle", "stochastic", 2),
    ("star", "stochastic", 5), ("star", "stochastic", 6),
    ("compelete", "stochastic", 5), ("compelete", "stochastic", 6), ("compelete", "stochastic", 16),
    ("dynamic", "stochastic", 6),
    # Sinkhorn cases that terminate (SURVEY.md section 7 lists the ones that hang)
    ("circle", "double_stochastic", 6), ("circle", "double_stochastic", 16),
    ("circle", "double_stochastic", 64), ("compelete", "double_stochastic", 6),
    # any other mode returns the raw 0/1 float64 adjacency
    ("circle", "none", 6), ("compelete", "none", 5),
]
GRAPH_SEED = 2028


def gen_graphs(sim_mod):
    comm = sim_mod.Simulator.communication_graph
    graphs, csr = {}, {}
    for topo, mode, n in GRAPH_CASES:
        key = f"{topo}_{mode}_{n}"
        torch.manual_seed(GRAPH_SEED)
        with contextlib.redirect_stdout(io.StringIO()):  # double_stochastic prints sums
            gs = comm(None, topo, mode, n)
        arr = np.stack([np.asarray(g.numpy() if torch.is_tensor(g) else g) for g in gs])
        graphs[key] = arr
        # CSR implied by Neighbors (DIST/simulators.py:91-97): one per time step
        fake = _Obj(args=_Obj(num_users=n),
                    clients=[_Obj(model=_Model({"id": j})) for j in range(n)])
        for t, g in enumerate(gs):
            rowptr, col, val = [0], [], []
            for i in range(n):
                for a, sd in sim_mod.Simulator.Neighbors(fake, i, g):
                    col.append(sd["id"])
                    val.append(float(a))
                rowptr.append(len(col))
            csr[f"{key}__t{t}__rowptr"] = np.asarray(rowptr, np.int32)
            csr[f"{key}__t{t}__col"] = np.asarray(col, np.int32)
            csr[f"{key}__t{t}__val"] = np.asarray(val, np.float32)
    return graphs, csr


def gen_mix(sim_mod, cli_mod, graphs):
    """One Jacobi mixing round through Neighbors + Client.consensus."""
    rng = np.random.default_rng(100)
    out = {}
    cases = []
    for topo, mode, n in GRAPH_CASES:
        if n <= 16:
            cases.append((f"{topo}_{mode}_{n}", "mini", MINI))
    cases += [("circle_stochastic_64", "flat1031", FLAT_1031),
              ("compelete_stochastic_16", "flat4097", FLAT_4097)]
    for gkey, lname, layout in cases:
        W = graphs[gkey]
        n = W.shape[1]
        P = layout_size(layout)
        X = random_rows(rng, n, P, special=True)
        if gkey == "circle_stochastic_6":  # propagation of non-finite values
            X[2, 5] = np.nan
            X[4, 7] = np.inf
        sds = rows_to_state_dicts(X, layout)
        fake = _Obj(args=_Obj(num_users=n), clients=[_Obj(model=_Model(sd)) for sd in sds])
        for t in range(W.shape[0]):
            g = torch.from_numpy(W[t]) if W.dtype == np.float32 else W[t]
            Y = np.zeros((n, P), np.float32)
            for i in range(n):
                Ni = sim_mod.Simulator.Neighbors(fake, i, g)
                me = _Obj(model=_Model(sds[i]))
                Y[i] = state_dict_to_row(cli_mod.Client.consensus(me, Ni))
            k = f"{gkey}__{lname}__t{t}"
            out[k + "__X"] = X
            out[k + "__Y"] = Y
    return out


class _TinyNet(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.l1 = torch.nn.Linear(13, 9)
        self.l2 = torch.nn.Linear(9, 4)

    def forward(self, x):
        return self.l2(torch.relu(self.l1(x)))


def gen_local_steps(dec_cli):
    """Per-step (w, buf, raw g) -> (g', w', buf') through the reference's
    update_model + torch.optim.SGD.step, for FedAvg / FedProx / FedAdmm."""
    out = {}
    T = 4
    for cname, lr, mom in (("FedAvg_Client", 0.1, 0.5), ("FedProx_Client", 0.1, 0.5),
                           ("FedAdmm_Client", 0.1, 0.5), ("FedAdmm_Client", 0.05, 0.0)):
        torch.manual_seed(7)
        cls = getattr(dec_cli, cname)
        model = _TinyNet()
        args = _Obj(rho=0.1, device="cpu", lr=lr, momentum=mom)
        c = cls.__new__(cls)
        c.args, c.model, c.criterion = args, model, torch.nn.CrossEntropyLoss()
        c.optimizer = torch.optim.SGD(model.parameters(), lr=lr, momentum=mom)
        theta = {k: v.detach().clone() + 0.3 * torch.randn_like(v) for k, v in model.state_dict().items()}
        if cname == "FedAdmm_Client":
            c.alpha = {k: 0.05 * torch.randn_like(v) for k, v in model.state_dict().items()}
            alpha0 = state_dict_to_row(c.alpha)
        rec = {n: [] for n in ("w", "buf", "g", "gp", "w1", "buf1")}
        for t in range(T):
            images = torch.randn(11, 13)
            labels = torch.randint(0, 4, (11,))
            shadow = copy.deepcopy(model)
            shadow.zero_grad()
            torch.nn.CrossEntropyLoss()(shadow(images), labels).backward()
            g_raw = np.concatenate([p.grad.numpy().reshape(-1) for p in shadow.parameters()])
            w0 = state_dict_to_row(model.state_dict())
            st = c.optimizer.state
            buf0 = (np.concatenate([st[p]["momentum_buffer"].numpy().reshape(-1) for p in model.parameters()])
                    if t > 0 and mom != 0 else np.zeros_like(w0))
            c.update_model(images, labels, theta)
            gp = np.concatenate([p.grad.numpy().reshape(-1) for p in model.parameters()])
            c.optimizer.step()
            w1 = state_dict_to_row(model.state_dict())
            buf1 = (np.concatenate([st[p]["momentum_buffer"].numpy().reshape(-1) for p in model.parameters()])
                    if mom != 0 else np.zeros_like(w0))
            for n, v in (("w", w0), ("buf", buf0), ("g", g_raw), ("gp", gp), ("w1", w1), ("buf1", buf1)):
                rec[n].append(v.astype(np.float32))
        key = f"{cname}__lr{lr}__mom{mom}"
        for n, v in rec.items():
            out[f"{key}__{n}"] = np.stack(v)
        out[f"{key}__theta"] = state_dict_to_row(theta)
        out[f"{key}__params"] = np.array([0.1, lr, mom], np.float64)
        if cname == "FedAdmm_Client":
            out[f"{key}__alpha"] = alpha0
            c.update_duals(theta)  # alpha += rho*(w - theta), w = final weights
            out[f"{key}__alpha1"] = state_dict_to_row(c.alpha)
            out[f"{key}__wfinal"] = state_dict_to_row(model.state_dict())
    return out


def gen_duals(dec_cli):
    """update_duals on random stacked inputs (mini layout, 5 agents)."""
    rng = np.random.default_rng(200)
    out = {}
    P = layout_size(MINI)
    for rho in (0.1, 0.01, 1.0):
        A = random_rows(rng, 5, P, special=True)
        Wt = random_rows(rng, 5, P, special=True)
        th = random_rows(rng, 1, P)[0]
        A1 = np.zeros_like(A)
        theta_sd = rows_to_state_dicts(th[None], MINI)[0]
        for k in range(5):
            c = _Obj(args=_Obj(rho=rho), model=_Model(rows_to_state_dicts(Wt[k:k + 1], MINI)[0]),
                     alpha=rows_to_state_dicts(A[k:k + 1], MINI)[0])
            dec_cli.FedAdmm_Client.update_duals(c, theta_sd)
            A1[k] = state_dict_to_row(c.alpha)
        key = f"rho{rho}"
        out.update({f"{key}__alpha": A, f"{key}__w": Wt, f"{key}__theta": th, f"{key}__alpha1": A1,
                    f"{key}__rho": np.array([rho])})
    return out


def gen_average(dec_srv):
    rng = np.random.default_rng(300)
    out = {}
    for name, m, layout in (("m7_mini", 7, MINI), ("m1_mini", 1, MINI), ("m10_flat1031", 10, FLAT_1031),
                            ("m3_flat4097", 3, FLAT_4097)):
        P = layout_size(layout)
        Wrows = random_rows(rng, m, P, special=True)
        sds = rows_to_state_dicts(Wrows, layout)
        theta = dec_srv.Server.average_weights(None, sds)
        out[f"{name}__W"] = Wrows
        out[f"{name}__theta"] = state_dict_to_row(theta)
    return out


def gen_host(dist_models, dist_sampling, dec_sampling):
    """Reference model init under a seed (layout + default-init RNG stream) and
    the user partitions (numpy RNG call sequence) on fixed synthetic labels."""
    out = {}
    for name in ("Model1", "Model3"):
        torch.manual_seed(2028)
        m = getattr(dist_models, name)()
        sd = m.state_dict()
        flat = np.concatenate([v.numpy().reshape(-1) for v in sd.values()])
        out[f"{name}__keys"] = np.array(list(sd.keys()))
        out[f"{name}__shapes"] = np.array([str(tuple(v.shape)) for v in sd.values()])
        out[f"{name}__sample"] = flat[::4999].copy()
        out[f"{name}__sum"] = np.array([flat.astype(np.float64).sum(), np.abs(flat.astype(np.float64)).sum()])
        out[f"{name}__P"] = np.array([flat.size])
    labels = np.random.default_rng(5).integers(0, 10, 1200)

    class _DS:
        def __init__(self, t):
            self.targets = torch.from_numpy(t)

        def __len__(self):
            return len(self.targets)

    ds = _DS(labels)
    for iid in (True, False):
        np.random.seed(77)
        args = _Obj(num_users=6, shards=2)
        g = dist_sampling.iid_split(ds, args) if iid else dist_sampling.noniid_split(ds, args)
        for u in range(6):
            out[f"dist_iid{iid}__u{u}"] = np.array(sorted(float(i) for i in g[u]))
            if not iid:
                out[f"dist_iid{iid}__u{u}__order"] = np.asarray(g[u], np.float64)
        out[f"dist_iid{iid}__after"] = np.random.random(3)
    np.random.seed(78)
    g = dec_sampling.mnist_iid(ds, 10)
    for u in range(10):
        out[f"dec_iid__u{u}"] = np.array(sorted(int(i) for i in g[u]))
    out["dec_iid__after"] = np.random.random(3)
    return out


def main():
    _placeholder_torchvision()
    dist = _import_project(DIST_SRC, ["simulators", "clients", "models", "sampling"])
    graphs, csr = gen_graphs(dist["simulators"])
    mix = gen_mix(dist["simulators"], dist["clients"], graphs)
    dist_models, dist_sampling = dist["models"], dist["sampling"]
    dec = _import_project(DEC_SRC, ["servers", "clients", "sampling"])
    host = gen_host(dist_models, dist_sampling, dec["sampling"])
    local = gen_local_steps(dec["clients"])
    duals = gen_duals(dec["clients"])
    avg = gen_average(dec["servers"])
    meta = dict(torch=torch.__version__, numpy=np.__version__, graph_seed=GRAPH_SEED)
    np.savez_compressed(os.path.join(OUT, "graphs.npz"), **{k: v for k, v in graphs.items()})
    np.savez_compressed(os.path.join(OUT, "csr.npz"), **csr)
    np.savez_compressed(os.path.join(OUT, "mix.npz"), **mix)
    np.savez_compressed(os.path.join(OUT, "local_steps.npz"), **local)
    np.savez_compressed(os.path.join(OUT, "duals.npz"), **duals)
    np.savez_compressed(os.path.join(OUT, "average.npz"), **avg)
    np.savez_compressed(os.path.join(OUT, "host.npz"), **host)
    with open(os.path.join(OUT, "META.txt"), "w") as f:
        for k, v in meta.items():
            f.write(f"{k}={v}\n")
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
