"""Golden FedADMM least-squares trajectories from the REFERENCE (build container
only; needs /root/reference):   python tests/golden/make_golden_admm.py

Runs the shipped FedAdmm_Server.run (DEC/servers.py:50-81) unchanged —
np.random.choice client sampling, FedAdmm_Client.update_weights with its
update_model / optimizer.step / update_duals (DEC/clients.py:36-53, :125-144),
average_weights (DEC/servers.py:42-48) and load_state_dict — on a
least-squares "model" instead of the CNN, which is what dol_admm_ls_round_f32
computes (BASELINE config 4's primal/dual side).  Three things are swapped in
through the reference's own extension points, nothing of its code is edited:
  * servers.Model1 -> LSModel: its parameters ARE the agent's w (several keys,
    so multi-key flattening is exercised); forward returns them as a [1, P] row;
  * servers.get_dataset -> a dataset whose item i carries the target row t_k
    of the user k that owns index i (user split: the reference's mnist_iid);
  * each client's criterion -> 0.5*sum((out - t)**2) with t = labels[0], so
    autograd's gradient is exactly fl(w - t).
Recorded (npz, no pickles): the targets, theta_0, every round's sampled order
and theta, and the final per-client w, momentum buffer and alpha rows.
torchvision: placeholder module only (unused by these paths).
"""
import contextlib
import io
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import DEC_SRC, _import_project, _placeholder_torchvision  # noqa: E402

LAYOUTS = {
    "mini": [("a.weight", (5, 3)), ("a.bias", (7,)), ("b.weight", (33, 4))],
    "flat1031": [("w", (1031,))],
}
# name -> (layout, num_users, frac, rounds, local_ep, items per user, local_bs, lr, momentum, rho, seed)
CASES = {
    "mini_mom": ("mini", 10, 0.3, 4, 2, 9, 4, 0.1, 0.5, 0.1, 2022),
    "flat_nomom": ("flat1031", 6, 0.5, 3, 1, 10, 3, 0.05, 0.0, 0.5, 7),
    "mini_full": ("mini", 5, 1.0, 3, 3, 6, 5, 0.2, 0.9, 0.01, 11),
}


def make_model_cls(layout):
    class LSModel(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.ps = torch.nn.ParameterDict()
            for k, shape in layout:
                self.ps[k.replace(".", "_")] = torch.nn.Parameter(torch.randn(*shape))

        def forward(self, x):
            return torch.cat([p.reshape(-1) for p in self.ps.values()]).view(1, -1)

    return LSModel


def ls_criterion(out, labels):
    return 0.5 * ((out - labels[:1]) ** 2).sum()


class _TargetSet:
    """Item i = (dummy image, target row of the user owning i)."""

    def __init__(self, n, P):
        self.n, self.P = n, P
        self.owner_targets = None

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return np.zeros(1, np.float32), self.owner_targets[i]


def flat(sd):
    return torch.cat([v.detach().reshape(-1).float() for v in sd.values()]).numpy()


def run_case(name):
    layout, N, frac, rounds, local_ep, items, bs, lr, mom, rho, seed = CASES[name]
    lay = LAYOUTS[layout]
    P = int(sum(np.prod(s) for _, s in lay))
    mods = _import_project(DEC_SRC, ["utils", "sampling", "servers"])
    U, S, srv = mods["utils"], mods["sampling"], mods["servers"]
    rng = np.random.default_rng(1000 + seed)
    targets = rng.standard_normal((N, P)).astype(np.float32)
    n_train = N * items

    def get_dataset(args):
        train, test = _TargetSet(n_train, P), _TargetSet(4, P)
        groups = S.mnist_iid(train, args.num_users)
        owner = np.zeros((n_train, P), np.float32)
        for u, idxs in groups.items():
            for i in idxs:
                owner[int(i)] = targets[u]
        train.owner_targets = owner
        test.owner_targets = np.zeros((4, P), np.float32)
        return train, test, groups

    srv.get_dataset = get_dataset
    srv.Model1 = make_model_cls(lay)
    args = U.DotDict(dict(num_users=N, local_ep=local_ep, local_bs=bs, lr=lr, model="Model1", dataset="synthetic",
                          iid=True, rho=rho, seed=seed, momentum=mom, verbose=False, device="cpu"))
    orders, thetas = [], []
    choice = np.random.choice

    def recording_choice(*a, **kw):
        r = choice(*a, **kw)
        orders.append(np.asarray(r, np.int64))
        return r

    with contextlib.redirect_stdout(io.StringIO()):
        s = srv.FedAdmm_Server(args)
        for c in s.clients + [s.global_client]:
            c.criterion = ls_criterion
        theta0 = flat(s.global_client.model.state_dict())
        steps = [len(c.loaders["train"]) for c in s.clients]
        np.random.choice = recording_choice
        try:
            for _ in range(rounds):
                s.run(frac, 1)
                thetas.append(flat(s.global_client.model.state_dict()))
        finally:
            np.random.choice = choice
    assert len(set(steps)) == 1, steps
    first_mom = []
    for c in s.clients:
        st = c.optimizer.state
        ps = list(c.model.parameters())
        first_mom.append(np.concatenate([st[p]["momentum_buffer"].numpy().reshape(-1) if p in st and
                                         st[p].get("momentum_buffer") is not None else np.zeros(p.numel(), np.float32)
                                         for p in ps]))
    key = name
    return {
        f"{key}__targets": targets, f"{key}__theta0": theta0, f"{key}__orders": np.stack(orders),
        f"{key}__thetas": np.stack(thetas), f"{key}__w": np.stack([flat(c.model.state_dict()) for c in s.clients]),
        f"{key}__mom": np.stack(first_mom).astype(np.float32),
        f"{key}__alpha": np.stack([flat(c.alpha) for c in s.clients]),
        f"{key}__params": np.array([N, frac, rounds, local_ep * steps[0], lr, mom, rho], np.float64),
    }


def main():
    _placeholder_torchvision()
    out = {}
    for name in CASES:
        out.update(run_case(name))
    np.savez_compressed(os.path.join(HERE, "admm_ls.npz"), **out)
    print("wrote admm_ls.npz", sorted(k for k in out if k.endswith("__params")))


if __name__ == "__main__":
    main()
