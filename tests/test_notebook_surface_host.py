"""The notebooks' own import lines and plotting calls against the drop-in
(host side, matplotlib Agg backend; no GPU).

WA.ipynb cell[9] and PD.ipynb cell[6] are executed verbatim (minus the IPython
magics) with the project directory on sys.path, the way the notebooks run from
`src/`.  The plots are then drawn from history rows in the exact schema the
drop-in's run loops append (checked against a real run in
tests/test_dropin_gpu.py::test_notebook_plots_after_one_round)."""
import math
import os
import sys
import types

import matplotlib
import pytest

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402

from conftest import PKG, PROJECT_MODULES  # noqa: E402

WA_CELL9 = """
import matplotlib.pyplot as plt
from simulators import NoConsDecFedAvg,DecFedAvg,Centeralized,FedLCon,GossipLearning
from utils import DotDict, servers_plot
import pandas as pd
import torch
import copy
"""

PD_CELL6 = """
import copy
import torch
from utils import DotDict,servers_plot
from servers import FedAdmm_Server, FedAvg_Server,FedProx_Server
import pandas as pd
import matplotlib.pyplot as plt
"""


def _run_cell(project, src):
    for m in PROJECT_MODULES:
        sys.modules.pop(m, None)
    path = os.path.join(PKG, project)
    sys.path.insert(0, path)
    try:
        ns = {}
        exec(compile(src, f"<{project} notebook cell>", "exec"), ns)
        return ns
    finally:
        sys.path.remove(path)


@pytest.fixture(autouse=True)
def _close_figures():
    yield
    plt.close("all")


def _wa_history(rounds, scale):
    return [{"round": r, "avg_test_acc": 0.1 * scale * (r + 1), "avg_test_loss": 2.0 - 0.1 * r,
             "avg_train_loss": 2.1 - 0.1 * r} for r in range(rounds)]


def test_wa_notebook_imports_and_servers_plot():
    ns = _run_cell("weighted_average", WA_CELL9)
    for name in ("NoConsDecFedAvg", "DecFedAvg", "Centeralized", "FedLCon", "GossipLearning", "DotDict"):
        assert name in ns
    args = ns["DotDict"](rounds=10)
    assert args.rounds == 10 and args.mode is None
    sims = [types.SimpleNamespace(history=_wa_history(3, s)) for s in (1, 2)]
    # WA.ipynb cell[39]: a history read back from CSV is a DataFrame
    sims.append(types.SimpleNamespace(history=ns["pd"].DataFrame(_wa_history(3, 3))))
    fig = ns["servers_plot"](sims, 10, 8, False, ["centeral", "no_cons_dec_iid", "no_cons_dec_non_iid"])
    axs = fig.axes
    assert len(axs) == 4
    assert fig._suptitle.get_text() == "| 10 Clients | frac: 8 | iid: False |"
    assert [len(a.lines) for a in axs] == [0, 3, 3, 3]  # train-accuracy panel empty, as the reference
    assert [ln.get_label() for ln in axs[1].lines] == ["centeral", "no_cons_dec_iid", "no_cons_dec_non_iid"]
    assert list(axs[2].lines[1].get_ydata()) == [h["avg_test_acc"] for h in _wa_history(3, 2)]


def _pd_server(cls, rounds):
    s = cls.__new__(cls)
    s.history = [{"round": r, "test_acc": 0.5 + 0.1 * r, "test_loss": 30.0 - r, "train_loss": 2.0 - 0.1 * r,
                  "train_acc": 0.4 + 0.1 * r} for r in range(rounds)]
    return s


def test_pd_notebook_imports_and_servers_plot():
    ns = _run_cell("primal_dual", PD_CELL6)
    servers = [_pd_server(ns[n], 4) for n in ("FedAvg_Server", "FedProx_Server", "FedAdmm_Server")]
    # PD.ipynb cell[27]
    fig = ns["servers_plot"](servers, 100, 0.1, True)
    axs = fig.axes
    assert fig._suptitle.get_text() == "| 100 Clients | frac: 0.1 | iid: True |"
    assert [len(a.lines) for a in axs] == [3, 3, 3, 3]
    assert [ln.get_label() for ln in axs[0].lines] == ["FedAvg", "FedProx", "FedAdmm"]
    assert list(axs[3].lines[2].get_ydata()) == [30.0, 29.0, 28.0, 27.0]


def _client_history(rounds, local_ep):
    return [{"global_round": r, "epoch": e, "train_loss": 1.0, "train_acc": 0.5, "val_acc": 0.6, "val_loss": 0.9}
            for r in range(rounds) for e in range(local_ep)]


@pytest.mark.parametrize("n", [100, 10, 7, 1])
def test_pd_server_plot(n):
    """Server.plot (DEC/servers.py:95-120) for the notebook's n = 100 (PD.ipynb
    cells 15/20/25) and for non-square n, where the reference indexes past its
    last client; never-sampled clients (no history) get empty panels."""
    ns = _run_cell("primal_dual", PD_CELL6)
    srv = ns["FedAdmm_Server"].__new__(ns["FedAdmm_Server"])
    srv.args = ns["DotDict"](num_users=n)
    srv.clients = [types.SimpleNamespace(history=_client_history(2, 3) if c % 3 else []) for c in range(n)]
    fig = srv.plot()
    s = math.ceil(math.sqrt(n))
    axs = fig.axes
    assert len(axs) == 2 * s * s
    for c in range(n):
        block, j = divmod(c, s)
        loss_ax, acc_ax = axs[2 * block * s + j], axs[(2 * block + 1) * s + j]
        assert loss_ax.get_title() == "Client #%d" % (c + 1)
        assert len(loss_ax.lines) == (2 if c % 3 else 0)
        assert len(acc_ax.lines) == (2 if c % 3 else 0)
        if c % 3:
            assert [ln.get_label() for ln in acc_ax.lines] == ["train", "val"]


def test_dataset_spec_per_project():
    """Each project's torchvision class, data dir and Normalize statistics
    (DIST/utils.py:72-95 vs DEC/utils.py:97-137), as the advisor flagged."""
    from dolhip.data import dataset_spec
    mn, half3 = ((0.1307,), (0.3081,)), ((0.5,) * 3, (0.5,) * 3)
    assert dataset_spec("mnist", "dist") == ("MNIST", "../data/mnist/") + mn
    assert dataset_spec("fmnist", "dist") == ("FashionMNIST", "../data/fmnist/") + half3
    assert dataset_spec("cifar10", "dist") == ("CIFAR10", "../data/cifar10/") + half3
    assert dataset_spec("cifar100", "dist") == ("CIFAR100", "../data/cifar100/") + half3
    with pytest.raises(ValueError):
        dataset_spec("svhn", "dist")
    assert dataset_spec("mnist", "dec") == ("MNIST", "../data/mnist/") + mn
    assert dataset_spec("fmnist", "dec") == ("FashionMNIST", "../data/fmnist/") + mn
    assert dataset_spec("cifar10", "dec") == ("CIFAR10", "../data/cifar/") + half3
    # `args.dataset == 'mnist' or 'fmnist'` is always true: any other name is FashionMNIST
    assert dataset_spec("cifar100", "dec") == ("FashionMNIST", "../data/fmnist/") + mn
