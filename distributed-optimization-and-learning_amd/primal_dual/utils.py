"""DotDict / setup_seed / DatasetSplit / get_dataset / servers_plot of the
federated project (DEC/utils.py).  Host-side; not on the hot path."""
import _engine  # noqa: F401
from dolhip.agent import DotDict, setup_seed  # noqa: F401
from dolhip.data import DatasetSplit, load_pair  # noqa: F401
from sampling import mnist_iid, mnist_noniid, cifar_iid, cifar_noniid


def servers_plot(servers, clients, frac, iid):
    """2x2 comparison figure of several servers' `history` (DEC/utils.py:29-51):
    mean train accuracy / loss over clients and the global model's test accuracy /
    loss per round, one line per server named after its class without
    '_Server' (PD.ipynb cell[27])."""
    import matplotlib.pyplot as plt
    import pandas as pd

    title = "| {} Clients | frac: {} | iid: {} |".format(clients, frac, iid)
    fig, axs = plt.subplots(2, 2, figsize=(30, 15))
    fig.suptitle(title, fontsize=36)
    panels = (((0, 0), "Average train accuracy of all clients", "Average Accuracy", "train_acc"),
              ((0, 1), "Average training loss of clients in a round", "Training loss", "train_loss"),
              ((1, 0), "Test Accuracy of Global model", "test_acc", "test_acc"),
              ((1, 1), "Test Loss of Global model", "test_loss", "test_loss"))
    for (r, c), head, ylabel, _ in panels:
        axs[r, c].set_title(head, fontsize=22)
        axs[r, c].set_ylabel(ylabel)
    for server in servers:
        hist = pd.DataFrame(server.history)
        name = type(server).__name__.replace("_Server", "")
        for (r, c), _, _, column in panels:
            axs[r, c].plot(hist[column], label=name)
    for ax in axs.flat:
        ax.set(xlabel="Communication rounds")
        ax.legend()
    plt.show()
    return fig


def get_dataset(args):
    """(train, test, user_groups) — DEC/utils.py:97-144 (dataset='synthetic'
    / 'synthetic-cifar' works offline)."""
    train, test = load_pair(args, "dec")
    # only "cifar10" takes the cifar splits (DEC/utils.py:98-111); the synthetic stand-in too
    cifar = args.dataset == "cifar10" or str(args.dataset).endswith("cifar")
    if args.iid:
        groups = (cifar_iid if cifar else mnist_iid)(train, args.num_users)
    else:
        groups = (cifar_noniid if cifar else mnist_noniid)(train, args.num_users)
    return train, test, groups


def exp_details(args):
    print("\nExperimental details:")
    for label, key in (("Model", "model"), ("Optimizer", "optimizer"), ("Global Rounds", "epochs"),
                       ("dataset", "dataset"), ("Num of users", "num_users"), ("Fraction of users", "frac"),
                       ("Learning  Rate", "lr"), ("rho", "rho"), ("Local Epochs", "local_ep"),
                       ("Local Batch size", "local_bs")):
        print(f"    {label:<18} : {args.get(key)}")
    print("    IID" if args.iid else "    Non-IID")
