"""DotDict / setup_seed / DatasetSplit / get_dataset / servers_plot of the
gossip project (DIST/utils.py).  Host-side; not on the hot path."""
import _engine  # noqa: F401
from dolhip.agent import DotDict, setup_seed  # noqa: F401
from dolhip.data import DatasetSplit, load_pair  # noqa: F401
from sampling import iid_split, noniid_split


def servers_plot(servers, clients, frac, iid, labels):
    """2x2 comparison figure of several simulators' `history` (DIST/utils.py:26-48):
    average train loss, test accuracy and test loss per communication round, one
    line per simulator named by `labels[i]` (the train-accuracy panel stays empty,
    as in the reference).  `server.history` may be the list of dicts `run()`
    appends or a DataFrame read back from the CSV (WA.ipynb cell[38])."""
    import matplotlib.pyplot as plt
    import pandas as pd

    title = "| {} Clients | frac: {} | iid: {} |".format(clients, frac, iid)
    fig, axs = plt.subplots(2, 2, figsize=(30, 15))
    fig.suptitle(title, fontsize=36)
    panels = (((0, 0), "Average train accuracy of all clients", "Average Accuracy", None),
              ((0, 1), "Average training loss of clients in a round", "Training loss", "avg_train_loss"),
              ((1, 0), "Average Test Accuracy of all clients", "test_acc", "avg_test_acc"),
              ((1, 1), "Average Test Loss of all clients", "test_loss", "avg_test_loss"))
    for (r, c), head, ylabel, _ in panels:
        axs[r, c].set_title(head, fontsize=22)
        axs[r, c].set_ylabel(ylabel)
    for i, server in enumerate(servers):
        hist = pd.DataFrame(server.history)
        for (r, c), _, _, column in panels:
            if column is not None:
                axs[r, c].plot(hist[column], label=labels[i])
    for ax in axs.flat:
        ax.set(xlabel="Communication rounds")
        ax.legend()
    plt.show()
    return fig


def get_dataset(args):
    """(train, test, user_groups) — DIST/utils.py:72-106; dataset='synthetic'
    works offline (no torchvision / network needed)."""
    if args.verbose:
        print(f"\n | Download Dataset {args.dataset} |")
    train, test = load_pair(args, "dist")
    groups = iid_split(train, args) if args.iid else noniid_split(train, args)
    return train, test, groups


def exp_details(args):
    print("\n | Parameters details |")
    for label, key in (("Model", "model"), ("Optimizer", "optimizer"), ("Global Rounds", "epochs"),
                       ("Dataset", "dataset"), ("Num of users", "num_users"), ("Fraction of users", "frac"),
                       ("Learning  Rate", "lr"), ("Rho", "rho"), ("Local Epochs", "local_ep"),
                       ("Local Batch size", "local_bs"), ("Random Seed", "seed")):
        print(f"    {label:<20}: {args.get(key)}")
    print("    IID" if args.iid else "    Non-IID")
