"""DotDict / setup_seed / DatasetSplit / get_dataset of the federated project
(DEC/utils.py).  Plotting is out of scope (not on the hot path)."""
import _engine  # noqa: F401
from dolhip.agent import DotDict, setup_seed  # noqa: F401
from dolhip.data import DatasetSplit, load_pair  # noqa: F401
from sampling import mnist_iid, mnist_noniid, cifar_iid, cifar_noniid


def get_dataset(args):
    """(train, test, user_groups) — DEC/utils.py:97-144 (dataset='synthetic'
    / 'synthetic-cifar' works offline)."""
    train, test = load_pair(args)
    cifar = str(args.dataset).startswith("cifar") or str(args.dataset).endswith("cifar")
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
