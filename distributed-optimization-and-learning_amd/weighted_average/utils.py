"""DotDict / setup_seed / DatasetSplit / get_dataset of the gossip project
(DIST/utils.py).  Plotting helpers are out of scope (not on the hot path)."""
import _engine  # noqa: F401
from dolhip.agent import DotDict, setup_seed  # noqa: F401
from dolhip.data import DatasetSplit, load_pair  # noqa: F401
from sampling import iid_split, noniid_split


def get_dataset(args):
    """(train, test, user_groups) — DIST/utils.py:72-106; dataset='synthetic'
    works offline (no torchvision / network needed)."""
    if args.verbose:
        print(f"\n | Download Dataset {args.dataset} |")
    train, test = load_pair(args)
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
