"""Host-side data plumbing the drop-in needs (OUT of the hot path).

Datasets are loaded once per run on the host; the reference downloads them
with torchvision (DIST/utils.py:72-106, DEC/utils.py:97-144).  torchvision and
the network may be absent, so `dataset='synthetic'` (or 'synthetic-cifar')
gives a seeded MNIST/CIFAR-shaped dataset whose generation consumes NO global
RNG.  The user splits consume the global numpy RNG exactly as the reference
does (same np.random.choice calls in the same order), so seeded drop-in runs
partition users identically.
"""
from __future__ import annotations

from typing import Dict, Sequence

import numpy as np
import torch
from torch.utils.data import Dataset


class SyntheticImages(Dataset):
    """Seeded image-classification data: class-dependent means + noise."""

    def __init__(self, n: int, shape=(1, 28, 28), classes: int = 10, seed: int = 0):
        rng = np.random.default_rng(seed)
        self.targets = torch.from_numpy(rng.integers(0, classes, n).astype(np.int64))
        centers = rng.standard_normal((classes,) + tuple(shape)).astype(np.float32)
        noise = rng.standard_normal((n,) + tuple(shape)).astype(np.float32)
        self.data = torch.from_numpy(centers[self.targets.numpy()] + 0.8 * noise)

    def __len__(self) -> int:
        return int(self.targets.shape[0])

    def __getitem__(self, i):
        return self.data[i], int(self.targets[i])


class DatasetSplit(Dataset):
    """Index view of a dataset (DIST/utils.py:59-69, DEC/utils.py:84-94)."""

    def __init__(self, dataset, idxs: Sequence[int]):
        self.dataset = dataset
        self.idxs = [int(i) for i in idxs]

    def __len__(self) -> int:
        return len(self.idxs)

    def __getitem__(self, item):
        image, label = self.dataset[self.idxs[item]]
        return torch.as_tensor(image), torch.as_tensor(label)


def iid_split(n_items: int, num_users: int) -> Dict[int, set]:
    """Equal random disjoint index sets (DIST/sampling.py:3-9, DEC/sampling.py:5-12)."""
    per = int(n_items / num_users)
    remaining = list(range(n_items))
    groups = {}
    for u in range(num_users):
        groups[u] = set(np.random.choice(remaining, per, replace=False))
        remaining = list(set(remaining) - groups[u])
    return groups


def shard_split(targets, num_users: int, shards_per_user: int, num_shards: int, imgs_per_shard: int):
    """Label-sorted shards dealt to users (DIST/sampling.py:11-28 with
    shards_per_user = args.shards; DEC/sampling.py:15-76 with 2 per user)."""
    labels = np.asarray(targets)[: num_shards * imgs_per_shard]
    order = np.vstack((np.arange(num_shards * imgs_per_shard), labels))
    order = order[:, order[1, :].argsort()][0, :]
    free = list(range(num_shards))
    groups = {u: np.array([]) for u in range(num_users)}
    for u in range(num_users):
        picked = set(np.random.choice(free, shards_per_user, replace=False))
        free = list(set(free) - picked)
        for s in picked:
            groups[u] = np.concatenate((groups[u], order[s * imgs_per_shard:(s + 1) * imgs_per_shard]), axis=0)
    return groups


def synthetic_pair(name: str, n_train: int = 6000, n_test: int = 1000, seed: int = 1234):
    shape = (3, 32, 32) if name.endswith("cifar") else (1, 28, 28)
    return (SyntheticImages(n_train, shape, 10, seed), SyntheticImages(n_test, shape, 10, seed + 1))


def dataset_spec(name: str, project: str):
    """(torchvision class name, data_dir, Normalize mean, Normalize std) exactly
    as each project's get_dataset picks them.

    * project "dist" (DIST/utils.py:72-95): dir ``../data/<name>/``; cifar10 /
      cifar100 (0.5,)*3; mnist (0.1307,)/(0.3081,); fmnist (0.5,)*3 — three
      channels on a 1-channel image, which torchvision's in-place Normalize
      rejects at the first item, as in the reference.  Any other name leaves
      the reference's train_dataset unbound (UnboundLocalError); here a
      ValueError.
    * project "dec" (DEC/utils.py:97-137): cifar10 in ``../data/cifar/``;
      every other name takes the mnist/fmnist branch (``args.dataset ==
      'mnist' or 'fmnist'`` is always true): mnist in ``../data/mnist/``,
      anything else FashionMNIST in ``../data/fmnist/`` — both with the MNIST
      statistics (0.1307,)/(0.3081,).
    """
    half3, mnist = ((0.5, 0.5, 0.5), (0.5, 0.5, 0.5)), ((0.1307,), (0.3081,))
    if project == "dist":
        table = {"cifar10": ("CIFAR10",) + half3, "cifar100": ("CIFAR100",) + half3,
                 "mnist": ("MNIST",) + mnist, "fmnist": ("FashionMNIST",) + half3}
        if name not in table:
            raise ValueError(f"unknown dataset '{name}' (DIST/utils.py:76-95 knows {sorted(table)})")
        cls, mean, std = table[name]
        return cls, f"../data/{name}/", mean, std
    if project == "dec":
        if name == "cifar10":
            return ("CIFAR10", "../data/cifar/") + half3
        if name == "mnist":
            return ("MNIST", "../data/mnist/") + mnist
        return ("FashionMNIST", "../data/fmnist/") + mnist
    raise ValueError(f"project must be 'dist' or 'dec', not {project!r}")


def torchvision_pair(name: str, project: str):
    cls, root, mean, std = dataset_spec(name, project)
    try:
        from torchvision import datasets, transforms
    except ImportError as e:  # no torchvision in this image: say what to use instead
        raise ImportError(f"dataset '{name}' needs torchvision (not installed); use dataset='synthetic'") from e
    tf = transforms.Compose([transforms.ToTensor(), transforms.Normalize(mean, std)])
    ctor = getattr(datasets, cls)
    return (ctor(root, train=True, download=True, transform=tf), ctor(root, train=False, download=True, transform=tf))


def load_pair(args, project: str):
    """(train, test) for one project ('dist' = weighted_average, 'dec' =
    primal_dual); 'synthetic*' names work offline."""
    name = args.dataset or "mnist"
    if str(name).startswith("synthetic"):
        return synthetic_pair(name, args.synthetic_train or 6000, args.synthetic_test or 1000,
                              args.synthetic_seed if args.synthetic_seed is not None else 1234)
    return torchvision_pair(name, project)
