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


def torchvision_pair(name: str, root: str):
    try:
        from torchvision import datasets, transforms  # noqa: F401
    except ImportError as e:  # no torchvision in this image: say what to use instead
        raise ImportError(f"dataset '{name}' needs torchvision (not installed); use dataset='synthetic'") from e
    if name == "cifar10":
        tf = transforms.Compose([transforms.ToTensor(), transforms.Normalize((0.5,) * 3, (0.5,) * 3)])
        return (datasets.CIFAR10(root, train=True, download=True, transform=tf),
                datasets.CIFAR10(root, train=False, download=True, transform=tf))
    if name == "cifar100":
        tf = transforms.Compose([transforms.ToTensor(), transforms.Normalize((0.5,) * 3, (0.5,) * 3)])
        return (datasets.CIFAR100(root, train=True, download=True, transform=tf),
                datasets.CIFAR100(root, train=False, download=True, transform=tf))
    if name == "fmnist":
        tf = transforms.Compose([transforms.ToTensor(), transforms.Normalize((0.5,), (0.5,))])
        return (datasets.FashionMNIST(root, train=True, download=True, transform=tf),
                datasets.FashionMNIST(root, train=False, download=True, transform=tf))
    tf = transforms.Compose([transforms.ToTensor(), transforms.Normalize((0.1307,), (0.3081,))])
    return (datasets.MNIST(root, train=True, download=True, transform=tf),
            datasets.MNIST(root, train=False, download=True, transform=tf))


def load_pair(args):
    name = args.dataset or "mnist"
    if str(name).startswith("synthetic"):
        return synthetic_pair(name, args.synthetic_train or 6000, args.synthetic_test or 1000,
                              args.synthetic_seed if args.synthetic_seed is not None else 1234)
    return torchvision_pair(name, f"../data/{name}/")
