"""User partitions of the federated project (DEC/sampling.py): same numpy RNG
call sequence as the reference.  The shard tables are the reference's; for a
dataset smaller than the table (e.g. synthetic data) the image count per
shard shrinks to fit."""
import numpy as np

import _engine  # noqa: F401
from dolhip.data import iid_split, shard_split

_MNIST = {100: (200, 300), 200: (400, 150), 500: (1000, 60)}
_CIFAR = {100: (200, 250), 200: (400, 125), 500: (1000, 50)}


def _noniid(dataset, num_users, table, default):
    num_shards, num_imgs = table.get(num_users, default)
    num_imgs = min(num_imgs, len(dataset) // num_shards)
    return shard_split(np.asarray(dataset.targets), num_users, 2, num_shards, num_imgs)


def mnist_iid(dataset, num_users):
    return iid_split(len(dataset), num_users)


def mnist_noniid(dataset, num_users):
    return _noniid(dataset, num_users, _MNIST, (2000, 30))


def cifar_iid(dataset, num_users):
    return iid_split(len(dataset), num_users)


def cifar_noniid(dataset, num_users):
    return _noniid(dataset, num_users, _CIFAR, (2000, 25))
