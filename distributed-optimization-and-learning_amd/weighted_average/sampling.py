"""User partitions of the gossip project (DIST/sampling.py): same numpy RNG
call sequence as the reference, so seeded runs split users identically."""
import numpy as np

import _engine  # noqa: F401
from dolhip.data import iid_split as _iid, shard_split as _shards


def iid_split(dataset, args):
    return _iid(len(dataset), args.num_users)


def noniid_split(dataset, args):
    num_shards = args.shards * args.num_users
    t = dataset.targets
    return _shards(t.numpy().copy() if hasattr(t, "numpy") else np.array(t), args.num_users, args.shards, num_shards,
                   len(dataset) // num_shards)
