"""Multi-rank logic on CPU with the gloo backend (world sizes 2 and 3).

The kernels are the HIP ops in production; here the sharding, halo exchange,
boundary-row handling and ordered chain reduce are exercised with the CPU
oracle injected as the arithmetic (the checker), and the gathered result is
compared bit-for-bit with a single-process oracle run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from dolhip import parallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def cpu_mix_ring(X, Y, w_prev, w_next, halo_prev=None, halo_next=None, P=None, n_rows=None):
    n = X.shape[0] if n_rows is None else n_rows
    P = X.shape[1] if P is None else P
    hp = None if halo_prev is None else halo_prev[:P].numpy()
    hn = None if halo_next is None else halo_next[:P].numpy()
    out = oracle.mix_ring(X[:n, :P].numpy(), w_prev[:n].numpy(), w_next[:n].numpy(), hp, hn)
    Y[:n, :P] = torch.from_numpy(out)
    return Y


def cpu_ordered_sum(W, order, acc_in=None, out=None, scale=1.0, P=None):
    if W is None or order.numel() == 0:
        res = acc_in[:P].numpy().astype(np.float32)
        if scale != 1.0:
            res = (res / np.float32(scale)).astype(np.float32)
    else:
        res = oracle.ordered_sum(W[:, :P].numpy(), order.numpy(),
                                 None if acc_in is None else acc_in[:P].numpy(), scale)
    out[:P] = torch.from_numpy(res)
    return out


def _worker(rank, world, port, N, P, rounds, order, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(11)
        X = rng.standard_normal((N, P)).astype(np.float32)
        wp = rng.random(N).astype(np.float32)
        wn = rng.random(N).astype(np.float32)
        ring = parallel.ShardedRing(N, P, wp, wn, "cpu", ld=P + 3, mix_ring=cpu_mix_ring)
        ring.x[:, :P] = torch.from_numpy(X[ring.lo:ring.hi])
        for _ in range(rounds):
            ring.step()
        mixed = ring.x[:, :P].clone()
        exact = parallel.global_mean_exact(ring.x, ring.lo, ring.hi, order, P, ordered_sum=cpu_ordered_sum)
        local = [g - ring.lo for g in order if ring.lo <= g < ring.hi]
        fast = parallel.global_mean(ring.x, local, len(order), P, ordered_sum=cpu_ordered_sum)
        q.put((rank, ring.lo, ring.hi, mixed.numpy(), exact.numpy()[:P].copy(), fast.numpy()[:P].copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N", [(2, 10), (3, 11), (2, 4)])
def test_sharded_ring_and_means_match_single_process(world, N):
    P, rounds = 37, 3
    order = [7 % N, 0, N - 1, 3, 1, 2]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, P, rounds, order, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    # single-process reference run of the same arithmetic
    rng = np.random.default_rng(11)
    X = rng.standard_normal((N, P)).astype(np.float32)
    wp = rng.random(N).astype(np.float32)
    wn = rng.random(N).astype(np.float32)
    for _ in range(rounds):
        X = oracle.mix_ring(X, wp, wn)
    got = np.concatenate([r[3] for r in res])
    assert oracle.bits_equal(got, X)
    want_mean = oracle.ordered_mean(X, np.array(order))
    for r in res:
        assert oracle.bits_equal(r[4], want_mean)  # exact chain: bit-identical on every rank
        np.testing.assert_allclose(r[5], want_mean, rtol=1e-5, atol=1e-6)  # all_reduce form
