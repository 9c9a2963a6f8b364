"""Bit-exactness at Model1's real 8-key layout (P = 1,663,370; SURVEY §7's
minimum slice N = 6 / 16): one mixing round for circle / complete /
double-stochastic circle W, update_duals and the ordered average, against
digests of the REFERENCE's own outputs (tests/golden/model1.json, made by
tests/golden/make_golden_model1.py; inputs regenerated here from the recorded
seeds).  CPU tier: the oracle; GPU tier: the HIP kernels through the C-ABI."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

import oracle
from conftest import GOLDEN
from dolhip import graph as G

M1 = json.load(open(os.path.join(GOLDEN, "model1.json")))
P = M1["P"]


def inputs(seed, n):
    return np.random.default_rng(seed).standard_normal((n, P), dtype=np.float32)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()


def graph_csr(c):
    torch.manual_seed(M1["graph_seed"])
    return G.csr_from_dense(G.communication_graph(c["topology"], c["mode"], c["n"])[0])


def test_layout_is_model1():
    from dolhip.models import Model1
    assert [[k, list(v.shape)] for k, v in Model1().state_dict().items()] == M1["layout"]


@pytest.mark.parametrize("key", sorted(M1["mix"]))
def test_oracle_mix_model1(key):
    c = M1["mix"][key]
    X = inputs(c["seed"], c["n"])
    csr = graph_csr(c)
    assert sha(oracle.mix_csr(X, csr.rowptr, csr.col, csr.val)) == c["Y"]["sha256"]


@pytest.mark.parametrize("n", ["6", "16"])
def test_oracle_duals_and_average_model1(n):
    d, a = M1["duals"][n], M1["average"][n]
    A, Wt = inputs(d["seeds"]["alpha"], d["n"]), inputs(d["seeds"]["w"], d["n"])
    th = inputs(d["seeds"]["theta"], 1)[0]
    a1, _ = oracle.admm_dual(A, Wt, th, np.float32(d["rho"]))
    assert sha(a1) == d["alpha1"]["sha256"]
    assert sha(oracle.ordered_mean(Wt, np.array(a["order"]))) == a["theta"]["sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("key", sorted(M1["mix"]))
def test_kernel_mix_model1(key, gpu):
    from dolhip.bank import AgentBank
    c = M1["mix"][key]
    X = inputs(c["seed"], c["n"])
    bank = AgentBank(c["n"], [(k, tuple(s)) for k, s in M1["layout"]], gpu)
    bank.rows()[:] = torch.from_numpy(X).to(gpu)
    plan = G.MixingPlan(graph_csr(c), gpu)
    bank.mix(plan)
    assert sha(bank.rows().cpu().numpy()) == c["Y"]["sha256"], plan.kind


@pytest.mark.gpu
@pytest.mark.parametrize("n", ["6", "16"])
def test_kernel_duals_and_average_model1(n, gpu):
    from dolhip import ops
    d, a = M1["duals"][n], M1["average"][n]
    A = torch.from_numpy(inputs(d["seeds"]["alpha"], d["n"])).to(gpu)
    Wt = torch.from_numpy(inputs(d["seeds"]["w"], d["n"])).to(gpu)
    th = torch.from_numpy(inputs(d["seeds"]["theta"], 1)[0]).to(gpu)
    ops.admm_dual(A, Wt, th, d["rho"])
    theta = ops.ordered_mean(Wt, torch.tensor(a["order"], dtype=torch.int32, device=gpu))
    torch.cuda.synchronize()
    assert sha(A.cpu().numpy()) == d["alpha1"]["sha256"]
    assert sha(theta.cpu().numpy()) == a["theta"]["sha256"]
