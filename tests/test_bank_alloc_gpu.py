"""Bank buffers in one mapped physical allocation (dol_bank_alloc /
dol_bank_free through bank.device_matrix): usable by torch and by the kernels
like any device tensor, same bits as a torch-allocated buffer, freed with the
last tensor that references it."""
import gc

import numpy as np
import pytest
import torch

import oracle
from oracle import bits_equal
from dolhip import bank as B
from dolhip import ops

pytestmark = pytest.mark.gpu


def test_mapped_matrix_round_trip_and_mix(gpu, monkeypatch):
    monkeypatch.setattr(B, "MAPPED_MIN_BYTES", 0)
    monkeypatch.setenv("DOL_BANK_ALLOC", "vmm")
    n, P = 37, 4100
    X = B.device_matrix(n, P + 60, gpu)
    Y = B.device_matrix(n, P + 60, gpu, zero=True)
    assert X.device == gpu and X.dtype == torch.float32 and X.is_contiguous()
    assert float(Y.abs().sum()) == 0.0
    rng = np.random.default_rng(3)
    Xh = rng.standard_normal((n, P)).astype(np.float32)
    wp, wn = rng.random(n).astype(np.float32), rng.random(n).astype(np.float32)
    X[:, :P] = torch.from_numpy(Xh).to(gpu)
    ops.mix_ring(X, Y, torch.from_numpy(wp).to(gpu), torch.from_numpy(wn).to(gpu), P=P)
    torch.cuda.synchronize()
    assert bits_equal(Y[:, :P].cpu().numpy(), oracle.mix_ring(Xh, wp, wn))
    view = X[3:5, 10:20]  # a view keeps the block alive after X is gone
    want = view.cpu().clone()
    del X
    gc.collect()
    assert torch.equal(view.cpu(), want)
    del view, Y
    gc.collect()
    torch.cuda.synchronize()


def test_bank_maps_large_state_when_asked(gpu, monkeypatch):
    made = []

    class Spy(B._MappedBlock):
        def __init__(self, *a):
            super().__init__(*a)
            made.append(self.ptr)

    monkeypatch.setattr(B, "_MappedBlock", Spy)
    monkeypatch.setattr(B, "MAPPED_MIN_BYTES", 1 << 20)
    monkeypatch.delenv("DOL_BANK_ALLOC", raising=False)
    B.AgentBank(64, 8192, gpu).buffer("x")  # default: torch's allocator
    assert made == []
    monkeypatch.setenv("DOL_BANK_ALLOC", "vmm")
    bank = B.AgentBank(64, 8192, gpu)  # 2 MiB per buffer: mapped
    x = bank.buffer("x", zero=True)
    assert made == [x.data_ptr()] and float(x.abs().sum()) == 0.0
    small = B.AgentBank(4, 64, gpu).buffer("x")  # below the threshold: torch's allocator
    assert len(made) == 1 and small.data_ptr() != made[0]
    monkeypatch.setenv("DOL_BANK_ALLOC", "torch")
    B.AgentBank(64, 8192, gpu).buffer("x")
    assert len(made) == 1
