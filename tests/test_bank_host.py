"""Host-side bank layout rules (dolhip/bank.py), no GPU: the agent-row stride
and the mapped-allocation switch."""
import pytest
import torch

from dolhip import bank as B


@pytest.mark.parametrize("P", [1, 63, 64, 4100, 101770, 262143, 262144, 1 << 20, 1_105_098, 1_663_370, 3_000_001])
def test_row_stride_rules(P):
    ld = B.row_stride(P)
    assert ld >= P and ld % B.ROW_ALIGN == 0  # 256-B aligned rows, every parameter inside
    if B.round_up(P, B.ROW_ALIGN) >= B.LONG_ROW:
        # >= 1 MiB rows: an odd multiple of 8 KiB (the ring round's best stride)
        assert ld % 4096 == 2048 and ld - P < 4096 + B.ROW_ALIGN
    else:
        assert ld % 2048 != 0 and ld - P < 1024 + B.ROW_ALIGN


def test_headline_stride():
    assert B.row_stride(1 << 20) == (1 << 20) + 2048


def test_device_matrix_never_maps_cpu_matrices(monkeypatch):
    monkeypatch.delenv("DOL_BANK_ALLOC", raising=False)
    made = []
    monkeypatch.setattr(B, "_MappedBlock", lambda *a: made.append(a))
    monkeypatch.setattr(B, "MAPPED_MIN_BYTES", 0)
    t = B.device_matrix(3, 8, "cpu")  # a CPU matrix never maps
    assert t.shape == (3, 8) and t.dtype == torch.float32 and made == []
    t = B.device_matrix(3, 8, "cpu", zero=True, mapped=True)
    assert float(t.abs().sum()) == 0.0 and made == []
