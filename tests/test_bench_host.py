"""Host-side pieces of bench.py that shape the reported numbers (no GPU):
the a n^2 + b n extrapolation of the CPU baselines, and the JSON contract's
kernel names for every ring-steps variant the product path may pick."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_fit_n2_n_recovers_exact_model(bench):
    a, b = 3e-7, 2e-4
    samples = {n: 1.0 / (a * n * n + b * n) for n in (128, 256)}
    fit = bench._fit_n2_n(samples, 1024)
    assert fit["a_s_per_agent2"] == pytest.approx(a, rel=1e-9)
    assert fit["b_s_per_agent"] == pytest.approx(b, rel=1e-9)
    assert fit["rounds_per_s"] == pytest.approx(1.0 / (a * 1024 ** 2 + b * 1024), rel=1e-9)


def test_fit_n2_n_linear_cost_is_not_squared(bench):
    """a per-agent (linear) cost must extrapolate linearly, not as n^2."""
    samples = {n: 1.0 / (1e-3 * n) for n in (128, 256)}
    fit = bench._fit_n2_n(samples, 1024)
    assert fit["rounds_per_s"] == pytest.approx(1.0 / (1e-3 * 1024), rel=1e-6)


def test_every_ring_steps_variant_has_a_kernel_name(bench):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))
    from dolhip import ops
    assert set(ops.RING_STEPS_VARIANTS) <= set(bench.RING_STEPS_KERNELS)
