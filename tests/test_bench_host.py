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


def test_fit_n2_n_noise_cannot_make_a_coefficient_negative(bench):
    """with samples whose exact solve has b < 0 (the middle size
    slow, the largest fast), the fit stays in a, b >= 0 and the extrapolated
    rate stays positive and finite."""
    samples = {64: 1.0 / 0.010, 128: 1.0 / 0.030, 256: 1.0 / 0.050}
    fit = bench._fit_n2_n(samples, 1024)
    assert fit["a_s_per_agent2"] >= 0.0 and fit["b_s_per_agent"] >= 0.0
    assert fit["rounds_per_s"] is not None and 0 < fit["rounds_per_s"] < samples[256]
    # a pure n^2 cost with one noisy point: a > 0 and a rate below the largest sample's
    noisy = {64: 1.0 / (1e-6 * 64 ** 2), 128: 1.0 / (1e-6 * 128 ** 2 * 1.2), 256: 1.0 / (1e-6 * 256 ** 2 * 0.9)}
    f2 = bench._fit_n2_n(noisy, 1024)
    assert f2["a_s_per_agent2"] > 0 and f2["b_s_per_agent"] >= 0 and f2["rounds_per_s"] < noisy[256]


def _bench_env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "DOL_BENCH_FAIL_RANK")}
    env.update(DOL_DIST_BACKEND="gloo", DOL_DEVICE_MAP="0", **extra)
    return env


def _run(cmd, env, timeout=240):
    import subprocess
    import sys
    return subprocess.run([sys.executable, *cmd], cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


def test_bench_gpus_n_spawns_n_ranks_itself():
    """`python bench.py --gpus 2` with no launcher around it
    starts two ranks itself and the relayed line says n_gpus 2, with the world
    size and backend each rank saw."""
    import json
    r = _run(["bench.py", "--gpus", "2", "--launch-check"], _bench_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [s for s in r.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    par = line["parallel"]
    assert par["world_size"] == 2 and par["backend"] == "gloo"
    assert [i["rank"] for i in par["ranks"]] == [0, 1]
    assert all(i["world_size"] == 2 and i["backend"] == "gloo" for i in par["ranks"])
    assert all(i["launcher"].startswith("bench.py") for i in par["ranks"])
    assert len({i["pid"] for i in par["ranks"]}) == 2


def test_bench_under_torchrun_keeps_working():
    import json
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = _run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
              "--master-port", str(port), "bench.py", "--gpus", "2", "--launch-check"], _bench_env())
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([s for s in r.stdout.splitlines() if s.startswith("{")][0])
    assert line["n_gpus"] == 2
    assert all(i["launcher"] == "torch.distributed.run" for i in line["parallel"]["ranks"])


def test_bench_refuses_fewer_ranks_than_asked():
    """A run whose joined world differs from --gpus exits non-zero (it used to
    warn and time one GPU)."""
    r = _run(["bench.py", "--gpus", "2", "--launch-check"], _bench_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2
    assert not [s for s in r.stdout.splitlines() if s.startswith("{")]


def test_bench_spawned_rank_failure_fails_the_run():
    """A rank that dies makes the launcher stop the others and exit non-zero
    without relaying a line (not after the collective timeout)."""
    import time
    t0 = time.time()
    r = _run(["bench.py", "--gpus", "3", "--launch-check"], _bench_env(DOL_BENCH_FAIL_RANK="1",
                                                                       DOL_COLLECTIVE_TIMEOUT_S="600"))
    assert r.returncode != 0
    assert not [s for s in r.stdout.splitlines() if s.startswith("{")]
    assert time.time() - t0 < 120


def test_every_ring_steps_variant_has_a_kernel_name(bench):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "distributed-optimization-and-learning_amd"))
    from dolhip import ops
    assert set(ops.RING_STEPS_VARIANTS) <= set(bench.RING_STEPS_KERNELS)
