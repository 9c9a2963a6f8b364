import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-optimization-and-learning_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not has_gpu():
        pytest.skip("no GPU")
    import torch
    return torch.device("cuda:0")


PROJECT_MODULES = ("_engine", "models", "utils", "sampling", "clients", "simulators", "servers")


def load_project(name, modules):
    """Import the flat modules of one drop-in project (weighted_average /
    primal_dual) the way the reference's notebooks do (their dir on sys.path),
    purging the other project's same-named modules first."""
    import importlib
    for m in PROJECT_MODULES:
        sys.modules.pop(m, None)
    path = os.path.join(PKG, name)
    sys.path.insert(0, path)
    try:
        return {m: importlib.import_module(m) for m in modules}
    finally:
        sys.path.remove(path)
