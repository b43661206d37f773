"""Shared fixtures: package loader, oracle, device context."""
import importlib.util
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: large-size checks")


def load_package():
    """Import async-multigrid_amd/ (dash in the directory name) as async_multigrid_amd."""
    if "async_multigrid_amd" in sys.modules:
        return sys.modules["async_multigrid_amd"]
    pkg_dir = os.path.join(ROOT, "async-multigrid_amd")
    spec = importlib.util.spec_from_file_location(
        "async_multigrid_amd", os.path.join(pkg_dir, "__init__.py"),
        submodule_search_locations=[pkg_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["async_multigrid_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def amg():
    return load_package()


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def ctx(amg):
    c = amg.Context(device=0, nstreams=16)
    yield c
    c.close()


def rng(seed=0):
    return np.random.default_rng(seed)


def random_csr(oracle, n, m, density_per_row=7, seed=0, diag_first=True, with_zero_diag=False):
    """Random sparse matrix, diagonal first in each row when square."""
    g = rng(seed)
    rp = [0]
    cols, vals = [], []
    for i in range(n):
        k = int(g.integers(0, 2 * density_per_row + 1))
        c = sorted(set(g.integers(0, m, size=k).tolist()))
        if n == m and diag_first:
            c = [i] + [x for x in c if x != i]
        v = g.uniform(-1, 1, size=len(c))
        if n == m and diag_first:
            v[0] = 0.0 if (with_zero_diag and i % 7 == 3) else 4.0 + abs(v[0])
        cols += c
        vals += v.tolist()
        rp.append(len(cols))
    return oracle.Csr(n, m, np.array(rp), np.array(cols, dtype=np.int32), np.array(vals))
