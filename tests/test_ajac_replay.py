"""tests/ajac_replay.py (the host replay of a DMEM_AsyncSmooth schedule) on
synthetic schedules: delivered on time it is synchronous Jacobi in residual
form (DMEM_Smooth.cpp:16-313 with no late delta); with every ghost delta one
relaxation late it is a different, still contracting iteration; a schedule that
waits on a relaxation no peer makes is refused."""
import numpy as np
import pytest
import scipy.sparse as sp

from ajac_replay import ajac_replay


def lap3(n):
    e = np.ones(n)
    T = sp.diags([-e[:-1], 2 * e, -e[:-1]], [-1, 0, 1])
    I = sp.identity(n)
    A = sp.kron(sp.kron(T, I), I) + sp.kron(sp.kron(I, T), I) + sp.kron(sp.kron(I, I), T)
    return sp.csr_matrix(A)


def schedule(R, K, lag):
    """per rank: update k, interior k, then the peers' deltas of sweep k - lag"""
    logs = []
    for q in range(R):
        ev = []
        for k in range(K):
            ev.append([1, k, 0, 0, 0])
            ev.append([2, k, 0, 0, 0])
            if k - lag >= 0:
                for p in range(R):
                    if p != q:
                        ev.append([3, p, k - lag, 0, 0])
        for k in range(max(0, K - lag), K):  # the drain
            for p in range(R):
                if p != q:
                    ev.append([3, p, k, 0, 0])
        logs.append(np.array(ev, dtype=np.float64))
    return logs


def test_on_time_is_synchronous_jacobi():
    n, K, w = 8, 10, 0.7
    A = lap3(n)
    N = A.shape[0]
    f = np.random.default_rng(3).uniform(-1, 1, N)
    x = np.zeros(N)
    for _ in range(K):
        x = x + w * (f - A @ x) / A.diagonal()
    for R in (1, 2, 3):
        rs = [N * q // R for q in range(R + 1)]
        xr, rr = ajac_replay(A, f, rs, schedule(R, K, 0), w)
        np.testing.assert_allclose(xr, x, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(rr, f - A @ xr, rtol=1e-10, atol=1e-12)


def test_late_deltas_and_refusal():
    n, K, w = 8, 12, 0.7
    A = lap3(n)
    N = A.shape[0]
    f = np.random.default_rng(4).uniform(-1, 1, N)
    rs = [0, N // 2, N]
    x0, _ = ajac_replay(A, f, rs, schedule(2, K, 0), w)
    x1, r1 = ajac_replay(A, f, rs, schedule(2, K, 1), w)
    assert not np.allclose(x0, x1)
    np.testing.assert_allclose(r1, f - A @ x1, rtol=1e-9, atol=1e-11)  # every delta applied once
    assert np.linalg.norm(f - A @ x1) < 0.5 * np.linalg.norm(f)
    bad = schedule(2, K, 0)
    bad[0] = np.concatenate([bad[0], [[3, 1, K + 5, 0, 0]]])
    with pytest.raises(RuntimeError):
        ajac_replay(A, f, rs, bad, w)
