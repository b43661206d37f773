"""CPU: the in-house classical AMG setup (amg_classical_*, csrc/amg_classical.cpp),
the hierarchy the reference takes from HYPRE_BoomerAMGSetup.  hypre is not in the
reference tree, so its output is not a fixture (parity unpinned); these tests pin
the restated algorithms' defining properties instead:
  * strength: hypre CreateS against a numpy restatement, one function per unknown;
  * C/F splitting: every F point that others depend on interpolates from a strong
    C neighbour; isolated points are F;
  * interpolation: C rows inject, F rows reach only C points within distance two,
    zero-row-sum rows interpolate constants exactly;
  * Galerkin: R == P^T and A_{l+1} == R (A P) bit for bit against the oracle's
    Gustavson product;
  * the oracle's SMEM_Solve converges on the hierarchy."""
import numpy as np
import pytest


def strength_np(A, theta, nfun=1):
    """hypre_BoomerAMGCreateS (serial, max_row_sum 1): S[i] = strong j != i."""
    S = []
    for i in range(A.nrows):
        cols = A.col[A.rowptr[i]:A.rowptr[i + 1]]
        vals = A.val[A.rowptr[i]:A.rowptr[i + 1]]
        diag = vals[cols == i].sum()
        off = (cols != i) & (cols % nfun == i % nfun)
        scale = 0.0
        for v in vals[off]:
            scale = max(scale, v) if diag < 0 else min(scale, v)
        strong = [int(c) for c, v, o in zip(cols, vals, off)
                  if o and ((v > theta * scale) if diag < 0 else (v < theta * scale))]
        S.append(strong)
    return S


def aniso(oracle, n, eps):
    """2-D anisotropic 5-pt operator (strong x coupling, eps in y), diagonal first."""
    rp, cj, cv = [0], [], []
    for y in range(n):
        for x in range(n):
            i = y * n + x
            cols, vals = [i], [2.0 + 2.0 * eps]
            for dx, dy, w in ((-1, 0, -1.0), (1, 0, -1.0), (0, -1, -eps), (0, 1, -eps)):
                if 0 <= x + dx < n and 0 <= y + dy < n:
                    cols.append((y + dy) * n + x + dx)
                    vals.append(w)
            cj += cols
            cv += vals
            rp.append(len(cj))
    return oracle.Csr(n * n, n * n, np.array(rp), np.array(cj, dtype=np.int32), np.array(cv))


def systems(oracle, n):
    """two interleaved 3-D Laplacians (unknown i % 2), weakly coupled across functions"""
    L = oracle.laplace_7pt(n)
    N = 2 * L.nrows
    rp, cj, cv = [0], [], []
    for i in range(N):
        p, fn = i // 2, i % 2
        cols = [2 * int(c) + fn for c in L.col[L.rowptr[p]:L.rowptr[p + 1]]]
        vals = list(L.val[L.rowptr[p]:L.rowptr[p + 1]])
        other = 2 * p + (1 - fn)
        cols.append(other)
        vals.append(-0.05)
        cj += cols
        cv += vals
        rp.append(len(cj))
    return oracle.Csr(N, N, np.array(rp), np.array(cj, dtype=np.int32), np.array(cv))


CASES = [("lap", 10, 6, 0.25), ("lap", 8, 6, 0.5), ("lap", 9, 6, 0.5), ("lap", 10, 3, 0.25),
         ("aniso", 10, 6, 0.25), ("aniso", 8, 6, 0.25)]


def build(amg, oracle, kind, ct, it, theta, nfun=1):
    A = {"lap": lambda: oracle.laplace_7pt(14), "aniso": lambda: aniso(oracle, 40, 0.01),
         "sys": lambda: systems(oracle, 10)}[kind]()
    H = amg.classical.ClassicalAMG(A.nrows, A.rowptr, A.col, A.val, coarsen_type=ct, interp_type=it,
                                   strong_threshold=theta, num_functions=nfun)
    return A, H


@pytest.mark.parametrize("kind,ct,it,theta", CASES + [("sys", 10, 6, 0.25)])
def test_splitting_and_interpolation(amg, oracle, kind, ct, it, theta):
    nfun = 2 if kind == "sys" else 1
    A0, H = build(amg, oracle, kind, ct, it, theta, nfun)
    assert H.L >= 3
    for lev in range(H.L - 1):
        A = oracle.Csr(*H.get(amg.AMG_GEN_A, lev))
        if lev == 0:
            assert np.array_equal(A.val, A0.val) and np.array_equal(A.col, A0.col)
        S = strength_np(A, theta, nfun)
        ST = [[] for _ in range(A.nrows)]
        for i, row in enumerate(S):
            for j in row:
                ST[j].append(i)
        cf = H.cf_marker(lev)
        assert set(np.unique(cf)) <= {-1, 1}
        C = cf == 1
        for i in range(A.nrows):
            if cf[i] == -1 and ST[i]:  # others depend on i: it interpolates from a strong C point
                assert any(C[j] for j in S[i]), (lev, i)
        n, nc, rp, cj, v = H.get(amg.AMG_GEN_P, lev)
        assert n == A.nrows and nc == C.sum()
        cidx = np.cumsum(C) - 1
        fine_of = np.nonzero(C)[0]
        for i in range(n):
            cols, vals = cj[rp[i]:rp[i + 1]], v[rp[i]:rp[i + 1]]
            assert np.all(np.diff(cols) > 0)
            if C[i]:
                assert list(cols) == [cidx[i]] and list(vals) == [1.0]
                continue
            reach = {j for j in S[i] if C[j]}
            if it == 6:
                for k in S[i]:
                    if not C[k]:
                        reach |= {j for j in S[k] if C[j]}
            assert set(fine_of[cols]) <= reach, (lev, i)
            assert all(f % nfun == i % nfun for f in fine_of[cols])
            row = A.val[A.rowptr[i]:A.rowptr[i + 1]]
            ac = A.col[A.rowptr[i]:A.rowptr[i + 1]]
            same = ac % nfun == i % nfun
            if abs(row[same].sum()) < 1e-13 * abs(row).max() and cols.size and np.all(row[ac != i] <= 0):
                np.testing.assert_allclose(vals.sum(), 1.0, rtol=1e-12)


@pytest.mark.parametrize("kind,ct,it,theta", CASES[:3] + [("sys", 10, 6, 0.25)])
def test_strength_matches_restatement(amg, oracle, kind, ct, it, theta):
    """The splitting is only as good as S: F points with dependents must see a C
    point among the numpy-restated strong neighbours, and the coarse grid holds
    exactly the C points (checked above); here S itself is exercised through
    direct interpolation, whose F rows are exactly the strong C neighbours."""
    nfun = 2 if kind == "sys" else 1
    A0, H = build(amg, oracle, kind, ct, amg.classical.AMG_CLASSICAL_DIRECT, theta, nfun)
    S = strength_np(A0, theta, nfun)
    cf = H.cf_marker(0)
    C = cf == 1
    fine_of = np.nonzero(C)[0]
    n, nc, rp, cj, v = H.get(amg.AMG_GEN_P, 0)
    for i in range(n):
        if not C[i]:
            assert set(fine_of[cj[rp[i]:rp[i + 1]]]) == {j for j in S[i] if C[j]} or rp[i] == rp[i + 1]


@pytest.mark.parametrize("kind,ct,it,theta", CASES)
def test_galerkin_bitwise(amg, oracle, kind, ct, it, theta):
    _, H = build(amg, oracle, kind, ct, it, theta)
    for lev in range(H.L - 1):
        A = oracle.Csr(*H.get(amg.AMG_GEN_A, lev))
        P = oracle.Csr(*H.get(amg.AMG_GEN_P, lev))
        R = oracle.Csr(*H.get(amg.AMG_GEN_R, lev))
        Ac = oracle.Csr(*H.get(amg.AMG_GEN_A, lev + 1))
        T = oracle.transpose(P)
        assert np.array_equal(T.rowptr, R.rowptr) and np.array_equal(T.col, R.col)
        assert np.array_equal(T.val.view(np.int64), R.val.view(np.int64))
        ref = oracle.spgemm(R, oracle.spgemm(A, P))
        assert np.array_equal(ref.rowptr, Ac.rowptr) and np.array_equal(ref.col, Ac.col)
        assert np.array_equal(ref.val.view(np.int64), Ac.val.view(np.int64))
        assert all(Ac.col[Ac.rowptr[i]] == i for i in range(Ac.nrows) if Ac.rowptr[i + 1] > Ac.rowptr[i])


@pytest.mark.parametrize("ct", [10, 8, 9])
def test_oracle_solve_converges(amg, oracle, ct):
    """SMEM_Solve (V(1,1) Jacobi, w = 0.8) on the in-house hierarchy of a 24^3
    Laplacian: a convergence factor typical of classical AMG."""
    A = oracle.laplace_7pt(24)
    H = amg.classical.ClassicalAMG(A.nrows, A.rowptr, A.col, A.val, coarsen_type=ct)
    As = [oracle.Csr(*H.get(amg.AMG_GEN_A, l)) for l in range(H.L)]
    Ps = [oracle.Csr(*H.get(amg.AMG_GEN_P, l)) for l in range(H.L - 1)]
    Rs = [oracle.Csr(*H.get(amg.AMG_GEN_R, l)) for l in range(H.L - 1)]
    assert As[-1].nrows <= 9 or H.L == 25
    OH = oracle.Hier(As, Ps, Rs, oracle.make_opts(smooth_weight=0.8, num_cycles=20))
    f = oracle.rhs_rand(A.nrows)
    _, hist, k = OH.solve(f)
    assert k == 20
    assert (hist[-1] / hist[0]) ** (1 / k) < 0.45


def test_pmis_seed_and_errors(amg, oracle):
    A = oracle.laplace_7pt(10)
    a = amg.classical.ClassicalAMG(A.nrows, A.rowptr, A.col, A.val, coarsen_type=9, seed=1)
    b = amg.classical.ClassicalAMG(A.nrows, A.rowptr, A.col, A.val, coarsen_type=9, seed=1)
    c = amg.classical.ClassicalAMG(A.nrows, A.rowptr, A.col, A.val, coarsen_type=9, seed=2)
    assert np.array_equal(a.cf_marker(0), b.cf_marker(0))
    assert not np.array_equal(a.cf_marker(0), c.cf_marker(0))
    with pytest.raises(amg.AmgError, match="coarsen_type"):
        amg.classical.ClassicalAMG(A.nrows, A.rowptr, A.col, A.val, coarsen_type=3)
    with pytest.raises(amg.AmgError, match="num_functions"):
        amg.classical.ClassicalAMG(A.nrows, A.rowptr, A.col, A.val, num_functions=7)


@pytest.mark.parametrize("ct,it", [(9, 6), (10, 6), (9, 3)])
def test_threaded_setup_identical(amg, monkeypatch, ct, it):
    """Strength and interpolation run over row ranges on host threads
    (AMG_SETUP_THREADS); the ranges are concatenated in row order, so every
    level's A, P and R is identical to the single-thread build (elasticity r=3,
    3 functions; with the variable set every level of >= 64 rows splits)."""
    n, rp, cj, v, _ = amg.classical.elasticity(3)
    mats = {}
    for t in ("1", "5"):
        monkeypatch.setenv("AMG_SETUP_THREADS", t)
        H = amg.classical.ClassicalAMG(n, rp, cj, v, coarsen_type=ct, strong_threshold=0.5, num_functions=3,
                                       interp_type=it)
        mats[t] = [H.get(w, l) for l in range(H.L) for w in (amg.AMG_GEN_A, amg.AMG_GEN_P, amg.AMG_GEN_R)
                   if not (w != amg.AMG_GEN_A and l == H.L - 1)]
        H.free()
    assert len(mats["1"]) == len(mats["5"]) >= 6
    for a, b in zip(mats["1"], mats["5"]):
        assert a[0] == b[0] and a[1] == b[1]
        for x, y in zip(a[2:], b[2:]):
            assert np.array_equal(x, y)
            if x.dtype == np.float64:
                assert np.array_equal(x.view(np.int64), y.view(np.int64))
