"""CPU: the DMEM elasticity problem generator (amg_elast_*, config 5).  MFEM is
not in the reference tree, so the assembly is restated (parity unpinned) and
pinned here by its defining properties: symmetry and definiteness, rigid-body
modes in the kernel of every row away from the fixed face, identity rows on
the fixed dofs, the total pull force, the material jump, and a classical
(num_functions = 3) hierarchy on which the oracle's SMEM_Solve converges."""
import numpy as np
import pytest
import scipy.sparse as sp


def problem(amg, r):
    n, rp, cj, v, b = amg.classical.elasticity(r)
    return n, rp, cj, v, b, sp.csr_matrix((v, cj, rp), shape=(n, n))


@pytest.mark.parametrize("r", [0, 1, 2])
def test_symmetric_definite_and_load(amg, r):
    n, rp, cj, v, b, A = problem(amg, r)
    s = 1 << r
    px, py, pz = 8 * s + 1, s + 1, s + 1
    assert n == 3 * px * py * pz
    assert abs(A - A.T).max() == 0.0
    assert all(cj[rp[i]] == i for i in range(n))  # diagonal first
    if n < 3000:
        assert np.linalg.eigvalsh(A.toarray()).min() > 0
    np.testing.assert_allclose(b.sum(), -1e-2, rtol=1e-12)
    nodes = np.arange(n) // 3
    x = nodes % px
    assert np.all(b[(np.arange(n) % 3) != 2] == 0) and np.all(b[x != px - 1] == 0)
    fixed = np.nonzero(x == 0)[0]
    for d in fixed:
        assert list(cj[rp[d]:rp[d + 1]]) == [d] and v[rp[d]] == 1.0
    assert not np.isin(cj, fixed).sum() - fixed.size  # fixed columns only on their own rows


@pytest.mark.parametrize("r", [1, 2])
def test_rigid_body_modes(amg, r):
    """Translations and infinitesimal rotations are exact in Q1 and strain-free:
    every row whose stencil does not touch the fixed face annihilates them."""
    n, rp, cj, v, b, A = problem(amg, r)
    s = 1 << r
    h = 1.0 / s
    px, py = 8 * s + 1, s + 1
    node = np.arange(n // 3)
    X = np.stack([node % px, (node // px) % py, node // (px * py)], 1) * h
    modes = []
    for d in range(3):
        u = np.zeros((n // 3, 3))
        u[:, d] = 1.0
        modes.append(u.ravel())
    for w in np.eye(3):
        modes.append(np.cross(w, X).ravel())
    xnode = (np.arange(n) // 3) % px
    free = xnode >= 2
    scale = np.abs(v).max()
    for u in modes:
        res = A @ u
        assert np.abs(res[free]).max() < 1e-12 * scale * max(1.0, np.abs(u).max())


def test_material_jump(amg):
    """lambda = mu = 50 on the first half of the beam: the diagonal there is 50x."""
    n, rp, cj, v, b, A = problem(amg, 2)
    px = 33
    d = A.diagonal()
    x = (np.arange(n) // 3) % px
    interior = (np.arange(n) // 3 // px) % 5
    mid = (interior == 2) & ((np.arange(n) // 3 // (px * 5)) == 2)
    left = d[mid & (x == 8)]
    right = d[mid & (x == 24)]
    np.testing.assert_allclose(left, 50.0 * right, rtol=1e-13)


def test_classical_hierarchy_converges(amg, oracle):
    n, rp, cj, v, b, _ = problem(amg, 2)
    H = amg.classical.ClassicalAMG(n, rp, cj, v, coarsen_type=9, strong_threshold=0.5, num_functions=3)
    As = [oracle.Csr(*H.get(amg.AMG_GEN_A, l)) for l in range(H.L)]
    Ps = [oracle.Csr(*H.get(amg.AMG_GEN_P, l)) for l in range(H.L - 1)]
    Rs = [oracle.Csr(*H.get(amg.AMG_GEN_R, l)) for l in range(H.L - 1)]
    cf = H.cf_marker(0)
    fine_of = np.nonzero(cf == 1)[0]
    P = Ps[0]
    for i in range(n):  # interpolation never mixes displacement components
        assert np.all(fine_of[P.col[P.rowptr[i]:P.rowptr[i + 1]]] % 3 == i % 3)
    OH = oracle.Hier(As, Ps, Rs, oracle.make_opts(smooth_weight=0.6, num_cycles=40))
    _, hist, k = OH.solve(b)
    assert np.all(np.diff(hist) < 0)
    assert hist[-1] < 0.6 * hist[0]
