"""CPU: the product's structured hierarchy generator against the oracle's
generic CSR SpGEMM (Galerkin R A P) and 7-pt builder -- bit for bit."""
import numpy as np
import pytest


def csr_of(oracle, g, which, level):
    return oracle.Csr(*g.host_csr(which, level))


def drop_zeros(oracle, M):
    keep = M.val != 0.0
    rows = np.repeat(np.arange(M.nrows), np.diff(M.rowptr))
    rp = np.concatenate([[0], np.cumsum(np.bincount(rows[keep], minlength=M.nrows))])
    return oracle.Csr(M.nrows, M.ncols, rp, M.col[keep], M.val[keep])


def same(a, b):
    return (a.nrows == b.nrows and a.ncols == b.ncols and np.array_equal(a.rowptr, b.rowptr)
            and np.array_equal(a.col, b.col)
            and np.array_equal(a.val.view(np.uint64), b.val.view(np.uint64)))


def test_level0_is_hypre_7pt(amg, oracle):
    for dims in ((16, 16, 16), (13, 7, 5)):
        g = amg.Gen(*dims)
        assert same(csr_of(oracle, g, amg.AMG_GEN_A, 0), oracle.laplace_7pt(*dims))


@pytest.mark.parametrize("interp", ["linear", "aggregate"])
@pytest.mark.parametrize("dims", [(16, 16, 16), (20, 12, 9)])
def test_galerkin_hierarchy_bitwise(amg, oracle, interp, dims):
    it = amg.AMG_INTERP_LINEAR if interp == "linear" else amg.AMG_INTERP_AGGREGATE
    g = amg.Gen(*dims, interp=it)
    assert g.L >= 3
    for l in range(g.L - 1):
        A = csr_of(oracle, g, amg.AMG_GEN_A, l)
        P = csr_of(oracle, g, amg.AMG_GEN_P, l)
        R = csr_of(oracle, g, amg.AMG_GEN_R, l)
        assert same(R, oracle.transpose(P)), f"R{l} != P{l}^T"
        rap = drop_zeros(oracle, oracle.spgemm(oracle.spgemm(R, A), P))
        assert same(csr_of(oracle, g, amg.AMG_GEN_A, l + 1), rap), f"A{l + 1} != R A P"


def test_plane_slabs_concatenate(amg, oracle):
    g = amg.Gen(12, 10, 8)
    for which, lev in ((amg.AMG_GEN_A, 0), (amg.AMG_GEN_A, 1), (amg.AMG_GEN_P, 0), (amg.AMG_GEN_R, 0)):
        full = g.host_csr(which, lev)
        nz = g.dims(lev + 1 if which == amg.AMG_GEN_R else lev)[2]
        cuts = [0, 1, nz // 2, nz]
        parts = [g.host_csr(which, lev, a, b) for a, b in zip(cuts[:-1], cuts[1:])]
        cj = np.concatenate([p[3] for p in parts])
        cv = np.concatenate([p[4] for p in parts])
        np.testing.assert_array_equal(cj, full[3])
        np.testing.assert_array_equal(cv, full[4])


def test_512_config_shape(amg):
    g = amg.Gen(512)
    assert g.L == 9 and g.dims(8) == (2, 2, 2)
    # planes z = 0,1: the -z face is missing on plane 0, +-x / +-y faces on both
    nnz2 = amg.lib.amg_gen_nnz(g.h, amg.AMG_GEN_A, 0, 0, 2)
    assert nnz2 == 2 * 7 * 512 ** 2 - (512 ** 2 + 2 * 2 * 2 * 512)
    # z0 = 7n - 6 side^2 = 937,951,232 at 512^3
    assert amg.lib.amg_gen_nnz(g.h, amg.AMG_GEN_A, 0, 0, 512) == 937951232


def test_rhs_rand_matches_oracle(amg, oracle):
    np.testing.assert_array_equal(amg.rhs_rand(0, 1000), oracle.rhs_rand(1000))
    np.testing.assert_array_equal(amg.rhs_rand(300, 700), oracle.rhs_rand(1000)[300:700])
