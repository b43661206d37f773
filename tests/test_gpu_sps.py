"""-smoother async_sps: stochastic parallel Southwell gating of the asynchronous
Jacobi smoother (DMEM_Smooth.cpp:165-291, 548-572) on the GPU
(amg_dist_async_sps).  One rank has no neighbours: exponential / inverse
gating always relax (x = 0), RANDOM relaxes exactly in the sweeps whose draw
of the reference's RandDouble stream falls below alpha -- and a skipped sweep
changes nothing, so the iterate is BIT-IDENTICAL to the oracle's async Jacobi
(or_dmem_async_jacobi) run for that many relaxations.  More ranks exchange
their residual L1 norms with the deltas: a band test (every rank relaxes in
sweep 0, fewer relaxations than sweeps overall, convergence)."""
import numpy as np
import pytest

from test_gpu_dist import run_ranks
from test_gpu_kernels import assert_bitwise

pytestmark = pytest.mark.gpu


def problem(amg, oracle, n=20):
    gen = amg.Gen(n)
    f = amg.rhs_rand(0, n ** 3)
    nr, nc, rp, cj, cv = gen.host_csr(amg.AMG_GEN_A, 0)
    return gen, f, oracle.Csr(nr, nc, rp, cj, cv)


def sps_ranks(amg, gen, f, nranks, K, **kw):
    opts = amg.default_opts(smooth_weight=0.7, **kw)
    hub = amg.dist.ThreadMailbox(nranks)

    def rank(q):
        c = amg.Context(0, nstreams=2)
        if nranks == 1:
            amg.dist.init_rccl(c, 1, 0, lambda b: b)
        else:
            amg.dist.init_host(c, nranks, q, amg.dist.HostTransport(hub, q))
        D = amg.dist.DistHier(c, gen, opts)
        try:
            rel, nrel = D.async_sps(f[D.row0:D.row0 + D.n0], K)
            x = D.get_u()
            row0 = D.row0
        finally:
            D.free()
            amg.dist.finalize(c)
            c.close()
        return row0, x, rel, nrel

    return sorted(run_ranks(nranks, rank), key=lambda t: t[0])


@pytest.mark.parametrize("kind,alpha", [("random", 0.5), ("random", 0.2), ("exp", 1.0), ("inverse", 1.0)])
def test_sps_one_rank_matches_oracle(amg, oracle, kind, alpha):
    gen, f, A = problem(amg, oracle)
    K, w = 20, 0.7
    t = {"random": amg.AMG_SPS_RANDOM, "exp": amg.AMG_SPS_EXPONENTIAL, "inverse": amg.AMG_SPS_INVERSE}[kind]
    res = sps_ranks(amg, gen, f, 1, K, sps_probability_type=t, sps_alpha=alpha)
    _, x, rel, nrel = res[0]
    if kind == "random":
        draws = amg.rand_double_stream(0, K - 1)
        want = 1 + int(np.sum(draws < alpha))
    else:
        want = K
    assert nrel == want
    x_o, rn_o = oracle.dmem_async_jacobi(A, f, nrel, w, None)
    assert_bitwise(x, x_o, "SPS-gated async Jacobi (one rank)")
    np.testing.assert_allclose(rel, rn_o / np.linalg.norm(f), rtol=1e-12)
    gen.free()


@pytest.mark.parametrize("nranks,kind,extra", [(2, "exp", {}), (3, "exp", {"sps_alpha": 0.5}),
                                               (3, "min_prob", {"sps_min_prob": 0.25}),
                                               (4, "inverse", {"sps_alpha": 2.0})])
def test_sps_ranks_band(amg, oracle, nranks, kind, extra):
    gen, f, A = problem(amg, oracle)
    K = 30
    t = amg.AMG_SPS_INVERSE if kind == "inverse" else amg.AMG_SPS_EXPONENTIAL
    res = sps_ranks(amg, gen, f, nranks, K, sps_probability_type=t, **extra)
    rels = [r[2] for r in res]
    assert all(r == rels[0] for r in rels)  # one allreduced norm
    nrel = [r[3] for r in res]
    assert all(1 <= k <= K for k in nrel), nrel
    assert sum(nrel) < nranks * K, nrel  # somebody skipped: the gate is live
    x = np.concatenate([r[1] for r in res])
    assert np.all(np.isfinite(x))
    # fewer relaxations than Jacobi with K sweeps, still a smoother: it converges
    _, rn_min = oracle.dmem_async_jacobi(A, f, min(nrel), 0.7, None)
    assert rels[0] < 1.0
    assert rels[0] <= 1.5 * rn_min / np.linalg.norm(f), (rels[0], nrel)
    gen.free()


def test_sps_refuses_accel(amg, oracle):
    gen, f, _ = problem(amg, oracle, 8)
    with pytest.raises(AssertionError, match="no accel_type with SPS"):  # run_ranks' list of errors
        sps_ranks(amg, gen, f, 1, 4, accel_type=amg.AMG_RICHARD_ACCEL, cheby_mu=1.0, cheby_delta=1.0)
    gen.free()
