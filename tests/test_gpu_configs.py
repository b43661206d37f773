"""Parity at the BASELINE.json config sizes.

* config 1 -- 64^3 7-pt, SMEM_Solve MULT V(1,1) weighted Jacobi (w = 0.8), 20 cycles
  (SEQ_AMG on the CPU in the reference; here the same solve on the GPU): iterate
  bit-identical to the oracle after the last cycle, residual history rtol 1e-12.
* config 2 -- 256^3, the same solve (SMEM_Sync_AMG, Jacobi): bitwise iterate and
  residual history rtol 1e-12, once with the default storage the bench runs
  (master-pattern CSR for the square operators) and once with every compressed form
  off (plain CSR through the general tile kernel).
* config 3 -- 256^3 SMEM_Async_AMG ASYNC_MULTADD with hybrid Jacobi-Gauss-Seidel:
  nondeterministic like the reference (SMEM_Async_AMG.cpp:7-437).  Under the
  round-robin schedule the iterate is bit-identical to the oracle's
  or_async_add; the free race's final relative residual must sit inside the
  band of 20 committed oracle runs (tests/golden/config3_band.json) on the same
  hierarchy, smoother and block partition.  The reference applies Chebyshev only on
  its synchronous path (SMEM_Solve.cpp:169-188), so the async
  solve runs without it; the Chebyshev-accelerated sync solve is checked bitwise at
  256^3 below.

Matching SMEM_Solve.cpp:128-215 and SMEM_Sync_AMG.cpp:8-145.  Tolerances: iterate
bit-exact; norms rtol 1e-12 (reduction order differs: OpenMP vs a device tree).
"""
import numpy as np
import pytest

from test_gpu_kernels import assert_bitwise
from test_gpu_solve import oracle_opts

pytestmark = pytest.mark.gpu


def host_levels(amg, oracle, g):
    L = g.L
    return {tag: [oracle.Csr(*g.host_csr(code, l)) for l in range(cnt)]
            for tag, code, cnt in (("A", amg.AMG_GEN_A, L), ("P", amg.AMG_GEN_P, L - 1),
                                   ("R", amg.AMG_GEN_R, L - 1))}


def free_hier(H):
    mats = [M for group in H._keep for M in group]
    H.free()
    for M in mats:
        M.free()


def formats_off(ctx, on):
    v = 1 if on else 0
    ctx.set_value_index(v)
    ctx.set_dict_index(v)
    ctx.set_row_pattern(v)
    ctx.set_pair_pattern(v)
    ctx.set_master_pattern(v)


def run_sync(amg, oracle, ctx, n, cycles, storage, **kw):
    g = amg.Gen(n, interp=amg.AMG_INTERP_LINEAR)
    host = host_levels(amg, oracle, g)
    opts = amg.default_opts(smooth_weight=0.8, num_cycles=cycles, tol=0.0, **kw)
    if storage == "default":
        # the device-side generator path the bench runs (compressed forms chosen at registration)
        H = amg.build_hierarchy(ctx, g, opts)
        A0 = H._keep[0][0]
        if n >= 64:
            assert A0.master_pattern != 0, "fine operator should take the master-pattern form"
    else:
        formats_off(ctx, False)
        try:
            dev = {k: [ctx.csr(M.nrows, M.ncols, M.rowptr, M.col, M.val) for M in v]
                   for k, v in host.items()}
        finally:
            formats_off(ctx, True)
        assert dev["A"][0].value_index == 0 and dev["A"][0].master_pattern == 0
        H = amg.Hier(ctx, dev["A"], dev["P"], dev["R"], opts)
    f = amg.rhs_rand(0, n ** 3)
    u_g, h_g, k_g = H.solve(f)
    free_hier(H)
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, opts))
    u_c, h_c, k_c = OH.solve(f)
    assert k_g == k_c == cycles
    assert_bitwise(u_g, u_c, f"{n}^3 iterate after {cycles} cycles ({storage})")
    np.testing.assert_allclose(h_g, h_c, rtol=1e-12, atol=0)
    g.free()
    return h_g


@pytest.mark.parametrize("storage", ["default", "csr"])
def test_config1_64cube_jacobi_vcycle(amg, oracle, ctx, storage):
    h = run_sync(amg, oracle, ctx, 64, 20, storage)
    assert h[-1] / h[0] < 1e-6


@pytest.mark.parametrize("storage", ["default", "csr"])
def test_config2_256cube_jacobi_vcycle(amg, oracle, ctx, storage):
    h = run_sync(amg, oracle, ctx, 256, 20, storage)
    assert h[-1] / h[0] < 1e-5


def test_config2_256cube_fused_outer_residual(amg, oracle, ctx):
    """The bench's setting (reuse_outer_residual 2: the outer residual fused into
    the next cycle's first sweep, residual vector not written) at 256^3."""
    run_sync(amg, oracle, ctx, 256, 12, "default", reuse_outer_residual=2)


def test_config3_256cube_cheby_sync(amg, oracle, ctx):
    """Chebyshev-accelerated SMEM_Solve (SMEM_Solve.cpp:169-188) at 256^3 with the
    eigen-bounds of the preconditioned operator from the GPU power iteration."""
    g = amg.Gen(256, interp=amg.AMG_INTERP_LINEAR)
    base = amg.default_opts(smooth_weight=0.8, num_cycles=8, tol=0.0)
    H = amg.build_hierarchy(ctx, g, base)
    emax, emin = H.eigs_power(20)
    free_hier(H)
    g.free()
    assert emax > 0.0 and emin < emax
    mu = (emax + emin) / (emax - emin)
    delta = 2.0 / (emax + emin)
    run_sync(amg, oracle, ctx, 256, 8, "default", cheby_flag=1, cheby_mu=mu, cheby_delta=delta)


def config3_setup(amg, oracle, n=256, w=0.8, B=64):
    g = amg.Gen(n, interp=amg.AMG_INTERP_LINEAR)
    host = host_levels(amg, oracle, g)
    L = g.L
    # MULTADD uses smoothed transfers P~ = (I - w D^-1 A) P, R~ = P~^T (SMEM_Setup.cpp:244-261)
    Ps, Rs = [], []
    for lev in range(L - 1):
        ps, rs = oracle.smooth_transfer(host["A"][lev], host["P"][lev], w)
        Ps.append(ps)
        Rs.append(rs)
    host = {"A": host["A"], "P": Ps, "R": Rs}
    f = amg.rhs_rand(0, n ** 3)
    blocks = {lev: np.unique(np.minimum(np.arange(0, host["A"][lev].nrows + B, B),
                                        host["A"][lev].nrows)).astype(np.int32)
              for lev in range(L)}
    return g, L, host, f, blocks


def test_config3_256cube_async_multadd_hybrid_jgs(amg, oracle, ctx):
    """config 3's race against a committed oracle band: tests/golden/config3_band.json
    holds 10 or_async_add runs with one thread per level and 10 with two (the
    reference's SMEM_Async_Add_AMG restated on OpenMP thread groups, generated by
    tools/gen_config3_band.py on this container's 8 cores).  The device's median
    run must lie in [0.5 min, 2 max] of those 20 oracle runs and no run beyond
    4 max (round 3 saw one run at 2.3x the others when a level stream queued
    behind the shared hardware queues); no band member comes from the device."""
    import json
    import os
    n, w, N, B = 256, 0.8, 8, 64
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "config3_band.json")))
    assert (fx["n"], fx["num_cycles"], fx["jgs_block_rows"]) == (n, N, B)
    orels = [x for v in fx["threads_per_level_runs"].values() for x in v]
    assert len(orels) >= 20
    lo, hi = min(orels), max(orels)
    g, L, host, f, blocks = config3_setup(amg, oracle, n, w, B)
    dev = {k: [ctx.csr(M.nrows, M.ncols, M.rowptr, M.col, M.val) for M in v] for k, v in host.items()}
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smoother=amg.AMG_HYBRID_JGS,
                            smooth_weight=w, num_cycles=N, tol=0.0, num_threads=0, jgs_block_rows=B)
    H = amg.Hier(ctx, dev["A"], dev["P"], dev["R"], opts)
    rels = []
    for _ in range(3):
        u, rel, cnt = H.async_solve(f)
        assert np.all(np.isfinite(u))
        assert list(cnt[:L - 1]) == [N] * (L - 1)
        rels.append(rel)
    free_hier(H)
    g.free()
    from async_band import in_band
    print(f"config 3 async: oracle band [{lo:.4e}, {hi:.4e}] width {hi / lo:.2f}x ({len(orels)} runs), "
          f"sync {fx['sync_multadd_relres']:.4e}, device {rels}")
    assert in_band(sorted(rels)[1], lo, hi), (rels, lo, hi)
    assert max(rels) <= 4.0 * hi, (rels, lo, hi)


def test_config3_256cube_round_robin_bitwise(amg, oracle, ctx):
    """config 3 with the arithmetic pinned: under the round-robin schedule
    (async_schedule 3: level corrections in turn, k_lo first) the device's
    ASYNC_MULTADD / hybrid JGS iterate at 256^3 is bit-identical to or_async_add
    under or_set_async_schedule(3)"""
    n, w, N, B = 256, 0.8, 4, 64
    g, L, host, f, blocks = config3_setup(amg, oracle, n, w, B)
    dev = {k: [ctx.csr(M.nrows, M.ncols, M.rowptr, M.col, M.val) for M in v] for k, v in host.items()}
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smoother=amg.AMG_HYBRID_JGS, smooth_weight=w,
                            num_cycles=N, tol=0.0, num_threads=0, jgs_block_rows=B, async_schedule=3)
    H = amg.Hier(ctx, dev["A"], dev["P"], dev["R"], opts)
    u, rel, cnt = H.async_solve(f)
    free_hier(H)
    g.free()
    OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, opts))
    for lev, blk in blocks.items():
        OH.set_blocks(lev, blk)
    oracle.lib().or_set_async_schedule(3)
    try:
        uo, relo, cnto = OH.async_add(f, [1] * L)
    finally:
        oracle.lib().or_set_async_schedule(0)
    assert list(cnt[:L - 1]) == list(cnto[:L - 1]) == [N] * (L - 1)
    assert_bitwise(u, uo, "config 3 round-robin iterate")
    assert abs(rel - relo) <= 1e-12 * relo
