"""Delay / fault injection (input.delay_type, delay_usec, delay_frac, fail_iter;
SMEM_Solve.cpp:33-43,112-146, DMEM_DelayProc DMEM_Misc.cpp:668-684): a delay
is a device-side wait on the stream the delayed work runs on, so it moves time
and never values -- synchronous results stay bit-identical, the wall clock
grows by the injected waits, and an async level group that is slowed down does
fewer corrections than the others under converge_test GLOBAL."""
import json
import os
import sys
import time

import numpy as np
import pytest

from test_gpu_dist import distributed
from test_gpu_kernels import assert_bitwise
from test_gpu_solve import gpu_hier, hierarchy

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def h24(amg, oracle):
    _, L, host = hierarchy(amg, oracle, 24, amg.AMG_INTERP_LINEAR)
    return L, host, amg.rhs_rand(0, 24 ** 3)


def timed_solve(amg, ctx, host, f, **kw):
    opts = amg.default_opts(smooth_weight=0.8, num_cycles=6, tol=0.0, **kw)
    H, _ = gpu_hier(amg, ctx, host, opts)
    H.solve(f)  # warm
    t0 = time.perf_counter()
    u, hist, k = H.solve(f)
    dt = time.perf_counter() - t0
    H.free()
    return u, hist, dt


@pytest.mark.parametrize("kind", ["one", "some", "all", "fail"])
def test_sync_delay_moves_time_not_values(amg, ctx, h24, kind):
    L, host, f = h24
    u0, h0, t0 = timed_solve(amg, ctx, host, f)
    dt = {"one": amg.AMG_DELAY_ONE, "some": amg.AMG_DELAY_SOME, "all": amg.AMG_DELAY_ALL,
          "fail": amg.AMG_FAIL_ONE}[kind]
    # 16 threads; DELAY_ALL: each cycle waits for the longest of 16 draws in
    # [0, 40 ms) (expected 37.6 ms); ONE / FAIL_ONE: one draw (expected 20 ms)
    u1, h1, t1 = timed_solve(amg, ctx, host, f, num_threads=16, delay_type=dt, delay_usec=20000,
                             delay_frac=0.5, fail_iter=3)
    assert_bitwise(u1, u0, f"delay {kind} iterate")
    assert_bitwise(h1, h0, f"delay {kind} norm history")
    lo = {"one": 0.010, "some": 0.10, "all": 0.15, "fail": 0.0}[kind]
    assert t1 - t0 >= lo, (kind, t0, t1)
    assert t1 - t0 < 6 * 0.040 + 1.0, (kind, t0, t1)


def test_async_delayed_group_does_fewer_corrections(amg, oracle, ctx):
    """ASYNC_MULTADD, converge_test GLOBAL: the coarsest group (thread T-1)
    waits 3 ms before each correction; the others keep correcting meanwhile,
    and the solve still converges."""
    _, L, host = hierarchy(amg, oracle, 24, amg.AMG_INTERP_LINEAR)
    Ps, Rs = [], []
    for lev in range(L - 1):
        ps, rs = oracle.smooth_transfer(host["A"][lev], host["P"][lev], 0.8)
        Ps.append(ps)
        Rs.append(rs)
    mult = {"A": host["A"], "P": Ps, "R": Rs}
    f = amg.rhs_rand(0, 24 ** 3)
    N = 8
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=N, tol=0.0,
                            num_threads=8, converge_test_type=amg.AMG_GLOBAL, delay_type=amg.AMG_DELAY_ONE,
                            delay_usec=3000)
    H, _ = gpu_hier(amg, ctx, mult, opts)
    u, rel, cnt = H.async_solve(f)
    H.free()
    k_hi = max(1, L - 1)
    assert np.all(np.isfinite(u)) and rel < 1.0
    assert cnt[k_hi - 1] >= N and np.all(cnt[:k_hi] >= N), cnt
    assert np.max(cnt[:k_hi - 1]) > cnt[k_hi - 1], cnt  # the undelayed groups ran ahead


@pytest.mark.parametrize("delay_rank", [-1, 1, 7])
def test_dist_delay(amg, ctx, delay_rank):
    """DMEM_DelayProc on the distributed MULT cycle (2 ranks over the host
    transport): every rank (-1), one rank, or none (rank 7 absent) waits 5 ms
    per cycle; the iterate is bit-identical in every case."""
    gen = amg.Gen(24, interp=amg.AMG_INTERP_LINEAR)
    f = amg.rhs_rand(0, 24 ** 3)
    base = amg.default_opts(smooth_weight=0.8, num_cycles=4, tol=0.0)
    u0, h0 = distributed(amg, gen, base, f, 4, 2, 0)
    opts = amg.default_opts(smooth_weight=0.8, num_cycles=4, tol=0.0, delay_type=amg.AMG_DELAY_ALL,
                            delay_usec=5000, delay_rank=delay_rank)
    t0 = time.perf_counter()
    u1, h1 = distributed(amg, gen, opts, f, 4, 2, 0)
    dt = time.perf_counter() - t0
    assert_bitwise(u1, u0, "delayed distributed iterate")
    np.testing.assert_array_equal(h1, h0)
    if delay_rank != 7:
        assert dt >= 4 * 0.005, dt


def coupling_run(amg, nranks, N=6, dus=20000, n=48):
    """every level's finish time (ms, rank by rank) of the distributed async
    additive solve, undelayed and with the coarsest correcting level delayed
    dus microseconds before each of its N corrections (delay_level)"""
    from test_gpu_dist import run_ranks
    gen = amg.Gen(n, interp=amg.AMG_INTERP_LINEAR)
    f = amg.rhs_rand(0, n ** 3)
    hub = amg.dist.ThreadMailbox(nranks, timeout=600.0)

    def rank(r, delay_level):
        kw = dict(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=0.8, num_cycles=N, tol=0.0, smooth_transfer=1)
        if delay_level >= 0:
            kw.update(delay_type=amg.AMG_DELAY_ALL, delay_usec=dus, delay_level=delay_level)
        opts = amg.default_opts(**kw)
        c = amg.Context(0, nstreams=gen.L)
        if nranks == 1:
            amg.dist.init_rccl(c, 1, 0, lambda b: b)
        else:
            amg.dist.init_host(c, nranks, r, amg.dist.HostTransport(hub, r))
        amg.dist.set_replicate_rows(c, 4096)
        D = amg.dist.DistHier(c, gen, opts, slab=True)
        D.async_solve(f[D.row0:D.row0 + D.n0])  # warm-up (setup of the async levels and channels)
        rel, cnt = D.async_solve(f[D.row0:D.row0 + D.n0])
        ms = D.async_level_ms()
        D.free()
        amg.dist.finalize(c)
        c.close()
        return rel, [int(x) for x in cnt], [float(x) for x in ms]

    base = run_ranks(nranks, lambda r: rank(r, -1))
    active = int(np.count_nonzero(base[0][1]))
    dl = active - 1
    dly = run_ranks(nranks, lambda r: rank(r, dl))
    gen.free()
    return {"active": active, "delayed": dl, "base": base, "dly": dly}


@pytest.mark.parametrize("nranks", [1, 2])
def test_dist_async_level_coupling(amg, nranks):
    """Levels of the distributed async additive solve are decoupled: each
    level group runs on its own host thread and stream and exchanges through
    its own device-resident channels (csrc/amg_link.cpp), as each DMEM grid
    polls only its own messages (DMEM_Comm.cpp:81-348).  Measured: the
    coarsest correcting level waits 20 ms before each of its N corrections
    (delay_level) and every level's finish time is read back
    (amg_dist_async_level_ms); the undelayed levels must finish in under half
    the delayed level's time, at one rank and at two (the host transport sets
    the channels up; every exchange goes through them).  The run is a child
    process with GPU_MAX_HW_QUEUES=16, so every level stream has a hardware
    queue of its own: with the default 4, streams share queues, and a delay
    kernel at the head of a shared queue stalls the other level behind it
    (that sharing, not the solver, coupled the single-rank levels of round 3)."""
    import json
    import os
    import subprocess
    import sys
    env = dict(os.environ, GPU_MAX_HW_QUEUES="16")
    out = subprocess.run([sys.executable, os.path.abspath(__file__), "coupling", str(nranks)], env=env,
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-4000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    N, dus = 6, 20000
    active, dl = res["active"], res["delayed"]
    assert active >= 3, res
    for r in range(nranks):
        ms0, ms1 = np.array(res["base"][r][2][:active]), np.array(res["dly"][r][2][:active])
        others = np.delete(ms1, dl)
        ratio = others / ms1[dl]
        print(f"{nranks} ranks, rank {r}: level finish ms undelayed {np.round(ms0, 2).tolist()}, "
              f"level {dl} delayed {N} x {dus / 1000:.0f} ms {np.round(ms1, 2).tolist()}, "
              f"undelayed levels' finish / delayed level's {np.round(ratio, 3).tolist()}")
        assert ms1[dl] >= N * dus / 1000 * 0.95, ms1
        assert np.all(ratio < 0.5), (ratio, "levels coupled")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "coupling":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from conftest import load_package
    res = coupling_run(load_package(), int(sys.argv[2]))
    print(json.dumps(res))
