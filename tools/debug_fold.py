"""Round-5 debug: FULL_ASYNC hybrid JGS with the level-0 correction folded
into the JGS (AMG_JGS_FOLD) against the oracle under round robin, timed."""
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_package  # noqa: E402

amg = load_package()
from oracle import pyoracle as oracle  # noqa: E402
from async_band import blocks64  # noqa: E402
from test_gpu_solve import gpu_hier, hierarchy, oracle_opts  # noqa: E402

_, L, host = hierarchy(amg, oracle, 64, amg.AMG_INTERP_LINEAR)
f = amg.rhs_rand(0, 64 ** 3)
ctx = amg.Context(0, nstreams=16)
for sched in (3, 0):
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smoother=amg.AMG_HYBRID_JGS, smooth_weight=0.8,
                            num_cycles=15, tol=0.0, async_schedule=sched, num_threads=0,
                            jgs_block_rows=64)
    H, _ = gpu_hier(amg, ctx, host, opts)
    H.async_solve(f)
    ctx.sync()
    t0 = time.perf_counter()
    u, rel, cnt = H.async_solve(f)
    ctx.sync()
    dt = time.perf_counter() - t0
    H.free()
    msg = f"sched {sched} fold {os.environ.get('AMG_JGS_FOLD', '1')}: {dt * 1e3:.2f} ms, relres {rel:.6e}"
    if sched == 3:
        OH = oracle.Hier(host["A"], host["P"], host["R"], oracle_opts(oracle, opts))
        for lev, blk in blocks64(host).items():
            OH.set_blocks(lev, blk)
        oracle.lib().or_set_async_schedule(3)
        try:
            uo, relo, _ = OH.async_add(f, [1] * L)
        finally:
            oracle.lib().or_set_async_schedule(0)
        msg += f", oracle {relo:.6e}, differing {int(np.count_nonzero(u.view(np.uint64) != uo.view(np.uint64)))}"
    print(msg, flush=True)
ctx.close()
