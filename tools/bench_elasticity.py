"""Config 5 on one MI355X: the DMEM elasticity problem (amg_elast_*, beam-hex
refined r times, Q1 byVDIM) on the in-house classical hierarchy
(num_functions = 3, PMIS fixed seed, extended+i, theta 0.5: the DMEM
parameters), SMEM_Solve MULT V(1,1) weighted Jacobi.  Prints one JSON line:
V-cycle iterations/s, fine SpMV time and its bytes in the stored format."""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
from conftest import load_package  # noqa: E402
from bench import storage, HBM_PEAK_GBS  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--refine", type=int, default=5)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--coarsen", type=int, default=9)
    p.add_argument("--theta", type=float, default=0.5)
    p.add_argument("--omega", type=float, default=0.6)
    p.add_argument("--gpu-setup", type=int, default=1, help="Galerkin products on the GPU (classical opts.device)")
    p.add_argument("--async-ranks", type=int, default=0,
                   help="also run config 5's asynchronous additive cycle (DMEM_Add: ASYNC_MULTADD, smoothed "
                        "transfers composed) on this hierarchy as R row-partitioned ranks (threads on this GPU)")
    p.add_argument("--async-cycles", type=int, default=10)
    p.add_argument("--async-omega", type=float, default=None, help="smooth weight of the async cycle (default --omega)")
    p.add_argument("--async-runs", type=int, default=2)
    a = p.parse_args()
    amg = load_package()
    t0 = time.time()
    n, rp, cj, v, b = amg.classical.elasticity(a.refine)
    t1 = time.time()
    H = amg.classical.ClassicalAMG(n, rp, cj, v, coarsen_type=a.coarsen, strong_threshold=a.theta,
                                   num_functions=3, device=0 if a.gpu_setup else -1)
    t2 = time.time()
    print(f"[elast] r={a.refine}: {n} dofs, {len(cj)} nnz; generated {t1 - t0:.1f}s, classical setup "
          f"{t2 - t1:.1f}s, {H.L} levels", file=sys.stderr, flush=True)
    ctx = amg.Context(0, 4)
    opts = amg.default_opts(smooth_weight=a.omega, num_cycles=1 << 30, tol=0.0, profile=1)
    Hd = H.hierarchy(ctx, opts)
    As = Hd._keep[0]
    sizes = [m.nrows for m in As]
    opc = sum(m.nnz for m in As) / As[0].nnz
    fv = ctx.vec(b)
    r0 = Hd.solve_start(fv, ctx.vec(n))
    Hd.iterate(a.warmup)
    ctx.sync()
    t3 = time.perf_counter()
    Hd.iterate(a.steps)
    ctx.sync()
    t4 = time.perf_counter()
    rn = Hd.resnorm()
    x, y = ctx.vec(n), ctx.vec(n)
    x.set(1.0)
    ms = C.c_double()
    amg.check(amg.lib.amg_matvec_timed(ctx.h, As[0].h, x.h, y.h, 20, C.byref(ms)))
    A0 = As[0]
    if A0.bsr3:
        # 3x3 blocks (bsr3_kernel): per block 4 (column) + 12 (value indices,
        # 3 rows x 4 bytes) or 72 (fp64) bytes; per block row the pointer,
        # diagonal position and mode (9 bytes); blocks ~ nnz / 9
        per = 16 if A0.bsr3 == 1 else 76
        mat_bytes = per * (A0.nnz // 9) + 9 * (n // 3)
        fmt = (f"bsr3 ({'value-indexed' if A0.bsr3 == 1 else 'fp64'} 3x3 blocks, "
               f"{amg.lib.amg_mat_bsr3_slice(A0.h)} block rows per slice)")
    else:
        mat_bytes, fmt = storage(A0.nrows, A0.nnz, A0.value_index, A0.dict_index, A0.row_pattern)
    spmv_bytes = mat_bytes + 16 * n
    # the same operator in value-indexed CSR (blocks off): the kernel it replaces
    ctx.set_bsr3(0)
    Ac = ctx.csr(n, n, rp, cj, v)
    ctx.set_bsr3(2)  # the default
    ms_csr = C.c_double()
    amg.check(amg.lib.amg_matvec_timed(ctx.h, Ac.h, x.h, y.h, 20, C.byref(ms_csr)))
    csr_bytes = storage(Ac.nrows, Ac.nnz, Ac.value_index, Ac.dict_index, Ac.row_pattern)[0] + 16 * n
    Ac.free()
    # the classical coarse levels' SpMV on their stored bytes (long rows: the
    # csr_long_kernel passes that dominate the V-cycle)
    coarse = []
    for lvl in range(1, min(len(As), 6)):
        M = As[lvl]
        if M.nrows < 4096:
            break
        xl, yl = ctx.vec(M.ncols), ctx.vec(M.nrows)
        xl.set(1.0)
        msl = C.c_double()
        amg.check(amg.lib.amg_matvec_timed(ctx.h, M.h, xl.h, yl.h, 20, C.byref(msl)))
        b_l, f_l = storage(M.nrows, M.nnz, M.value_index, M.dict_index, M.row_pattern)
        b_l += 8 * (M.nrows + M.ncols)
        coarse.append({"level": lvl, "rows": int(M.nrows), "nnz": int(M.nnz), "per_row": M.nnz / M.nrows,
                       "format": f_l, "ms": msl.value, "bytes": b_l,
                       "gbs": b_l / (msl.value * 1e-3) / 1e9, "frac": b_l / (msl.value * 1e-3) / 1e9 / HBM_PEAK_GBS})
        xl.free()
        yl.free()
    out = {"workload": f"DMEM elasticity (config 5 restated) r={a.refine}: {n} dofs, beam-hex Q1 byVDIM, "
                       f"classical hierarchy (coarsen {a.coarsen}, ext+i, theta {a.theta}, 3 functions), "
                       f"SMEM_Solve MULT V(1,1) Jacobi w={a.omega}",
           "it_per_s": a.steps / (t4 - t3), "ms_per_step": (t4 - t3) * 1e3 / a.steps,
           "dofs": n, "nnz_A0": int(A0.nnz), "levels": len(sizes), "level_rows": sizes,
           "operator_complexity": opc, "matrix_format": fmt,
           "fine_spmv": {"ms": ms.value, "bytes": spmv_bytes, "gbs": spmv_bytes / (ms.value * 1e-3) / 1e9,
                         "frac": spmv_bytes / (ms.value * 1e-3) / 1e9 / HBM_PEAK_GBS},
           "fine_spmv_csr": {"ms": ms_csr.value, "bytes": csr_bytes,
                             "gbs": csr_bytes / (ms_csr.value * 1e-3) / 1e9},
           "roofline": {"bound": "hbm", "kernel": f"fine SpMV y = A0 x ({fmt})",
                        "achieved": spmv_bytes / (ms.value * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": spmv_bytes / (ms.value * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                        "alg_bytes_per_launch": spmv_bytes, "avg_launch_ms": ms.value},
           "coarse_spmv": coarse,
           "relres_after": rn / r0, "cycles": a.warmup + a.steps,
           "setup_s": {"generate": t1 - t0, "classical": t2 - t1,
                       "galerkin_on": "gpu" if a.gpu_setup else "host"}}
    Hd.free()
    ctx.close()
    if a.async_ranks:
        out["async_additive"] = async_leg(amg, H, b, a)
    print(json.dumps(out), flush=True)


def async_leg(amg, H, b, a):
    """DMEM_Add's asynchronous additive cycle (DMEM_Add.cpp:20-178) on the
    elasticity hierarchy: R ranks (threads, one GPU, per-level device-resident
    channels), every level group on its own host thread and stream, N
    corrections per level with the reference's smoothed transfers composed
    (smooth_transfer = 1).  Additive cycles/s = N over the slowest level's
    finish; relres after the race; the level finish times."""
    import numpy as np
    from test_gpu_classical import host_levels
    from test_gpu_dist import run_ranks, split_host
    lv = host_levels(amg, H)
    L = len(lv["A"])
    R, N = a.async_ranks, a.async_cycles
    w = a.async_omega if a.async_omega is not None else a.omega
    opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=w, num_cycles=N, tol=0.0, smooth_transfer=1)
    host = {k: [tuple(m) for m in v] for k, v in lv.items()}

    class _M:  # split_host wants .nrows / .ncols / .rowptr / .col / .val
        def __init__(self, t):
            self.nrows, self.ncols, self.rowptr, self.col, self.val = t
    host = {k: [_M(t) for t in v] for k, v in host.items()}
    cuts = tuple((i + 1) / R for i in range(R - 1))
    rs, parts = split_host(host, cuts)
    del host, lv
    hub = amg.dist.ThreadMailbox(R, timeout=1200.0)
    fb = np.ascontiguousarray(b, dtype=np.float64)

    def rank(r):
        c = amg.Context(0, nstreams=L + 2)
        if R == 1:
            amg.dist.init_rccl(c, 1, 0, lambda x: x)
        else:
            amg.dist.init_host(c, R, r, amg.dist.HostTransport(hub, r))
        A, P, Rm = parts[r]
        D = amg.dist.DistHier.from_parts(c, rs, A, P, Rm, opts)
        res = []
        for q in range(a.async_runs + 1):  # the first solve sets up the level groups and channels
            amg.dist.barrier(c)
            t1 = time.perf_counter()
            rel, cnt = D.async_solve(fb[D.row0:D.row0 + D.n0])
            dt = time.perf_counter() - t1
            if q:
                res.append((rel, [int(x) for x in cnt], [float(x) for x in D.async_level_ms()], dt))
        D.free()
        amg.dist.finalize(c)
        c.close()
        return res

    t0 = time.time()
    out = run_ranks(R, rank)
    runs = []
    for q in range(a.async_runs):
        lvms = np.max(np.array([out[r][q][2] for r in range(R)]), axis=0)
        active = int(np.count_nonzero(out[0][q][1]))
        slowest = float(np.max(lvms[:active]))
        runs.append({"relres": out[0][q][0], "corrections": out[0][q][1][:active],
                     "level_finish_ms": [round(x, 2) for x in lvms[:active].tolist()],
                     "wall_s": max(out[r][q][3] for r in range(R)), "cycles_per_s": N / (slowest * 1e-3)})
        print(f"[elast async] {R} ranks run {q}: relres {runs[-1]['relres']:.4e}, slowest level {slowest:.1f} ms",
              file=sys.stderr, flush=True)
    best = max(runs, key=lambda r: r["cycles_per_s"])
    return {"metric": "asynchronous additive cycles/s (every level N corrections)", "value": best["cycles_per_s"],
            "ranks": R, "num_cycles": N, "smooth_weight": w, "levels": L, "runs": runs,
            "workload": f"DMEM_Add ASYNC_MULTADD, smoothed transfers composed, {R} row-partitioned ranks "
                        "(threads) on one GPU, per-level device-resident channels",
            "setup_and_runs_s": time.time() - t0}


if __name__ == "__main__":
    main()
