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
        fmt = f"bsr3 ({'value-indexed' if A0.bsr3 == 1 else 'fp64'} 3x3 blocks)"
    else:
        mat_bytes, fmt = storage(A0.nrows, A0.nnz, A0.value_index, A0.dict_index, A0.row_pattern)
    spmv_bytes = mat_bytes + 16 * n
    # the same operator in value-indexed CSR (blocks off): the kernel it replaces
    ctx.set_bsr3(0)
    Ac = ctx.csr(n, n, rp, cj, v)
    ctx.set_bsr3(1)
    ms_csr = C.c_double()
    amg.check(amg.lib.amg_matvec_timed(ctx.h, Ac.h, x.h, y.h, 20, C.byref(ms_csr)))
    csr_bytes = storage(Ac.nrows, Ac.nnz, Ac.value_index, Ac.dict_index, Ac.row_pattern)[0] + 16 * n
    Ac.free()
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
           "relres_after": rn / r0, "cycles": a.warmup + a.steps,
           "setup_s": {"generate": t1 - t0, "classical": t2 - t1,
                       "galerkin_on": "gpu" if a.gpu_setup else "host"}}
    print(json.dumps(out), flush=True)
    Hd.free()
    ctx.close()


if __name__ == "__main__":
    main()
