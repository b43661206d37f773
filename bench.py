"""bench.py -- V-cycle iterations/s and fine-grid SpMV HBM GB/s on the 512^3
7-pt Laplacian (BASELINE.json metric), one process per GPU.

A step is one outer iteration of SMEM_Solve (SMEM_Solve.cpp:128-240): one
multiplicative V(1,1) cycle with weighted Jacobi (w = 0.8) over the whole
9-level geometric Galerkin hierarchy, the outer residual f - A u and its
2-norm.  Inputs (matrices, RHS, iterate) are resident in HBM before the timed
region.  Scaling is strong: the 512^3 problem is split into z-slabs across
ranks.  Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--n", type=int, default=512)
    p.add_argument("--smooth-weight", type=float, default=0.8)
    p.add_argument("--reuse-outer-residual", type=int, default=2)
    p.add_argument("--cpu-baseline", type=int, default=1)
    p.add_argument("--cpu-cycles", type=int, default=20)
    p.add_argument("--cpu-all-cores", type=int, default=3,
                   help="outer iterations of the CPU sample also timed on every host core "
                        "(os.cpu_count() threads); 0: off")
    p.add_argument("--fuse-outer", type=int, default=-1,
                   help="level 0's last post sweep fused with the outer residual (0 off, 1, 2; -1: the library "
                        "default / AMG_FUSE_OUTER)")
    p.add_argument("--general", type=int, default=1,
                   help="also time the general (plain-CSR, CSR-transfer) V-cycle on the same 512^3 solve")
    p.add_argument("--seq-cycles", type=int, default=200,
                   help="outer iterations of the config-1 (64^3) SEQ leg on one core, and of its GPU rate")
    p.add_argument("--spmv-reps", type=int, default=20)
    p.add_argument("--ajac-ranks", type=int, default=2,
                   help="ranks (processes) of the DMEM_AsyncSmooth overlap leg on the same operator; <2: off")
    p.add_argument("--ajac-sweeps", type=int, default=12)
    p.add_argument("--force-dist", type=int, default=0,
                   help="run the distributed (RCCL) path even at one rank")
    p.add_argument("--dist-form", choices=("slab", "rows"), default="slab",
                   help="distributed hierarchy: z-slab extended operators (default) or the "
                        "row-partitioned [owned | ghost] CSR form")
    return p.parse_args()


def storage(nrows, nnz, vi, dc, rp, pp=0, mp=0):
    """(matrix bytes the hot kernels stream per pass, format name), DESIGN.md Sec.4:
    master-pattern and paired-row-pattern CSR read one byte per pair of rows; row-pattern-coded
    CSR one byte per row; dictionary-coded one byte per
    entry + the row pointer; value-indexed 4 (col) + 1 per entry + the row
    pointer; CSR 4 (col) + 8 (val) per entry + the row pointer."""
    if pp and mp:
        vals = "one value per offset" if mp < 0 else "per-pattern values"
        return (nrows + 1) // 2, (f"csr-mp ({abs(mp)}-offset master list, {vals}, {pp} row-pair use masks "
                                  f"over {rp} row patterns)")
    if pp:
        return (nrows + 1) // 2, (f"csr-rpp ({pp} row-pair patterns over {rp} row patterns and a "
                                  f"{dc}-entry (offset, value) dictionary)")
    if rp:
        return nrows, f"csr-rp ({rp} row patterns over a {dc}-entry (offset, value) dictionary)"
    if dc:
        return nnz + 4 * (nrows + 1), f"csr-dc ({dc}-entry (offset, value) dictionary)"
    if vi:
        return 5 * nnz + 4 * (nrows + 1), f"csr-vi ({vi}-entry value table)"
    return 12 * nnz + 4 * (nrows + 1), "csr"


def load_traffic(n, kernel):
    """HBM bytes per launch of a fine-level kernel from the rocprofv3 --pmc passes
    (FETCH_SIZE and WRITE_SIZE, corrected by calibration streams of known size:
    tools/pmc_fine.py -> profiles/traffic.json "kernels"), if profiled for n."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        d = json.load(open(path))
        return d[str(n)]["kernels"][kernel]["bytes_per_launch"]
    except Exception:
        return None


def fine_kernels(n0, mat_bytes, ms, launches, fused, fmt, fused_prolong=0, fused_outer=0):
    """Per-launch time (HIP events on the compute stream inside the timed loop)
    and algorithmic bytes of each fine-level kernel of a step.
    Profile categories: 0 level-0 residual (fused with R0 when fused & 1),
    1 post-smoothing sweep (fused with P0 when fused_prolong & 1), 2 R0, 3 P0
    prolongation + correction, 4 outer residual + norm (fused with the next
    cycle's first sweep)."""
    def per(c):
        return ms[c] / launches[c] if launches[c] else None
    out = {}
    if fused_outer:
        # one march: the last post sweep u' = u + w (f - A u)./a and the outer
        # residual of u' + norm + the next first sweep u'' (mz_sweep_outer_kernel)
        out["post_sweep_outer_residual"] = (
            per(4), mat_bytes + (32 if fused_outer == 1 else 24) * n0,
            "level-0 post-smoothing sweep fused with the outer residual r = f - A0 u' + norm partials and the "
            f"next cycle's first Jacobi sweep in one plane march (reads f, u; writes {'u, ' if fused_outer == 1 else ''}"
            f"u_next; {fmt}" + ("" if fused_outer == 1 else "; u' itself written only in a batch's last step") + ")")
    else:
        out["outer_residual_sweep"] = (per(4), mat_bytes + 24 * n0,
                                       "outer residual r = f - A0 u + norm partials, fused with the next "
                                       f"cycle's first Jacobi sweep (reads f, u; writes u_next; {fmt})")
    if fused_outer:
        pass
    elif fused_prolong & 1:
        out["prolong_sweep"] = (per(1), mat_bytes + 24 * n0 + 8 * (n0 // 8),
                                "geometric prolongation u + P0 e fused into the post-smoothing Jacobi sweep "
                                f"(reads f, u, e; writes u_next; {fmt})")
    else:
        out["post_sweep"] = (per(1), mat_bytes + 24 * n0,
                             f"post-smoothing Jacobi sweep (reads f, u; writes u_next; {fmt})")
    if fused & 1:
        # the coarse level's zero-guess sweep rides on it (reads a_1, writes u_1)
        out["residual_restrict"] = (per(0), mat_bytes + 16 * n0 + 24 * (n0 // 8),
                                    "level-0 residual fused with the geometric restriction and level 1's "
                                    "zero-guess sweep (reads f, u, a_1; writes f_1, u_1)")
    else:
        out["residual"] = (per(0), mat_bytes + 24 * n0, f"level-0 residual ({fmt})")
        out["restrict0"] = (per(2), None, "R0 restriction")
    if fused_prolong & 1:
        pass
    elif fused & 2:
        out["prolong0"] = (per(3), 16 * n0 + 8 * (n0 // 8),
                           "geometric prolongation + correction u += P0 e (reads u, e; writes u)")
    else:
        out["prolong0"] = (per(3), None, "P0 prolongation + correction (CSR form)")
    res = {}
    for k, (t, b, what) in out.items():
        if t is None or b is None:
            continue
        gbs = b / (t * 1e-3) / 1e9
        res[k] = {"ms": t, "bytes": b, "gbs": gbs, "frac": gbs / HBM_PEAK_GBS, "what": what}
    return res


def host_info():
    """the host CPU the baseline ran on (model, cores, binding)"""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count()
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "affinity_cpus": avail,
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"), "OMP_PROC_BIND": os.environ.get("OMP_PROC_BIND"),
            "OMP_PLACES": os.environ.get("OMP_PLACES")}


# taken at import, before the oracle's OpenMP runtime binds this thread (OMP_PROC_BIND)
HOST_INFO = host_info()


def seq_baseline(amg, args):
    """Config 1 (SEQ_AMG 64^3, sync Jacobi V-cycle on CPU): the oracle's loops on
    ONE thread (or_set_threads(1): the SEQ configuration of BASELINE.md Sec.3)
    for args.seq_cycles outer iterations, beside the GPU's rate on the same
    64^3 solve (HIP path, same hierarchy / RHS / options)."""
    from oracle import pyoracle as po
    n = 64
    gen = amg.Gen(n, interp=amg.AMG_INTERP_LINEAR)
    L = gen.L
    host = {tag: [po.Csr(*gen.host_csr(code, l)) for l in range(cnt)]
            for tag, code, cnt in (("A", amg.AMG_GEN_A, L), ("P", amg.AMG_GEN_P, L - 1), ("R", amg.AMG_GEN_R, L - 1))}
    f = amg.rhs_rand(0, n ** 3)
    po.lib().or_set_threads(1)
    try:
        opts = po.make_opts(smooth_weight=args.smooth_weight, num_cycles=args.seq_cycles, tol=0.0, num_threads=1)
        u, hist, k = po.Hier(host["A"], host["P"], host["R"], opts).solve(f)
        secs = po.lib().or_last_loop_seconds()
    finally:
        po.lib().or_set_threads(max(1, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
    gen.free()
    return {"value": k / secs, "unit": "V-cycle iters/s", "cores": 1, "kind": "port",
            "sample": f"config 1: {k} outer iterations (V(1,1) Jacobi w={args.smooth_weight} + residual + norm) "
                      f"of the {n}^3 7-pt solve ({L}-level geometric Galerkin hierarchy), oracle/amg_oracle.c "
                      "loops on one thread", "seconds": secs, "relres": float(hist[-1] / hist[0])}


def gpu_config1(amg, args):
    """the GPU's rate on config 1's 64^3 solve (the SEQ leg's workload)"""
    n = 64
    ctx = amg.Context(device=0, nstreams=4)
    if args.fuse_outer >= 0:
        ctx.set_fuse_outer(args.fuse_outer)
    gen = amg.Gen(n, interp=amg.AMG_INTERP_LINEAR)
    L = gen.L
    As = [gen.register(ctx, amg.AMG_GEN_A, l) for l in range(L)]
    Ps = [gen.register(ctx, amg.AMG_GEN_P, l) for l in range(L - 1)]
    Rs = [gen.register(ctx, amg.AMG_GEN_R, l) for l in range(L - 1)]
    opts = amg.default_opts(smooth_weight=args.smooth_weight, num_cycles=1 << 30, tol=0.0,
                            reuse_outer_residual=args.reuse_outer_residual)
    H = amg.Hier(ctx, As, Ps, Rs, opts)
    f = ctx.vec(amg.rhs_rand(0, n ** 3))
    u0 = ctx.vec(n ** 3)
    r0 = H.solve_start(f, u0)
    H.iterate(20)
    ctx.sync()
    t1 = time.perf_counter()
    H.iterate(args.seq_cycles)
    ctx.sync()
    dt = time.perf_counter() - t1
    rel = H.resnorm() / r0
    H.free()
    for M in As + Ps + Rs:
        M.free()
    gen.free()
    ctx.close()
    return {"value": args.seq_cycles / dt, "unit": "V-cycle iters/s", "steps": args.seq_cycles,
            "relres_after_warmup_and_steps": rel, "workload": f"config 1 ({n}^3) on the GPU"}


def general_csr_vcycle(amg, gen, f_host, args):
    """The same 512^3 solve on the GENERAL path -- the one a BoomerAMG or
    elasticity hierarchy takes: every operator in plain CSR (no value index,
    dictionary, row / pair / master patterns, no plane march) and the transfers
    as CSR SpMVs (no geometric kernels, no fused residual + restriction):
    csr_tile_kernel for every SpMV / residual / sweep (SMEM_MatVec.cpp:95-259,
    SMEM_Smooth.cpp:6-49).  Timed like the headline (HIP events per fine
    kernel on the compute stream), with its own dominant-kernel roofline on the
    CSR bytes of SURVEY.md Sec.8(d) (12 nnz + 28 n for a residual / sweep)."""
    n = args.n
    ctx = amg.Context(device=0, nstreams=4)
    for fn in (ctx.set_value_index, ctx.set_dict_index, ctx.set_row_pattern, ctx.set_pair_pattern,
               ctx.set_master_pattern, ctx.set_fuse_transfer):
        fn(0)
    ctx.set_plane_march(0)
    t0 = time.time()
    L = gen.L
    As = [gen.register(ctx, amg.AMG_GEN_A, l) for l in range(L)]
    Ps = [gen.register(ctx, amg.AMG_GEN_P, l) for l in range(L - 1)]
    Rs = [gen.register(ctx, amg.AMG_GEN_R, l) for l in range(L - 1)]
    assert As[0].value_index == 0 and As[0].plane_march == 0
    opts = amg.default_opts(smooth_weight=args.smooth_weight, num_cycles=1 << 30, tol=0.0,
                            reuse_outer_residual=args.reuse_outer_residual, profile=1)
    H = amg.Hier(ctx, As, Ps, Rs, opts)
    assert H.fused == 0
    f = ctx.vec(f_host)
    u0 = ctx.vec(n ** 3)
    r0 = H.solve_start(f, u0)
    H.iterate(args.warmup)
    ctx.sync()
    H.profile(reset=True)
    t1 = time.perf_counter()
    H.iterate(args.steps)
    ctx.sync()
    dt = time.perf_counter() - t1
    rel = H.resnorm() / r0
    ms, launches = H.profile(reset=True)
    n0, z0 = As[0].nrows, As[0].nnz
    zP, zR, nc = Ps[0].nnz, Rs[0].nnz, As[1].nrows
    def per(c):
        return ms[c] / launches[c] if launches[c] else None
    # algorithmic CSR bytes per launch (b = 12)
    kern = {"outer_residual_sweep": (per(4), 12 * z0 + 36 * n0, "outer residual + norm fused with the next "
                                     "first Jacobi sweep, plain CSR (reads f, u; writes r... u_next)"),
            "post_sweep": (per(1), 12 * z0 + 28 * n0, "post-smoothing Jacobi sweep, plain CSR"),
            "residual": (per(0), 12 * z0 + 28 * n0, "level-0 residual r = f - A u, plain CSR"),
            "restrict0": (per(2), 12 * zR + 4 * nc + 8 * n0 + 8 * nc, "R0 restriction SpMV, plain CSR"),
            "prolong0": (per(3), 12 * zP + 28 * n0 + 8 * nc, "P0 prolongation + correction u += P0 e, plain CSR")}
    if args.reuse_outer_residual >= 2:
        kern["outer_residual_sweep"] = (per(4), 12 * z0 + 28 * n0, kern["outer_residual_sweep"][2]
                                        .replace("r... ", ""))
    res = {}
    for k, (t, b, what) in kern.items():
        if t is None:
            continue
        gbs = b / (t * 1e-3) / 1e9
        res[k] = {"ms": t, "bytes": b, "gbs": gbs, "frac": gbs / HBM_PEAK_GBS, "what": what}
    dom = max(res, key=lambda k: res[k]["ms"])
    out = {"value": args.steps / dt, "unit": "V-cycle iters/s", "ms_per_step": dt * 1e3 / args.steps,
           "steps": args.steps, "relres": rel, "setup_s": time.time() - t0 - dt,
           "workload": f"{n}^3 7-pt, the headline's solve with every operator plain CSR and CSR transfers "
                       "(compressed forms, plane march and geometric / fused transfers off)",
           "fine_kernels": res,
           "roofline": {"bound": "hbm", "kernel": f"{dom}: {res[dom]['what']}", "achieved": res[dom]["gbs"],
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": res[dom]["frac"],
                        "alg_bytes_per_launch": res[dom]["bytes"], "avg_launch_ms": res[dom]["ms"]}}
    log(f"[general] plain-CSR V-cycle {out['value']:.1f} it/s ({out['ms_per_step']:.2f} ms/step); dominant "
        f"{dom} {res[dom]['ms']:.3f} ms = {res[dom]['frac']:.3f} of peak")
    H.free()
    for M in As + Ps + Rs:
        M.free()
    ctx.close()
    return out


def async_jacobi_overlap(args):
    """DMEM_AsyncSmooth (DMEM_Smooth.cpp:16-313) on the same 512^3 operator as
    args.ajac_ranks row-partitioned ranks, one PROCESS each on this GPU (the
    production layout: every process with the box's default hardware queues),
    under torch.distributed.run as child processes (tools/bench_async_jacobi.py):
    per rank the fraction of each sweep's exchange window (the delta copies on
    the communication stream) that the interior product on the compute stream
    covers (amg_dist_async_jacobi_stats), and the sweeps per second"""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.ajac_ranks}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "tools", "bench_async_jacobi.py"),
           "--grid", str(args.n), "--sweeps", str(args.ajac_sweeps), "--omega", str(args.smooth_weight)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if p.returncode != 0:
        raise RuntimeError(f"async Jacobi leg exit {p.returncode}: {p.stderr[-800:]}")
    res = json.loads(p.stdout.strip().splitlines()[-1])
    log(f"[ajac] {args.ajac_ranks} processes: {res['sweeps_per_s']:.1f} sweeps/s, exchange hidden "
        f"{res['hidden_fraction_min']:.3f} (min) / {res['hidden_fraction_mean']:.3f} (mean)")
    return res


def cpu_baseline(gen, amg, f, args):
    """The oracle (C restatement of SMEM_Solve, OpenMP) on the host cores, on a
    bounded sample of the same workload: args.cpu_cycles outer iterations of
    the same 512^3 solve."""
    from oracle import pyoracle as po
    t0 = time.time()
    L = gen.L
    host = {}
    for tag, code, cnt in (("A", amg.AMG_GEN_A, L), ("P", amg.AMG_GEN_P, L - 1),
                           ("R", amg.AMG_GEN_R, L - 1)):
        host[tag] = [po.Csr(*gen.host_csr(code, l)) for l in range(cnt)]
    log(f"[cpu] host hierarchy built in {time.time() - t0:.1f}s")
    opts = po.make_opts(smooth_weight=args.smooth_weight, num_cycles=args.cpu_cycles, tol=0.0)
    H = po.Hier(host["A"], host["P"], host["R"], opts)
    u, hist, k = H.solve(f)
    secs = po.lib().or_last_loop_seconds()
    threads = po.lib().or_num_threads()
    # OMP_NUM_THREADS=$(nproc), OMP_PROC_BIND=close -- the
    # same sample again on every host core (os.cpu_count(): the whole machine,
    # beyond this process's share of it where the box gives it one)
    allc = None
    ncpu = os.cpu_count() or 1
    if args.cpu_all_cores > 0 and ncpu > threads:
        # a shorter sample: where the process's CPU share is smaller than the
        # machine (a GPU box's slice) these threads oversubscribe it
        HA = po.Hier(host["A"], host["P"], host["R"],
                     po.make_opts(smooth_weight=args.smooth_weight, num_cycles=args.cpu_all_cores, tol=0.0))
        po.lib().or_set_threads(ncpu)
        try:
            ua, ha, ka = HA.solve(f)
            sa = po.lib().or_last_loop_seconds()
            ta = po.lib().or_num_threads()
            allc = {"value": ka / sa, "unit": "V-cycle iters/s", "cores": ta, "seconds": sa,
                    "affinity_cpus": HOST_INFO.get("affinity_cpus"),
                    "sample": f"{ka} outer iterations of the same solve on {ta} threads = os.cpu_count() "
                              f"(OMP_PROC_BIND {os.environ.get('OMP_PROC_BIND')}; this process may run on "
                              f"{HOST_INFO.get('affinity_cpus')} of them)"}
            log(f"[cpu] all cores: {allc['value']:.4f} it/s on {ta} threads")
        finally:
            po.lib().or_set_threads(threads)
            del HA
    del H, host
    return ({"value": k / secs, "unit": "V-cycle iters/s", "cores": threads, "kind": "port",
             "sample": f"{k} outer iterations (V(1,1) Jacobi + residual + norm) of the same "
                       f"{args.n}^3 solve, oracle/amg_oracle.c OpenMP, {threads} threads",
             "seconds": secs, "all_cores": allc,
             "host": dict(HOST_INFO, **{k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OMP_PROC_BIND",
                                                                      "OMP_PLACES")})}, u, hist[-1] / hist[0])


def check_parity(u_par, u_cpu, rel_cpu, cycles):
    """The headline workload's result against the oracle: the GPU iterate after
    `cycles` outer iterations of the same solve must be bit-identical to the
    oracle's (SMEM_Solve.cpp:128-215, SMEM_Sync_AMG.cpp:8-145), and the final
    relative residual equal to rtol 1e-12 (reduction order differs)."""
    if u_par is None:
        return None
    u_gpu, rel_gpu = u_par
    same = u_gpu.view(np.uint64) == u_cpu.view(np.uint64)
    same |= np.isnan(u_gpu) & np.isnan(u_cpu)
    nbad = int(u_gpu.size - np.count_nonzero(same))
    maxrel = float(np.max(np.abs(u_gpu - u_cpu)) / max(np.max(np.abs(u_cpu)), 1e-300))
    return {"cycles": cycles, "iterate_bitwise": bool(nbad == 0), "mismatched_entries": nbad,
            "max_abs_diff_rel": maxrel, "relres_gpu": float(rel_gpu), "relres_oracle": float(rel_cpu),
            "relres_rtol_ok": bool(abs(rel_gpu - rel_cpu) <= 1e-12 * abs(rel_cpu))}


def launch_ranks(args):
    """`bench.py --gpus N` with N > 1 outside torchrun: start torchrun with N ranks
    as a child process (nothing here has touched the GPU yet) and exit with its
    status; the ranks re-enter main() with WORLD_SIZE set."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        log(f"[bench] --gpus {args.gpus} but WORLD_SIZE {world}: refusing to report a mislabeled run")
        sys.exit(2)
    if world > 1 or args.force_dist:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
        import bench_dist
        return bench_dist.main(args, world, rank)

    from conftest import load_package
    amg = load_package()
    n = args.n
    t0 = time.time()
    ctx = amg.Context(device=0, nstreams=4)
    if args.fuse_outer >= 0:
        ctx.set_fuse_outer(args.fuse_outer)
    gen = amg.Gen(n, interp=amg.AMG_INTERP_LINEAR)
    L = gen.L
    As = [gen.register(ctx, amg.AMG_GEN_A, l) for l in range(L)]
    Ps = [gen.register(ctx, amg.AMG_GEN_P, l) for l in range(L - 1)]
    Rs = [gen.register(ctx, amg.AMG_GEN_R, l) for l in range(L - 1)]
    log(f"[gpu] {L}-level hierarchy registered in {time.time() - t0:.1f}s; "
        f"nnz(A0)={As[0].nnz} nnz(P0)={Ps[0].nnz}")
    opts = amg.default_opts(smooth_weight=args.smooth_weight, num_cycles=1 << 30, tol=0.0,
                            reuse_outer_residual=args.reuse_outer_residual, profile=1)
    H = amg.Hier(ctx, As, Ps, Rs, opts)
    f_host = amg.rhs_rand(0, n ** 3)
    f = ctx.vec(f_host)
    u0 = ctx.vec(n ** 3)
    r0 = H.solve_start(f, u0)
    H.iterate(args.warmup)
    ctx.sync()
    H.profile(reset=True)
    ctx.sync()
    t1 = time.perf_counter()
    H.iterate(args.steps)
    ctx.sync()
    t2 = time.perf_counter()
    rn = H.resnorm()
    ms, launches = H.profile(reset=True)
    dt = t2 - t1
    value = args.steps / dt
    log(f"[gpu] {args.steps} steps in {dt * 1e3:.2f} ms -> {value:.2f} it/s; relres {rn / r0:.3e}")
    u_par = None
    if args.cpu_baseline:
        # parity leg (untimed): restart the same solve and run exactly the
        # oracle's cpu_cycles outer iterations, keep the iterate for the check
        u0.set(0.0)
        r0p = H.solve_start(f, u0)
        H.iterate(args.cpu_cycles)
        H.get_u(u0)
        u_par = (u0.download(), H.resnorm() / r0p)

    n0 = As[0].nrows
    z0 = As[0].nnz
    # matrix bytes per pass in the format the kernels stream
    mat_bytes, fmt = storage(n0, z0, As[0].value_index, As[0].dict_index, As[0].row_pattern,
                             As[0].pair_pattern, As[0].master_pattern)
    fused = H.fused
    fused_prolong = H.fused_prolong
    fused_outer = H.fused_outer
    plane_march = As[0].plane_march
    kernels = fine_kernels(n0, mat_bytes, ms, launches, fused, fmt, fused_prolong, fused_outer)
    # fine-grid SpMV y = A x (matrix + x + y), events on the same stream
    x = ctx.vec(n0)
    x.set(1.0)
    y = ctx.vec(n0)
    import ctypes as C
    spmv_ms = C.c_double()
    amg.check(amg.lib.amg_matvec_timed(ctx.h, As[0].h, x.h, y.h, args.spmv_reps, C.byref(spmv_ms)))
    spmv_bytes = mat_bytes + 16 * n0
    spmv_gbs = spmv_bytes / (spmv_ms.value * 1e-3) / 1e9
    # the general kernels on the same operator: A0 registered again with the
    # compressed forms off (plain CSR, the reference's storage) and with only the
    # value index on (CSR-VI), timed the same way -- the kernels an unstructured
    # (BoomerAMG / elasticity) hierarchy runs
    general = {}
    for tag, vi in (("csr", 0), ("csr_vi", 1)):
        ctx.set_value_index(vi)
        ctx.set_dict_index(0)
        ctx.set_row_pattern(0)
        ctx.set_pair_pattern(0)
        ctx.set_master_pattern(0)
        Ag = gen.register(ctx, amg.AMG_GEN_A, 0)
        gms = C.c_double()
        amg.check(amg.lib.amg_matvec_timed(ctx.h, Ag.h, x.h, y.h, args.spmv_reps, C.byref(gms)))
        gb, gfmt = storage(n0, z0, Ag.value_index, 0, 0)
        gbytes = gb + 16 * n0
        general[tag] = {"format": gfmt, "ms": gms.value, "bytes": gbytes,
                        "gbs": gbytes / (gms.value * 1e-3) / 1e9,
                        "frac": gbytes / (gms.value * 1e-3) / 1e9 / HBM_PEAK_GBS}
        log(f"[gpu] fine SpMV {gfmt}: {gms.value:.3f} ms ({general[tag]['gbs']:.0f} GB/s)")
        Ag.free()
    for fn in (ctx.set_value_index, ctx.set_dict_index, ctx.set_row_pattern, ctx.set_pair_pattern,
               ctx.set_master_pattern):
        fn(1)
    # practical ceiling: STREAM triad over three 2 GiB arrays on the same device
    triad = C.c_double()
    amg.check(amg.lib.amg_stream_triad(ctx.h, 1 << 28, 10, C.byref(triad)))
    log(f"[gpu] STREAM triad {triad.value:.0f} GB/s")
    for k, v in kernels.items():
        log(f"[gpu] {k}: {v['ms']:.3f} ms, {v['gbs']:.0f} GB/s ({v['frac']:.3f} of peak, "
            f"{v['gbs'] / triad.value:.3f} of triad)")
    log(f"[gpu] fine SpMV {spmv_ms.value:.3f} ms ({spmv_gbs:.0f} GB/s)")
    dom = max(kernels, key=lambda k: kernels[k]["ms"])
    dk = kernels[dom]
    roofline = {"bound": "hbm", "kernel": f"{dom}: {dk['what']}", "achieved": dk["gbs"], "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": dk["frac"], "traffic": load_traffic(n, dom),
                "alg_bytes_per_launch": dk["bytes"], "avg_launch_ms": dk["ms"],
                "frac_of_stream_triad": dk["gbs"] / triad.value,
                "selection": "the fine-level kernel with the largest time per step (fine_kernels)"}
    x.free()
    y.free()
    H.free()
    for M in As + Ps + Rs:
        M.free()
    ctx.close()

    ajac = None
    if args.ajac_ranks > 1:
        try:
            ajac = async_jacobi_overlap(args)
        except Exception as e:  # noqa: BLE001
            log(f"[ajac] failed: {e!r}")
    vgen = None
    if args.general:
        try:
            vgen = general_csr_vcycle(amg, gen, f_host, args)
        except Exception as e:  # noqa: BLE001
            log(f"[general] failed: {e!r}")
    cpu, parity, seq = None, None, None
    if args.cpu_baseline:
        # OMP_PROC_BIND=close for the SMEM leg; read by
        # libgomp when the oracle library loads, which happens below
        os.environ.setdefault("OMP_PROC_BIND", "close")
        try:
            seq = {"cpu": seq_baseline(amg, args), "gpu": gpu_config1(amg, args)}
            seq["gpu_over_cpu"] = seq["gpu"]["value"] / seq["cpu"]["value"]
            log(f"[seq] config 1 (64^3): CPU 1 core {seq['cpu']['value']:.2f} it/s, GPU {seq['gpu']['value']:.1f} it/s")
        except Exception as e:  # noqa: BLE001
            log(f"[seq] config-1 leg failed: {e!r}")
        try:
            cpu, u_cpu, rel_cpu = cpu_baseline(gen, amg, f_host, args)
            log(f"[cpu] {cpu['value']:.4f} it/s on {cpu['cores']} threads")
            parity = check_parity(u_par, u_cpu, rel_cpu, args.cpu_cycles)
            log(f"[parity] {parity}")
        except Exception as e:  # the GPU number stands on its own
            log(f"[cpu] baseline failed: {e!r}")
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "V-cycle iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (7-pt Laplacian, RandDouble(-1,1) RHS after srand(0))",
        "config": {"workload": f"{n}^3 7-pt Laplacian, SMEM_Solve MULT V(1,1) Jacobi w={args.smooth_weight}, "
                               f"{L}-level geometric Galerkin hierarchy, outer residual + norm per step",
                   "n": n, "levels": L, "nnz_A0": z0, "rows": n0,
                   "reuse_outer_residual": args.reuse_outer_residual,
                   "matrix_format": fmt, "plane_march": plane_march,
                   "march_points": [A.march_points for A in As], "geometric_transfers": fused,
                   "fused_prolong_sweep": fused_prolong,
                   "fused_post_sweep_outer_residual": fused_outer,
                   "parallelism": "single GPU"},
        "fine_spmv": {"gbs": spmv_gbs, "ms": spmv_ms.value, "bytes": spmv_bytes,
                      "frac": spmv_gbs / HBM_PEAK_GBS, "format": fmt},
        "fine_spmv_csr": general["csr"],
        "fine_spmv_csr_vi": general["csr_vi"],
        "roofline_csr": {"bound": "hbm", "kernel": "fine-grid SpMV y = A0 x, plain CSR tile kernel",
                         "achieved": general["csr"]["gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": general["csr"]["frac"], "alg_bytes_per_launch": general["csr"]["bytes"],
                         "avg_launch_ms": general["csr"]["ms"]},
        "stream_triad_gbs": triad.value,
        "roofline": roofline,
        "fine_kernels": kernels,
        "cpu_baseline": cpu,
        "cpu_baseline_seq": seq,
        "vcycle_general_csr": vgen,
        "async_jacobi_overlap": ajac,
        "parity": parity,
        "final_relres": rn / r0,
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
