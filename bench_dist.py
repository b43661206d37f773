"""bench_dist.py -- the N>1 leg of bench.py (launched by torchrun, one rank per GPU).

The 512^3 problem is split into z-slabs (strong scaling).  Every rank builds
its slab rows of every distributed level from the structured generator, the
RCCL communicator is created from a unique id broadcast over the gloo group
torchrun sets up, and each step is one SMEM_Solve outer iteration of the
slab-distributed V-cycle (ghost rows over RCCL p2p on a communication stream,
overlapped with the slab interior; replicated coarse levels; RCCL allreduce
of the residual norm).  Time = max over ranks of the K timed steps, bracketed
by barriers and device synchronisation.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main(args, world, rank):
    import torch
    import torch.distributed as tdist
    from conftest import load_package
    from bench import METRIC, HBM_PEAK_GBS, storage

    local = int(os.environ.get("LOCAL_RANK", rank))
    # stdout carries exactly one JSON line: gloo / RCCL banners go to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    amg = load_package()
    n = args.n
    t0 = time.time()
    ctx = amg.Context(device=local, nstreams=2)

    def bcast(obj):
        lst = [obj]
        tdist.broadcast_object_list(lst, src=0)
        return lst[0]

    amg.dist.init_rccl(ctx, world, rank, bcast)
    gen = amg.Gen(n, interp=amg.AMG_INTERP_LINEAR)
    opts = amg.default_opts(smooth_weight=args.smooth_weight, num_cycles=1 << 30, tol=0.0,
                            reuse_outer_residual=args.reuse_outer_residual, profile=1)
    slab = getattr(args, "dist_form", "slab") == "slab"
    D = amg.dist.DistHier(ctx, gen, opts, slab=slab)
    nnz_local, vi, dc, rp = D.matrix_info(0)
    Ld, geo_mask, fused0 = D.slab_info()
    if slab:
        # the extended slab operator streams its owned planes (plane march:
        # n/2 pattern bytes per pass, as one GPU)
        mat_bytes, fmt = (D.n0 + 1) // 2, ("7-pt plane march over the owned planes of the extended slab "
                                            "operator (csr-mp master form, one pattern byte per row pair)")
    else:
        mat_bytes, fmt = storage(D.n0, nnz_local, vi, dc, rp, D.pair_pattern(0))
    if rank == 0:
        log(f"[dist] {world} ranks, {gen.L} levels, slab {D.n0} rows / {nnz_local} nnz on rank 0; "
            f"setup {time.time() - t0:.1f}s")
    f = amg.rhs_rand(D.row0, D.row0 + D.n0)
    r0 = D.solve_start(f)
    D.iterate(args.warmup)
    amg.dist.barrier(ctx)
    D.profile(reset=True)
    tdist.barrier()
    torch.cuda.synchronize(local)
    t1 = time.perf_counter()
    D.iterate(args.steps)
    amg.dist.barrier(ctx)
    torch.cuda.synchronize(local)
    t2 = time.perf_counter()
    tdist.barrier()
    dt = torch.tensor([t2 - t1], dtype=torch.float64)
    tdist.all_reduce(dt, op=tdist.ReduceOp.MAX)
    dt = float(dt.item())
    rn = D.resnorm()
    ms, launches = D.profile(reset=True)
    res_ms = ms[0] / max(launches[0], 1)
    res_bytes = mat_bytes + 24 * D.n0
    kernels = None
    if slab:
        # the fine-level kernels of a step on this rank's slab (bench.fine_kernels,
        # DESIGN.md Sec.4 byte counts over the owned rows)
        from bench import fine_kernels
        fmask = (1 if fused0 else 0) | (2 if geo_mask & 1 else 0)
        kernels = fine_kernels(D.n0, mat_bytes, ms, launches, fmask, fmt)
    all_k = [None] * world
    tdist.all_gather_object(all_k, kernels)
    u_par = None
    if args.cpu_baseline:
        # parity leg (untimed): restart and run exactly the oracle's cpu_cycles
        # outer iterations; rank 0 gathers the slabs of the iterate
        r0p = D.solve_start(f)
        D.iterate(args.cpu_cycles)
        rel_p = D.resnorm() / r0p
        u_loc = torch.from_numpy(D.get_u())
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        tdist.all_gather(sizes, torch.tensor([u_loc.numel()], dtype=torch.int64))
        if rank == 0:
            parts = [torch.empty(int(sz.item()), dtype=torch.float64) for sz in sizes]
            tdist.gather(u_loc, parts, dst=0)
            u_par = (torch.cat(parts).numpy(), rel_p)
        else:
            tdist.gather(u_loc, None, dst=0)
    spmv_ms = D.fine_spmv_ms(args.spmv_reps)
    spmv_bytes = mat_bytes + 16 * D.n0
    # aggregate fine SpMV rate: all ranks' algorithmic bytes over the slowest rank's time
    agg = torch.tensor([float(spmv_bytes), spmv_ms, float(res_bytes), res_ms], dtype=torch.float64)
    parts = [torch.zeros_like(agg) for _ in range(world)]
    tdist.all_gather(parts, agg)
    P = torch.stack(parts).numpy()
    D.free()
    amg.dist.finalize(ctx)
    ctx.close()
    cpu, parity = None, None
    if rank == 0 and args.cpu_baseline:
        from bench import cpu_baseline, check_parity
        try:
            cpu, u_cpu, rel_cpu = cpu_baseline(gen, amg, amg.rhs_rand(0, n ** 3), args)
            parity = check_parity(u_par, u_cpu, rel_cpu, args.cpu_cycles)
            log(f"[cpu] {cpu['value']:.4f} it/s on {cpu['cores']} threads; [parity] {parity}")
        except Exception as e:
            log(f"[cpu] baseline failed: {e!r}")
    if rank == 0:
        value = args.steps / dt
        spmv_gbs = P[:, 0].sum() / (P[:, 1].max() * 1e-3) / 1e9
        res_gbs = P[:, 2].sum() / (P[:, 3].max() * 1e-3) / 1e9
        ach0 = res_bytes / (res_ms * 1e-3) / 1e9
        if kernels:
            dom = max(kernels, key=lambda k: kernels[k]["ms"])
            dk = kernels[dom]
            agg = sum(k[dom]["bytes"] for k in all_k) / (max(k[dom]["ms"] for k in all_k) * 1e-3) / 1e9
            roof = {"bound": "hbm", "kernel": f"{dom}: {dk['what']} (rank 0 slab, incl. ghost-plane exchange "
                                              "waits)",
                    "achieved": dk["gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": dk["frac"],
                    "traffic": None,
                    "traffic_note": "PMC FETCH/WRITE passes are single-GPU runs of bench.py (profiles/traffic.json)",
                    "alg_bytes_per_launch": dk["bytes"], "avg_launch_ms": dk["ms"], "aggregate_gbs": agg,
                    "selection": "the fine-level kernel with the largest time per step on rank 0"}
        else:
            roof = {"bound": "hbm", "kernel": f"fine-grid residual SpGEMV r = f - A0 u ({fmt}, rank 0 "
                                              "slab, incl. ghost exchange wait)",
                    "achieved": ach0, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": ach0 / HBM_PEAK_GBS, "traffic": None,
                    "traffic_note": "PMC FETCH/WRITE passes are single-GPU runs of bench.py "
                                    "(profiles/traffic.json); the per-rank slab residual is the "
                                    "same kernel on a z-slab and is not profiled per rank",
                    "alg_bytes_per_launch": res_bytes, "avg_launch_ms": res_ms,
                    "aggregate_gbs": res_gbs}
        log(f"[dist] {args.steps} steps in {dt * 1e3:.2f} ms -> {value:.2f} it/s; relres {rn / r0:.3e}; "
            f"fine SpMV aggregate {spmv_gbs:.0f} GB/s")
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
            "config": {"workload": f"{n}^3 7-pt Laplacian, SMEM_Solve MULT V(1,1) Jacobi "
                                   f"w={args.smooth_weight}, {gen.L}-level geometric Galerkin "
                                   f"hierarchy, z-slab partition, RCCL ghost exchange",
                       "n": n, "levels": gen.L, "parallelism": f"slab{world}", "matrix_format": fmt,
                       "dist_form": "z-slab extended operators (amg_dist_hier_create_slab)" if slab
                                    else "row-partitioned [owned | ghost] CSR (amg_dist_hier_create_structured)",
                       "distributed_levels": Ld if slab else None,
                       "geometric_transfer_levels": geo_mask if slab else None,
                       "fused_residual_restriction": bool(fused0) if slab else None,
                       "reuse_outer_residual": args.reuse_outer_residual},
            "fine_spmv": {"gbs_aggregate": spmv_gbs, "ms_max": float(P[:, 1].max()),
                          "frac_per_gpu": spmv_gbs / world / HBM_PEAK_GBS},
            "roofline": roof,
            "fine_kernels": kernels,
            # the CPU baseline is reported at N = 1 only (the oracle still runs at
            # N > 1 for the parity leg: the gathered iterate against it, bitwise)
            "cpu_baseline": cpu if world == 1 else None,
            "parity": parity,
            "final_relres": rn / r0,
        }
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    tdist.barrier()
    tdist.destroy_process_group()
