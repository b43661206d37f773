"""Level-grouped asynchronous additive solve (DMEM_Add) with the ranks as
PROCESSES on one MI355X: payloads over gloo (D2H / H2D per correction) against
device-resident payloads (amg_grid_add_create_ipc: IPC-mapped slot pools,
gloo carries control words and acknowledgements only).

One grid per level, one process per grid.  Each process times its
amg_grid_add_solve after a gloo barrier; wall = the slowest rank's solve.
Reports grid cycles per second (all grids' cycles over the wall), messages and
the final relative residuals.  The hierarchy uses smoothed transfers built on
the host with the oracle's SpGEMM, as tools/bench_async.py does (setup, not
timed).

usage: python tools/bench_grid_ipc.py [--n 64] [--cycles 50] [--reps 3]
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _rank(rank, world, port, n, cycles, reps, ipc, q):
    try:
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from conftest import load_package
        from oracle import pyoracle as po
        from test_gpu_dist import split_host
        amg = load_package()
        g = amg.Gen(n, interp=amg.AMG_INTERP_LINEAR)
        L = g.L
        A = [po.Csr(*g.host_csr(amg.AMG_GEN_A, l)) for l in range(L)]
        P = [po.Csr(*g.host_csr(amg.AMG_GEN_P, l)) for l in range(L - 1)]
        Ps, Rs = [], []
        for l in range(L - 1):
            p, r = po.smooth_transfer(A[l], P[l], 0.8)
            Ps.append(p)
            Rs.append(r)
        f = amg.rhs_rand(0, n ** 3)
        rank_grid, rank_rows = amg.grid.layout((1,) * L, n ** 3)
        groups = {k: dist.new_group([r for r in range(world) if rank_grid[r] == k]) for k in range(L)}
        my = int(rank_grid[rank])
        rs, parts = split_host({"A": A, "P": Ps, "R": Rs}, ())
        opts = amg.default_opts(solver=amg.AMG_ASYNC_MULTADD, smooth_weight=0.8, tol=0.0, num_cycles=cycles,
                                max_inflight=2, converge_test_type=amg.AMG_LOCAL)
        c = amg.Context(0, nstreams=2)
        amg.dist.init_host(c, 1, 0, amg.dist.HostTransport(amg.dist.ThreadMailbox(1), 0))
        Ap, Pp, Rp = parts[0]
        D = amg.dist.DistHier.from_parts(c, rs, Ap, Pp, Rp, opts)
        T = amg.grid.TorchNbTransport(groups[my])
        G = amg.grid.GridAdd(T, my, world, rank, rank_grid, rank_rows, dist_hier=D, ipc=ipc)
        runs = []
        for rep in range(reps + 1):
            c.sync()
            dist.barrier()
            t0 = time.perf_counter()
            x, cyc, rel, msgs = G.solve(f)
            runs.append((time.perf_counter() - t0, cyc, rel, int(msgs[0])))
        G.free()
        dist.barrier()
        D.free()
        amg.dist.finalize(c)
        c.close()
        dist.destroy_process_group()
        q.put((rank, runs[1:]))  # rep 0 warms up
    except BaseException as ex:  # noqa: BLE001
        q.put((rank, repr(ex)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--cycles", type=int, default=50)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import multiprocessing as mp
    from conftest import load_package
    amg = load_package()
    L = amg.Gen(a.n, interp=amg.AMG_INTERP_LINEAR).L
    out = {"config": {"workload": f"{a.n}^3 7-pt Laplacian, level-grouped ASYNC_MULTADD (DMEM_Add), {L} grids "
                                  f"x 1 process on one GPU, {a.cycles} cycles per grid, LOCAL convergence, "
                                  "max_inflight 2, gloo control plane"}}
    for transport in ("host", "ipc"):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        ps = [ctx.Process(target=_rank, args=(r, L, port, a.n, a.cycles, a.reps, transport == "ipc", q), daemon=True)
              for r in range(L)]
        for p in ps:
            p.start()
        res = {}
        try:
            for _ in range(L):
                item = q.get(timeout=300)
                res[item[0]] = item[1]
        finally:
            for p in ps:
                p.join(30)
                if p.is_alive():
                    p.kill()
        bad = {r: v for r, v in res.items() if isinstance(v, str)}
        if bad:
            raise RuntimeError(f"{transport}: {bad}")
        reps = []
        for i in range(a.reps):
            wall = max(res[r][i][0] for r in res)
            reps.append({"wall_ms": 1e3 * wall, "grid_cycles_per_s": sum(res[r][i][1] for r in res) / wall,
                         "messages": sum(res[r][i][3] for r in res),
                         "rel": [res[r][i][2] for r in sorted(res)]})
        best = max(reps, key=lambda r: r["grid_cycles_per_s"])
        out[transport] = {"best": best, "grid_cycles_per_s": [r["grid_cycles_per_s"] for r in reps]}
        print(f"[grid-ipc] {transport}: {best['grid_cycles_per_s']:.0f} grid cycles/s", file=sys.stderr, flush=True)
    out["ipc_over_host"] = out["ipc"]["best"]["grid_cycles_per_s"] / out["host"]["best"]["grid_cycles_per_s"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
