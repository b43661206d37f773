"""DMEM_AsyncSmooth (DMEM_Smooth.cpp:16-313) at config 4's size: the 512^3 fine
operator as R row-partitioned ranks (threads of this process) on one GPU,
K relaxations, the ghost deltas over the device-resident channels.  Prints
one JSON line: relres, sweeps/s, and per rank the overlap record of
amg_dist_async_jacobi_stats (the fraction of each sweep's exchange window
covered by the interior product, the windows, on-time / late deltas, the
host's flow-control wait).  Run it with GPU_MAX_HW_QUEUES >= 4 R so that no
rank's compute and communication streams share a hardware queue.

usage: python tools/bench_async_jacobi.py [--n 512] [--ranks 2] [--sweeps 12]
       python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
           tools/bench_async_jacobi.py            (one PROCESS per rank: the production
           layout, each process with its own hardware queues; rank 0 prints the line)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main_procs(a):
    """one process per rank (torchrun, gloo for setup): the deltas over the
    cross-process channels (IPC-mapped slots, shared-memory sequence words)"""
    import torch.distributed as tdist
    from conftest import load_package
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    json_fd = os.dup(1)
    os.dup2(2, 1)  # stdout carries only the JSON line
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    amg = load_package()
    n, K = a.n, a.sweeps
    gen = amg.Gen(n)
    f = amg.rhs_rand(0, n ** 3)
    c = amg.Context(0, nstreams=2)
    tr = amg.dist.HostTransport(amg.dist.TorchGroupHub(), rank)
    amg.dist.init_host(c, world, rank, tr)
    amg.dist.set_replicate_rows(c, 1 << 18)
    D = amg.dist.DistHier(c, gen, amg.default_opts(smooth_weight=a.omega))
    fl = f[D.row0:D.row0 + D.n0]
    D.async_jacobi(fl, 2, 0)  # warm-up: channels, buffers
    c.sync()
    tdist.barrier()
    t0 = time.perf_counter()
    rel = D.async_jacobi(fl, K, 0)
    c.sync()
    dt = time.perf_counter() - t0
    st = D.async_jacobi_stats()
    D.free()
    amg.dist.finalize(c)
    c.close()
    gen.free()
    allr = [None] * world
    tdist.all_gather_object(allr, (rel, dt, st))
    tdist.destroy_process_group()
    if rank == 0:
        wall = max(t[1] for t in allr)
        hid = [t[2]["hidden_fraction"] for t in allr]
        out = {"workload": f"{n}^3 7-pt, DMEM_AsyncSmooth (asynchronous Jacobi, w={a.omega}), {world} "
                           f"row-partitioned ranks as PROCESSES on one GPU (each its own hardware queues), {K} "
                           "relaxations, deltas over the cross-process device-resident channels",
               "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "relres": allr[0][0],
               "sweeps_per_s": K / wall, "hidden_fraction_min": min(hid), "hidden_fraction_mean": sum(hid) / world,
               "ranks": [t[2] for t in allr]}
        os.write(json_fd, (json.dumps(out) + "\n").encode())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", "--grid", dest="n", type=int, default=512)
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--sweeps", type=int, default=12)
    ap.add_argument("--omega", type=float, default=0.8)
    a = ap.parse_args()
    if "WORLD_SIZE" in os.environ:
        return main_procs(a)
    from conftest import load_package
    from test_gpu_dist import run_ranks
    amg = load_package()
    n, R, K = a.n, a.ranks, a.sweeps
    gen = amg.Gen(n)
    f = amg.rhs_rand(0, n ** 3)
    opts = amg.default_opts(smooth_weight=a.omega)
    hub = amg.dist.ThreadMailbox(R, timeout=900.0)
    # contexts in rank order (bench.py async_jacobi_overlap: each rank's compute
    # and communication streams on different hardware queues)
    ctxs = [amg.Context(0, nstreams=2) for _ in range(R)]

    def rank(q):
        c = ctxs[q]
        amg.dist.init_host(c, R, q, amg.dist.HostTransport(hub, q))
        amg.dist.set_replicate_rows(c, 1 << 18)
        D = amg.dist.DistHier(c, gen, opts)
        fl = f[D.row0:D.row0 + D.n0]
        D.async_jacobi(fl, 2, 0)  # warm-up: channels, buffers
        c.sync()
        amg.dist.barrier(c)
        t0 = time.perf_counter()
        rel = D.async_jacobi(fl, K, 0)
        c.sync()
        dt = time.perf_counter() - t0
        st = D.async_jacobi_stats()
        D.free()
        amg.dist.finalize(c)
        c.close()
        return rel, dt, st

    res = run_ranks(R, rank)
    wall = max(t[1] for t in res)
    out = {"workload": f"{n}^3 7-pt, DMEM_AsyncSmooth (asynchronous Jacobi, w={a.omega}), {R} row-partitioned "
                       f"ranks (threads) on one GPU, {K} relaxations, deltas over the device-resident channels",
           "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "relres": res[0][0],
           "sweeps_per_s": K / wall, "ranks": [t[2] for t in res]}
    print(json.dumps(out))
    for q, t in enumerate(res):
        st = t[2]
        print(f"rank {q}: hidden {st['hidden_fraction']:.3f}, exchange {st['exchange_ms_per_sweep']:.3f} ms, interior "
              f"{st['interior_ms_per_sweep']:.3f} ms, on time {st['on_time_fraction']:.3f}, send wait "
              f"{st['send_wait_ms_per_sweep']:.3f} ms/sweep", file=sys.stderr)
    gen.free()


if __name__ == "__main__":
    main()
