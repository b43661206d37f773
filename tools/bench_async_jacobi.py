"""DMEM_AsyncSmooth (DMEM_Smooth.cpp:16-313) at config 4's size: the 512^3 fine
operator as R row-partitioned ranks (threads of this process) on one GPU,
K relaxations, the ghost deltas over the device-resident channels.  Prints
one JSON line: relres, sweeps/s, and per rank the overlap record of
amg_dist_async_jacobi_stats (the fraction of each sweep's exchange window
covered by the interior product, the windows, on-time / late deltas, the
host's flow-control wait).  Run it with GPU_MAX_HW_QUEUES >= 4 R so that no
rank's compute and communication streams share a hardware queue.

usage: python tools/bench_async_jacobi.py [--n 512] [--ranks 2] [--sweeps 12]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--sweeps", type=int, default=12)
    ap.add_argument("--omega", type=float, default=0.8)
    a = ap.parse_args()
    from conftest import load_package
    from test_gpu_dist import run_ranks
    amg = load_package()
    n, R, K = a.n, a.ranks, a.sweeps
    gen = amg.Gen(n)
    f = amg.rhs_rand(0, n ** 3)
    opts = amg.default_opts(smooth_weight=a.omega)
    hub = amg.dist.ThreadMailbox(R, timeout=900.0)

    def rank(q):
        c = amg.Context(0, nstreams=2)
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
