"""Slab hierarchy vs one GPU under env switches (development check)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def one(dims, nranks, rep, cycles=3):
    import numpy as np
    from conftest import load_package
    from test_gpu_dist import single_gpu
    from test_gpu_slab import slab_ranks
    amg = load_package()
    ctx = amg.Context(0, nstreams=4)
    gen = amg.Gen(*dims)
    opts = amg.default_opts(num_cycles=cycles, tol=0.0, smooth_weight=0.8)
    f = amg.rhs_rand(0, dims[0] * dims[1] * dims[2])
    u1, h1 = single_gpu(amg, ctx, gen, opts, f, cycles)
    info = []
    ud, hd = slab_ranks(amg, gen, opts, f, cycles, nranks, rep, info=info)
    bad = np.nonzero(u1.view(np.uint64) != ud.view(np.uint64))[0]
    print(f"dims={dims} ranks={nranks} rep={rep} info={info} mismatches={bad.size} "
          f"first={bad[:3]} maxdiff={np.max(np.abs(u1 - ud)):.3e} h1={h1[-1]:.4e} hd={hd[-1]:.4e}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        d = tuple(int(x) for x in sys.argv[1].split(","))
        one(d, int(sys.argv[2]), int(sys.argv[3]))
        sys.exit(0)
    runs = [({}, "64,64,64", 3, 1 << 12), ({"AMG_SLAB_NO_OVERLAP": "1"}, "64,64,64", 2, 1 << 18),
            ({"AMG_SLAB_NO_OVERLAP": "2"}, "64,64,64", 2, 1 << 18),
            ({"AMG_PLANE_MARCH_XCD": "0"}, "64,64,64", 2, 1 << 18),
            ({"AMG_SLAB_NO_OVERLAP": "2", "AMG_PLANE_MARCH": "4"}, "64,64,64", 2, 1 << 18), ({}, "64,64,64", 2, 1 << 18)]
    for env, d, nr, rep in runs:
        e = dict(os.environ)
        e.update(env)
        print("env", env, flush=True)
        r = subprocess.run([sys.executable, __file__, d, str(nr), str(rep)], env=e, timeout=300)
        if r.returncode != 0:
            print("rc", r.returncode, flush=True)
            if r.returncode < 0 or r.returncode > 1:
                break
