"""Workload for the sweep over-fetch study (tools/gpu_overfetch.sh): a 2 GiB
read calibration stream (gfx950 FETCH_SIZE counts half the bytes read), then
three 512^3 V-cycles in the default storage; the march knobs come from the
environment (AMG_MZ_LINES, AMG_PLANE_MARCH, AMG_PLANE_MARCH_XCD, AMG_MZ_NT)."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_package  # noqa: E402

amg = load_package()
lib = amg.lib
n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
ctx = amg.Context(0, 4)
amg.check(lib.amg_pmc_calib(ctx.h, 0, 2 << 30))
g = amg.Gen(n)
H = amg.build_hierarchy(ctx, g, amg.default_opts(smooth_weight=0.8, num_cycles=1 << 30, tol=0.0,
                                                  reuse_outer_residual=2))
f = ctx.vec(amg.rhs_rand(0, n ** 3))
H.solve_start(f, ctx.vec(n ** 3))
H.iterate(3)
ctx.sync()
H.free()
print("ok", flush=True)
