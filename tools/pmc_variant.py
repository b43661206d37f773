"""Run tuning variants (names given on the command line) on the 512^3 A0, a few
launches each, for rocprofv3 --pmc passes (FETCH_SIZE per variant, told apart
by dispatch order: each variant's launches are contiguous)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["AMG_DEV_LIB"] = "1"  # tuning variants live in the development build
from conftest import load_package  # noqa: E402

amg = load_package()
lib = amg.lib
lib.amg_dev_tune_name.restype = C.c_char_p
lib.amg_dev_tune_spmv.argtypes = [C.c_void_p] * 4 + [C.c_int, C.c_int, C.POINTER(C.c_double)]
names = sys.argv[1].split(",")
ctx = amg.Context(0, 2)
g = amg.Gen(512)
A = g.register(ctx, amg.AMG_GEN_A, 0)
x = ctx.vec(np.random.default_rng(0).uniform(-1, 1, A.ncols))
y = ctx.vec(A.nrows)
byname = {lib.amg_dev_tune_name(v).decode(): v for v in range(lib.amg_dev_tune_count())}
for nm in names:
    ms = C.c_double()
    amg.check(lib.amg_dev_tune_spmv(ctx.h, A.h, x.h, y.h, byname[nm], 4, C.byref(ms)))
    print(nm, ms.value, flush=True)
