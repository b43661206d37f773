"""Interleaved A/B timing of CSR tile-kernel configurations on the 512^3
fine operator (y = A0 x); also checks every variant returns identical bits."""
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
n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
prefixes = tuple(sys.argv[3].encode().split(b",")) if len(sys.argv) > 3 else None  # e.g. dc,rp
ctx = amg.Context(0, 2)
if n < 0:  # elasticity r = -n: the classical hierarchy's operators (long coarse rows)
    ne, rp, cj, v, b = amg.classical.elasticity(-n)
    H = amg.classical.ClassicalAMG(ne, rp, cj, v, coarsen_type=9, strong_threshold=0.5, num_functions=3)
    mats = {f"E{l}": H.register(ctx, amg.AMG_GEN_A, l) for l in range(min(H.L, 5))}
else:
    g = amg.Gen(n)
    mats = {"A0": g.register(ctx, amg.AMG_GEN_A, 0), "A1": g.register(ctx, amg.AMG_GEN_A, 1),
            "R0": g.register(ctx, amg.AMG_GEN_R, 0), "P0": g.register(ctx, amg.AMG_GEN_P, 0)}
nv = lib.amg_dev_tune_count()
for name, A in mats.items():
    x = ctx.vec(np.random.default_rng(0).uniform(-1, 1, A.ncols))
    y = ctx.vec(A.nrows)
    ref = None
    res = {v: [] for v in range(nv)}
    vlist = [v for v in range(nv) if name == "A0" or not lib.amg_dev_tune_name(v).startswith(b"ABL")]
    if prefixes:
        vlist = [v for v in vlist if lib.amg_dev_tune_name(v).startswith(prefixes)]
    for r in range(rounds):
        for v in vlist:
            ms = C.c_double()
            amg.check(lib.amg_dev_tune_spmv(ctx.h, A.h, x.h, y.h, v, 10, C.byref(ms)))
            res[v].append(ms.value)
            out = y.download()
            if lib.amg_dev_tune_name(v).startswith(b"ABL"):
                continue
            if ref is None:
                ref = out
            elif not np.array_equal(out.view(np.uint64), ref.view(np.uint64)):
                print(f"{name} variant {v}: RESULT MISMATCH")
    for v in vlist:
        nm = lib.amg_dev_tune_name(v)
        bpe = 1 if nm.startswith(b"dc") and A.dict_index else 5 if nm.startswith(b"vi") and A.value_index else 12
        nbytes = bpe * A.nnz + 4 * (A.nrows + 1) + 8 * A.ncols + 8 * A.nrows
        if nm.startswith(b"rp") and A.row_pattern:
            nbytes = A.nrows + 8 * A.ncols + 8 * A.nrows
        t = np.median(res[v])
        print(f"{name:3s} {lib.amg_dev_tune_name(v).decode():22s} median {t:.3f} ms  min {min(res[v]):.3f}"
              f"  {nbytes / t / 1e6:.0f} GB/s")
    x.free(); y.free()
