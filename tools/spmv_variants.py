"""Fine-grid SpMV y = A0 x (512^3 7-pt, the default storage) timed with HIP
events under the march knobs given in the environment; prints ms and GB/s on
the algorithmic bytes (n/2 + 16n)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_package  # noqa: E402

amg = load_package()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
ctx = amg.Context(0, 2)
g = amg.Gen(n)
A = g.register(ctx, amg.AMG_GEN_A, 0)
x = ctx.vec(np.random.default_rng(0).uniform(-1, 1, A.ncols))
y = ctx.vec(A.nrows)
ms = C.c_double()
amg.check(amg.lib.amg_matvec_timed(ctx.h, A.h, x.h, y.h, 5, C.byref(ms)))
amg.check(amg.lib.amg_matvec_timed(ctx.h, A.h, x.h, y.h, 40, C.byref(ms)))
rows = n ** 3
b = (rows + 1) // 2 + 16 * rows
env = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("AMG_"))
print(f"{env or 'default'}: {ms.value:.4f} ms  {b / ms.value / 1e6:.0f} GB/s  frac {b / ms.value / 1e6 / 8000:.3f}",
      flush=True)
