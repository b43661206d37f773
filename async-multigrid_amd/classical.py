"""In-house classical AMG setup (amg_classical_*): the hierarchy the reference
gets from HYPRE_BoomerAMGSetup (SMEM_Setup.cpp:55-70, DMEM_Setup.cpp:169-173),
built on the host by the library -- strength of connection, HMIS / PMIS
coarsening, extended+i or direct interpolation, Galerkin R A P."""
import ctypes as C

import numpy as np

from . import abi
from .abi import (AMG_CLASSICAL_DIRECT, AMG_CLASSICAL_EXT_I, AMG_COARSEN_HMIS,  # noqa: F401
                  AMG_COARSEN_PMIS, AMG_COARSEN_PMIS_FIXED, AMG_GEN_A, AMG_GEN_P, AMG_GEN_R)


def elasticity(refine):
    """The DMEM elasticity problem (amg_elast_*): (n, rowptr, col, val, rhs) as
    numpy copies; num_functions = 3 (byVDIM)."""
    from . import check, lib
    h = C.c_void_p()
    check(lib.amg_elast_create(int(refine), C.byref(h)))
    try:
        n, nz = C.c_int(), C.c_longlong()
        rp, cj, v, b = abi._ip(), abi._ip(), abi._dp(), abi._dp()
        check(lib.amg_elast_get(h, C.byref(n), C.byref(nz), C.byref(rp), C.byref(cj), C.byref(v), C.byref(b)))
        N, Z = n.value, nz.value
        return (N, np.ctypeslib.as_array(rp, (N + 1,)).copy(), np.ctypeslib.as_array(cj, (Z,)).copy(),
                np.ctypeslib.as_array(v, (Z,)).copy(), np.ctypeslib.as_array(b, (N,)).copy())
    finally:
        lib.amg_elast_free(h)


def default_opts(**kw):
    """SMEM parameters (SMEM_Main.cpp:29-35): HMIS, ext+i, theta 0.25; DMEM uses
    coarsen_type=9, strong_threshold=0.5 (DMEM_Main.cpp:38-49)."""
    from . import lib
    o = abi.AmgClassicalOpts()
    lib.amg_classical_opts_default(C.byref(o))
    for k, v in kw.items():
        if not hasattr(o, k):
            raise AttributeError(k)
        setattr(o, k, v)
    return o


class ClassicalAMG:
    """Host hierarchy from a square CSR (diagonal first)."""

    def __init__(self, n, rowptr, col, val, opts=None, **kw):
        from . import check, lib
        self._lib = lib
        o = opts if opts is not None else default_opts(**kw)
        rp = np.ascontiguousarray(rowptr, dtype=np.int32)
        cj = np.ascontiguousarray(col, dtype=np.int32)
        v = np.ascontiguousarray(val, dtype=np.float64)
        h = C.c_void_p()
        check(lib.amg_classical_setup(C.byref(o), int(n), rp.ctypes.data_as(abi._ip),
                                      cj.ctypes.data_as(abi._ip), v.ctypes.data_as(abi._dp), C.byref(h)))
        self.h = h
        self.L = lib.amg_classical_levels(h)

    def get(self, which, level):
        """(nrows, ncols, rowptr, col, val) numpy copies of operator which (AMG_GEN_A/P/R)."""
        from . import check
        nr, nc, nz = C.c_int(), C.c_int(), C.c_longlong()
        rp, cj, v = abi._ip(), abi._ip(), abi._dp()
        check(self._lib.amg_classical_get(self.h, which, level, C.byref(nr), C.byref(nc), C.byref(nz),
                                          C.byref(rp), C.byref(cj), C.byref(v)))
        n, z = nr.value, nz.value
        return (n, nc.value, np.ctypeslib.as_array(rp, (n + 1,)).copy(),
                np.ctypeslib.as_array(cj, (max(z, 1),))[:z].copy() if z else np.zeros(0, np.int32),
                np.ctypeslib.as_array(v, (max(z, 1),))[:z].copy() if z else np.zeros(0))

    def cf_marker(self, level):
        from . import check
        n = self.get(AMG_GEN_A, level)[0]
        cf = np.zeros(n, dtype=np.int32)
        check(self._lib.amg_classical_cf_marker(self.h, level, cf.ctypes.data_as(abi._ip)))
        return cf

    def register(self, ctx, which, level):
        from . import Mat, check
        h = C.c_void_p()
        check(self._lib.amg_classical_register(ctx.h, self.h, which, level, C.byref(h)))
        return Mat(ctx, h)

    def hierarchy(self, ctx, opts, levels=None):
        """Register every level on the device and build a Hier (amg_hier_create)."""
        from . import Hier
        L = self.L if levels is None else levels
        As = [self.register(ctx, AMG_GEN_A, l) for l in range(L)]
        Ps = [self.register(ctx, AMG_GEN_P, l) for l in range(L - 1)]
        Rs = [self.register(ctx, AMG_GEN_R, l) for l in range(L - 1)]
        return Hier(ctx, As, Ps, Rs, opts)

    def free(self):
        if self.h:
            self._lib.amg_classical_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
