"""CPU: the C-ABI library loads and exports every symbol include/*.h declares."""
import ctypes as C
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_header(amg):
    names = amg.abi.header_symbols()
    assert len(names) > 40
    missing = [n for n in names if not hasattr(amg.lib, n)]
    assert not missing, missing


def test_prototypes_cover_header(amg):
    names = set(amg.abi.header_symbols())
    proto = set(amg.abi.PROTOTYPES)
    assert names <= proto, sorted(names - proto)


def test_opts_defaults_match_reference(amg):
    # SMEM_Main.cpp:65-105
    o = amg.default_opts()
    assert (o.solver, o.smoother) == (amg.AMG_MULT, amg.AMG_JACOBI)
    assert (o.num_pre_smooth_sweeps, o.num_post_smooth_sweeps) == (1, 1)
    assert o.smooth_weight == 1.0 and o.tol == 1e-9 and o.check_resnorm == 1
    assert o.num_cycles == 20 and o.cheby_flag == 0


def test_version_and_error_string(amg):
    assert amg.lib.amg_version() >= 1
    assert isinstance(amg.lib.amg_last_error(), bytes)
    # a bad argument is reported, not aborted (no device needed: generator path)
    h = C.c_void_p()
    st = amg.lib.amg_gen_create(0, 4, 4, 0, 5, 9, C.byref(h))
    assert st < 0 and b"bad dimensions" in amg.lib.amg_last_error()
