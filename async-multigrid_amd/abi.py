"""ctypes prototypes of every entry point declared in include/amg_mi355x.h.

The library is loaded from the package's lib/ directory (built in-tree by
__graft_entry__.build()).  There is no fallback: if the shared object is
missing, importing the package raises.
"""
import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libamg_mi355x.so")
# development build with the SpMV tuning harness (make -C csrc dev); only the
# tools/ tuning scripts select it, by setting AMG_DEV_LIB=1 before import
if os.environ.get("AMG_DEV_LIB") == "1":
    LIB_PATH = os.path.join(_HERE, "lib", "libamg_mi355x_dev.so")
# host-checked build (make -C csrc chk: bounds-checked containers, host debug
# info) for diagnosing host faults; selected by AMG_CHK_LIB=1
if os.environ.get("AMG_CHK_LIB") == "1":
    LIB_PATH = os.path.join(_HERE, "lib", "libamg_mi355x_chk.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "amg_mi355x.h")

_p = C.c_void_p
_i = C.c_int
_ll = C.c_longlong
_d = C.c_double
_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)
_llp = C.POINTER(C.c_longlong)
_pp = C.POINTER(C.c_void_p)

AMG_OK = 0
AMG_JACOBI, AMG_GAUSS_SEIDEL, AMG_HYBRID_JGS, AMG_SYMM_JACOBI = 0, 1, 2, 3
AMG_SEMI_ASYNC_GS, AMG_ASYNC_GS = 4, 5
AMG_L1_JACOBI, AMG_L1_HYBRID_JGS = 6, 12
AMG_MULT, AMG_AFACX, AMG_MULTADD, AMG_ASYNC_AFACX, AMG_ASYNC_MULTADD = 0, 1, 2, 5, 6
AMG_BPX = 3
AMG_FULL_ASYNC, AMG_SEMI_ASYNC = 0, 1
AMG_LOCAL, AMG_GLOBAL = 0, 1
AMG_READ_SOL, AMG_READ_RES = 0, 1
AMG_NO_ACCEL, AMG_RICHARD_ACCEL, AMG_CHEBY_RECUR_ACCEL = 0, 1, 2
AMG_VEC_F, AMG_VEC_U, AMG_VEC_R = 0, 1, 2
AMG_INTERP_LINEAR, AMG_INTERP_AGGREGATE = 0, 1
AMG_GEN_A, AMG_GEN_P, AMG_GEN_R = 0, 1, 2


class AmgOpts(C.Structure):
    _fields_ = [("solver", _i), ("smoother", _i),
                ("num_pre_smooth_sweeps", _i), ("num_post_smooth_sweeps", _i),
                ("num_fine_smooth_sweeps", _i), ("num_coarse_smooth_sweeps", _i),
                ("smooth_weight", _d), ("num_cycles", _i), ("tol", _d),
                ("check_resnorm", _i), ("cheby_flag", _i), ("cheby_mu", _d),
                ("cheby_delta", _d), ("num_threads", _i), ("jgs_block_rows", _i),
                ("reuse_outer_residual", _i), ("async_type", _i), ("profile", _i),
                ("accel_type", _i), ("cheby_grid", _i), ("res_compute_type", _i),
                ("read_type", _i), ("converge_test_type", _i),
                ("delay_type", _i), ("delay_usec", _i), ("delay_frac", _d), ("fail_iter", _i),
                ("delay_rank", _i), ("max_inflight", _i), ("async_comm_save_divisor", _i),
                ("sps_probability_type", _i), ("sps_alpha", _d), ("sps_min_prob", _d),
                ("delay_level", _i), ("async_schedule", _i),
                ("smooth_transfer", _i)]


AMG_SCHED_FREE, AMG_SCHED_FINEST_FIRST, AMG_SCHED_COARSEST_FIRST, AMG_SCHED_ROUND_ROBIN, AMG_SCHED_TIMED = 0, 1, 2, 3, 4
AMG_DELAY_NONE, AMG_DELAY_ONE, AMG_DELAY_SOME, AMG_DELAY_ALL, AMG_FAIL_ONE = 0, 1, 2, 3, 4
AMG_SPS_EXPONENTIAL, AMG_SPS_INVERSE, AMG_SPS_RANDOM = 0, 1, 2


class AmgClassicalOpts(C.Structure):
    _fields_ = [("coarsen_type", _i), ("interp_type", _i), ("strong_threshold", _d),
                ("max_row_sum", _d), ("max_levels", _i), ("max_coarse_size", _i),
                ("num_functions", _i), ("seed", C.c_ulonglong), ("device", _i)]


AMG_COARSEN_PMIS, AMG_COARSEN_PMIS_FIXED, AMG_COARSEN_HMIS = 8, 9, 10
AMG_CLASSICAL_DIRECT, AMG_CLASSICAL_EXT_I = 3, 6

# name -> (restype, argtypes)
PROTOTYPES = {
    "amg_opts_default": (None, [C.POINTER(AmgOpts)]),
    "amg_init": (_i, [_pp, _i, _i]),
    "amg_finalize": (_i, [_p]),
    "amg_sync": (_i, [_p]),
    "amg_device_errors": (_i, [_p, _ip]),
    "amg_last_error": (C.c_char_p, []),
    "amg_version": (_i, []),
    "amg_csr_register": (_i, [_p, _i, _i, _ll, _ip, _ip, _dp, _i, _pp]),
    "amg_mat_free": (_i, [_p]),
    "amg_set_value_index": (_i, [_p, _i]),
    "amg_mat_value_index": (_i, [_p]),
    "amg_set_dict_index": (_i, [_p, _i]),
    "amg_mat_dict_index": (_i, [_p]),
    "amg_set_row_pattern": (_i, [_p, _i]),
    "amg_mat_row_pattern": (_i, [_p]),
    "amg_set_pair_pattern": (_i, [_p, _i]),
    "amg_mat_pair_pattern": (_i, [_p]),
    "amg_set_pair_anchor16": (_i, [_p, _i]),
    "amg_mat_pair_anchor16": (_i, [_p]),
    "amg_set_master_pattern": (_i, [_p, _i]),
    "amg_mat_master_pattern": (_i, [_p]),
    "amg_set_plane_march": (_i, [_p, _i, _i, _i]),
    "amg_mat_plane_march": (_i, [_p]),
    "amg_mat_march_points": (_i, [_p]),
    "amg_set_bsr3": (_i, [_p, _i]),
    "amg_mat_bsr3": (_i, [_p]),
    "amg_mat_bsr3_slice": (_i, [_p]),
    "amg_mat_info": (_i, [_p, _ip, _ip, _llp]),
    "amg_mat_download": (_i, [_p, _p, _ip, _ip, _dp]),
    "amg_vec_create": (_i, [_p, _i, _pp]),
    "amg_vec_free": (_i, [_p]),
    "amg_vec_size": (_i, [_p]),
    "amg_vec_upload": (_i, [_p, _p, _dp]),
    "amg_vec_download": (_i, [_p, _p, _dp]),
    "amg_vec_set": (_i, [_p, _p, _d]),
    "amg_vec_copy": (_i, [_p, _p, _p]),
    "amg_vec_axpy": (_i, [_p, _d, _p, _p]),
    "amg_vec_ivaxpy": (_i, [_p, _p, _p, _p]),
    "amg_vec_scale": (_i, [_p, _d, _p]),
    "amg_vec_norm2": (_i, [_p, _p, _dp]),
    "amg_vec_dot": (_i, [_p, _p, _p, _dp]),
    "amg_matvec": (_i, [_p, _p, _p, _p, _i, _i]),
    "amg_matvec_t": (_i, [_p, _p, _p, _p, _i]),
    "amg_spgemv": (_i, [_p, _p, _p, _p, _d, _d, _p, _i, _i]),
    "amg_matvec_timed": (_i, [_p, _p, _p, _p, _i, _dp]),
    "amg_stream_triad": (_i, [_p, _ll, _i, _dp]),
    "amg_pmc_calib": (_i, [_p, _i, _ll]),
    "amg_residual": (_i, [_p, _p, _p, _p, _p, _p, _i, _i]),
    "amg_jacobi": (_i, [_p, _p, _p, _p, _p, _d, _i, _i, _i, _i, _i]),
    "amg_l1_jacobi": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i]),
    "amg_hybrid_jgs": (_i, [_p, _p, _p, _p, _p, _ip, _i, _p, _d, _i, _i, _i]),
    "amg_gauss_seidel": (_i, [_p, _p, _p, _p, _i]),
    "amg_async_gauss_seidel": (_i, [_p, _p, _p, _p, _ip, _i, _i, _i, _i]),
    "amg_sym_jacobi": (_i, [_p, _p, _p, _p, _p, _p, _d, _p, _i, _i, _i, _i, _i]),
    "amg_l1_norms": (_i, [_p, _p, _p]),
    "amg_a_diag": (_i, [_p, _p, _d, _p]),
    "amg_hier_create": (_i, [_p, _i, _pp, _pp, _pp, C.POINTER(AmgOpts), _pp]),
    "amg_hier_free": (_i, [_p]),
    "amg_hier_fused": (_i, [_p]),
    "amg_set_fuse_transfer": (_i, [_p, _i]),
    "amg_hier_fused_prolong": (_i, [_p]),
    "amg_set_fuse_prolong": (_i, [_p, _i]),
    "amg_set_jgs_wave": (_i, [_p, _i]),
    "amg_set_jgs_small": (_i, [_p, _i]),
    "amg_set_jgs_fold": (_i, [_p, _i]),
    "amg_set_march_lines": (_i, [_p, _i]),
    "amg_set_march_lines_gemv": (_i, [_p, _i]),
    "amg_set_march_tuning": (_i, [_p, _i, _i, _i, _i]),
    "amg_set_fuse_outer": (_i, [_p, _i]),
    "amg_set_outer_slab": (_i, [_p, _i]),
    "amg_set_long_form": (_i, [_p, _i, _i]),
    "amg_hier_fused_outer": (_i, [_p]),
    "amg_set_graphs": (_i, [_p, _i]),
    "amg_hier_set_opts": (_i, [_p, C.POINTER(AmgOpts)]),
    "amg_hier_set_blocks": (_i, [_p, _i, _ip, _i]),
    "amg_hier_vec": (_i, [_p, _i, _i, _pp]),
    "amg_solve": (_i, [_p, _p, _p, _dp, _ip]),
    "amg_solve_start": (_i, [_p, _p, _p, _dp]),
    "amg_solve_iterate": (_i, [_p, _i]),
    "amg_solve_resnorm": (_i, [_p, _dp]),
    "amg_solve_get_u": (_i, [_p, _p]),
    "amg_vcycle": (_i, [_p]),
    "amg_async_solve": (_i, [_p, _p, _p, _ip, _dp]),
    "amg_async_level_ms": (_i, [_p, _dp]),
    "amg_hier_set_async_durations": (_i, [_p, _dp, _i]),
    "amg_hier_set_async_times": (_i, [_p, _dp, _ip, _i]),
    "amg_async_correction_ms": (_i, [_p, _i, _dp, _i, _ip]),
    "amg_async_update_windows": (_i, [_p, _i, _dp, _i, _ip]),
    "amg_async_update_rows": (_i, [_p, _i, _i, _dp, _i, _ip]),
    "amg_eigs_power": (_i, [_p, _i, _dp, _dp]),
    "amg_hier_profile_read": (_i, [_p, _dp, _llp, _i]),
    "amg_gen_create": (_i, [_i, _i, _i, _i, _i, _i, _pp]),
    "amg_gen_free": (_i, [_p]),
    "amg_gen_num_levels": (_i, [_p]),
    "amg_gen_dims": (_i, [_p, _i, _ip, _ip, _ip]),
    "amg_gen_nnz": (_ll, [_p, _i, _i, _i, _i]),
    "amg_gen_fill": (_i, [_p, _i, _i, _i, _i, _ip, _ip, _dp, _i]),
    "amg_gen_register": (_i, [_p, _p, _i, _i, _i, _i, _pp]),
    "amg_rhs_rand": (_i, [_ll, _ll, _d, _d, _dp]),
    "amg_classical_opts_default": (None, [C.POINTER(AmgClassicalOpts)]),
    "amg_classical_setup": (_i, [C.POINTER(AmgClassicalOpts), _i, _ip, _ip, _dp, _pp]),
    "amg_classical_levels": (_i, [_p]),
    "amg_classical_get": (_i, [_p, _i, _i, _ip, _ip, _llp, C.POINTER(_ip), C.POINTER(_ip),
                               C.POINTER(_dp)]),
    "amg_classical_register": (_i, [_p, _p, _i, _i, _pp]),
    "amg_classical_cf_marker": (_i, [_p, _i, _ip]),
    "amg_classical_free": (_i, [_p]),
    "amg_elast_create": (_i, [_i, _pp]),
    "amg_elast_get": (_i, [_p, _ip, _llp, C.POINTER(_ip), C.POINTER(_ip), C.POINTER(_dp), C.POINTER(_dp)]),
    "amg_elast_free": (_i, [_p]),
    # distributed (RCCL) interface
    "amg_dist_unique_id_size": (_i, []),
    "amg_dist_get_unique_id": (_i, [C.c_char_p]),
    "amg_dist_init": (_i, [_p, _i, _i, C.c_char_p]),
    "amg_dist_finalize": (_i, [_p]),
    "amg_dist_allreduce_sum": (_i, [_p, _dp, _i]),
    "amg_dist_barrier": (_i, [_p]),
    "amg_dist_hier_create_structured": (_i, [_p, _p, C.POINTER(AmgOpts), _pp]),
    "amg_dist_hier_create_slab": (_i, [_p, _p, C.POINTER(AmgOpts), _pp]),
    "amg_dist_hier_slab_info": (_i, [_p, _ip, _ip, _ip]),
    "amg_dist_hier_local_rows": (_i, [_p, _i, _ip, _ip]),
    "amg_dist_hier_matrix_info": (_i, [_p, _i, _llp, _ip, _ip, _ip]),
    "amg_dist_hier_pair_pattern": (_i, [_p, _i, _ip]),
    "amg_dist_solve_start": (_i, [_p, _dp, _dp]),
    "amg_dist_solve_iterate": (_i, [_p, _i]),
    "amg_dist_solve_resnorm": (_i, [_p, _dp]),
    "amg_dist_get_u": (_i, [_p, _dp]),
    "amg_dist_hier_free": (_i, [_p]),
    "amg_dist_profile_read": (_i, [_p, _dp, _llp, _i]),
    "amg_dist_fine_spmv": (_i, [_p, _i, _dp]),
    "amg_dist_init_host": (_i, [_p, _i, _i, C.c_void_p, _p]),
    "amg_dist_hier_set_replicate_rows": (_i, [_p, _ll]),
    "amg_dist_async_solve": (_i, [_p, _dp, _ip, _dp]),
    "amg_dist_async_level_ms": (_i, [_p, _dp]),
    "amg_dist_hier_set_async_durations": (_i, [_p, _dp, _i]),
    "amg_dist_hier_set_async_times": (_i, [_p, _dp, _ip, _i]),
    "amg_dist_async_correction_ms": (_i, [_p, _i, _dp, _i, _ip]),
    "amg_dist_async_update_windows": (_i, [_p, _i, _dp, _i, _ip]),
    "amg_dist_async_update_rows": (_i, [_p, _i, _i, _dp, _i, _ip]),
    "amg_dist_async_jacobi": (_i, [_p, _dp, _i, _i, _dp]),
    "amg_dist_async_jacobi_stats": (_i, [_p, _dp, _i]),
    "amg_dist_async_jacobi_log": (_i, [_p, _dp, _i, _ip]),
    "amg_dist_async_sps": (_i, [_p, _dp, _i, _dp, C.POINTER(C.c_longlong)]),
    "amg_rand_double_stream": (_i, [C.c_uint, _i, _d, _d, _dp]),
    "amg_dist_structured_row_starts": (_i, [_p, _i, _llp]),
    "amg_dist_hier_create": (_i, [_p, _i, _llp, C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.POINTER(AmgOpts), _pp]),
}


class AmgCsrPart(C.Structure):
    _fields_ = [("nrows", _i), ("nnz", _ll), ("rowptr", _ip), ("col", _ip), ("val", _dp)]


class AmgHostCsr(C.Structure):
    _fields_ = [("nrows", _i), ("ncols", _i), ("nnz", _ll), ("rowptr", _ip), ("col", _ip), ("val", _dp)]


_ISEND = C.CFUNCTYPE(_i, _p, _i, _i, _dp, _ll, _llp)
_IRECV = _ISEND
_TEST = C.CFUNCTYPE(_i, _p, _ll, _ip)
_WAIT = C.CFUNCTYPE(_i, _p, _ll)
_ALLRED = C.CFUNCTYPE(_i, _p, _dp, _i)


class AmgNbTransport(C.Structure):
    _fields_ = [("user", _p), ("isend", _ISEND), ("irecv", _IRECV), ("test", _TEST), ("wait", _WAIT),
                ("grid_allreduce", _ALLRED)]


PROTOTYPES.update({
    "amg_grid_partition": (_i, [_i, _i, _dp, _ip]),
    "amg_grid_add_create": (_i, [_p, _i, _i, _i, _ip, _llp, C.POINTER(AmgNbTransport), _pp]),
    "amg_devhub_create": (_i, [_i, _ip, _pp]),
    "amg_devhub_free": (_i, [_p]),
    "amg_grid_add_create_devhub": (_i, [_p, _i, _i, _i, _ip, _llp, _p, _pp]),
    "amg_grid_add_create_ipc": (_i, [_p, _i, _i, _i, _ip, _llp, C.POINTER(AmgNbTransport), _pp]),
    "amg_grid_add_create_host": (_i, [_i, _dp, _d, C.POINTER(AmgOpts), _i, _i, _i, _ip, _llp,
                                      C.POINTER(AmgNbTransport), _pp]),
    "amg_grid_add_solve": (_i, [_p, _dp, _dp, _ip, _dp, _llp]),
    "amg_grid_add_peers": (_i, [_p, _ip, _ip]),
    "amg_grid_add_free": (_i, [_p]),
    "amg_triplet_read": (_i, [C.c_char_p, _i, _i, C.POINTER(AmgHostCsr)]),
    "amg_triplet_read_part": (_i, [C.c_char_p, _i, _ip, C.POINTER(AmgHostCsr)]),
    "amg_triplet_write": (_i, [C.c_char_p, _i, _i, _ip, _ip, _dp, _i]),
    "amg_triplet_text_to_bin": (_i, [C.c_char_p, C.c_char_p]),
    "amg_host_csr_free": (None, [C.POINTER(AmgHostCsr)]),
})


# amg_host_xchg_fn: (user, op, npeers, peers, send, send_bytes, recv, recv_bytes) -> int
HOST_XCHG_FN = C.CFUNCTYPE(_i, _p, _i, _i, _ip, _pp, _llp, _pp, _llp)


def header_symbols(path=HEADER):
    """Names of every function the public header declares."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(amg_[a-z_0-9]+)\s*\(", txt, flags=re.M)
    return sorted(set(names))


class AmgError(RuntimeError):
    pass


def load(path=LIB_PATH):
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build the HIP library first (python -c 'import __graft_entry__ as g; g.build()')")
    lib = C.CDLL(path)
    for name, (res, args) in PROTOTYPES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    return lib
