"""Binary triplet matrix files (-problem file) through the C-ABI
(amg_triplet_*, csrc/amg_io.cpp): ReadBinary_fread_HypreParCSR (Misc.cpp:800-915),
ParReadBinary_fread (DMEM_BuildMatrix.cpp:1488-1560), PrintCSRMatrix
(Misc.cpp:753-797) and TextToBin (TextToBin.cpp:5-39)."""
import ctypes as C

import numpy as np

from .abi import AmgHostCsr
from . import lib, check

RECORD = np.dtype([("i", "<i4"), ("j", "<i4"), ("val", "<f8")])  # Triplet_AOS


def _take(h):
    n, nnz = h.nrows, h.nnz
    rowptr = np.ctypeslib.as_array(h.rowptr, (n + 1,)).copy() if n >= 0 and h.rowptr else np.zeros(1, np.int32)
    col = np.ctypeslib.as_array(h.col, (nnz,)).copy() if nnz else np.zeros(0, np.int32)
    val = np.ctypeslib.as_array(h.val, (nnz,)).copy() if nnz else np.zeros(0, np.float64)
    out = (h.nrows, h.ncols, rowptr, col, val)
    lib.amg_host_csr_free(C.byref(h))
    return out


def read(path, symm=1, remove_disconnected=0):
    """(nrows, ncols, rowptr, col, val) of a binary triplet file, rows diagonal-first."""
    h = AmgHostCsr()
    check(lib.amg_triplet_read(str(path).encode(), int(symm), int(remove_disconnected), C.byref(h)))
    return _take(h)


def read_part(path, ncols):
    """(first_row, (nrows, ncols, rowptr, col, val)) of one rank's row file."""
    h = AmgHostCsr()
    first = C.c_int()
    check(lib.amg_triplet_read_part(str(path).encode(), int(ncols), C.byref(first), C.byref(h)))
    return first.value, _take(h)


def write(path, nrows, ncols, rowptr, col, val, binary=1):
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int32)
    col = np.ascontiguousarray(col, dtype=np.int32)
    val = np.ascontiguousarray(val, dtype=np.float64)
    ip = C.POINTER(C.c_int)
    check(lib.amg_triplet_write(str(path).encode(), int(nrows), int(ncols), rowptr.ctypes.data_as(ip),
                                col.ctypes.data_as(ip), val.ctypes.data_as(C.POINTER(C.c_double)), int(binary)))


def text_to_bin(in_path, out_path):
    check(lib.amg_triplet_text_to_bin(str(in_path).encode(), str(out_path).encode()))
