"""ctypes bindings to the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module. It loads:

* ``oracle/build/libhpccg_oracle.so`` -- the C restatement (hpccg_oracle.c),
  each function citing the reference file:line it follows;
* ``oracle/_ref/libhpccg_ref.so`` (optional) -- the reference's own sources
  compiled here by ``oracle/Makefile`` plus our extern "C" shim (ref_shim.cpp).

Arrays are numpy; CSR uses int64 row pointers, int32 columns, float64 values.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "build", "libhpccg_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libhpccg_ref.so")
REF_OMP_SO = os.path.join(HERE, "_ref", "libhpccg_ref_omp.so")

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_lp = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")

_lib = None


def build() -> None:
    """Compile the C restatement (and the reference build when REF exists)."""
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)
    if os.path.isdir("/root/reference"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True,
                       stderr=subprocess.DEVNULL)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)
        L = C.CDLL(ORACLE_SO)
        L.oracle_count_nnz.restype = C.c_longlong
        L.oracle_count_nnz.argtypes = [C.c_int] * 6
        L.oracle_generate.restype = C.c_int
        L.oracle_generate.argtypes = [C.c_int] * 6 + [_lp, _ip, _dp, _dp, _dp, _dp]
        L.oracle_sparsemv.restype = None
        L.oracle_sparsemv.argtypes = [C.c_int, _lp, _ip, _dp, _dp, _dp, C.c_int]
        L.oracle_ddot.restype = C.c_double
        L.oracle_ddot.argtypes = [C.c_int, _dp, _dp, C.c_int]
        L.oracle_waxpby.restype = None
        L.oracle_waxpby.argtypes = [C.c_int, C.c_double, _dp, C.c_double, _dp, _dp, C.c_int]
        L.oracle_hpccg.restype = C.c_int
        L.oracle_hpccg.argtypes = [C.c_int, _lp, _ip, _dp, _dp, _dp, C.c_int, C.c_double,
                                   C.POINTER(C.c_int), C.POINTER(C.c_double), _dp, C.c_void_p,
                                   C.c_int]
        L.oracle_compute_residual.restype = C.c_double
        L.oracle_compute_residual.argtypes = [C.c_int, _dp, _dp]
        L.oracle_max_threads.restype = C.c_int
        _lib = L
    return _lib


class CSR:
    """A generated problem: CSR matrix plus x0, b, xexact."""

    def __init__(self, row_ptr, cols, vals, x, b, xexact, start_row=0, total_nrow=None):
        self.row_ptr, self.cols, self.vals = row_ptr, cols, vals
        self.x, self.b, self.xexact = x, b, xexact
        self.nrow = len(row_ptr) - 1
        self.start_row = start_row
        self.total_nrow = self.nrow if total_nrow is None else total_nrow

    @property
    def nnz(self) -> int:
        return int(self.row_ptr[-1])


def generate(nx: int, ny: int, nz: int, rank: int = 0, size: int = 1,
             use_7pt: bool = False) -> CSR:
    """generate_matrix.cpp:196-307 restated (global column indices)."""
    L = lib()
    n = nx * ny * nz
    nnz = L.oracle_count_nnz(nx, ny, nz, rank, size, int(use_7pt))
    row_ptr = np.zeros(n + 1, np.int64)
    cols = np.zeros(max(nnz, 1), np.int32)
    vals = np.zeros(max(nnz, 1), np.float64)
    x = np.zeros(n, np.float64)
    b = np.zeros(n, np.float64)
    xe = np.zeros(n, np.float64)
    L.oracle_generate(nx, ny, nz, rank, size, int(use_7pt), row_ptr, cols, vals, x, b, xe)
    return CSR(row_ptr, cols[:nnz], vals[:nnz], x, b, xe, start_row=n * rank,
               total_nrow=n * size)


def sparsemv(A: CSR, x: np.ndarray, nthreads: int = 1) -> np.ndarray:
    y = np.zeros(A.nrow, np.float64)
    vals = A.vals if A.nnz else np.zeros(1)
    cols = A.cols if A.nnz else np.zeros(1, np.int32)
    lib().oracle_sparsemv(A.nrow, A.row_ptr, cols, vals, np.ascontiguousarray(x, np.float64), y,
                          nthreads)
    return y


def ddot(x: np.ndarray, y: np.ndarray, nthreads: int = 1) -> float:
    return lib().oracle_ddot(len(x), np.ascontiguousarray(x, np.float64),
                             np.ascontiguousarray(y, np.float64), nthreads)


def waxpby(alpha: float, x: np.ndarray, beta: float, y: np.ndarray, nthreads: int = 1):
    w = np.zeros(len(x), np.float64)
    lib().oracle_waxpby(len(x), alpha, np.ascontiguousarray(x, np.float64), beta,
                        np.ascontiguousarray(y, np.float64), w, nthreads)
    return w


def hpccg(A: CSR, b=None, x=None, max_iter: int = 500, tolerance: float = 0.0,
          nthreads: int = 1, trace: bool = True):
    """HPCCG.cpp:312-402 restated. Returns dict(niters, normr, x, times, trace)."""
    b = A.b if b is None else b
    x = (A.x if x is None else x).copy()
    times = np.zeros(7, np.float64)
    tr = np.full(max(max_iter, 1), np.nan, np.float64)
    it = C.c_int(0)
    nr = C.c_double(0.0)
    vals = A.vals if A.nnz else np.zeros(1)
    cols = A.cols if A.nnz else np.zeros(1, np.int32)
    lib().oracle_hpccg(A.nrow, A.row_ptr, cols, vals, np.ascontiguousarray(b), x, max_iter,
                       tolerance, C.byref(it), C.byref(nr), times,
                       tr.ctypes.data_as(C.c_void_p) if trace else None, nthreads)
    return {"niters": it.value, "normr": nr.value, "x": x, "times": times,
            "trace": tr[: it.value + 1] if trace else None}


def print_freq(max_iter: int) -> int:
    """HPCCG.cpp:342-344."""
    pf = max_iter // 10
    return max(1, min(pf, 50))


def max_threads() -> int:
    return lib().oracle_max_threads()


# ---------------------------------------------------------------------------
# Reference build (oracle/_ref), only where it was compiled (this container).
# ---------------------------------------------------------------------------
_ref = None


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def ref_lib(omp: bool = False) -> C.CDLL:
    global _ref
    path = REF_OMP_SO if omp else REF_SO
    if omp:
        L = C.CDLL(path)
    else:
        if _ref is not None:
            return _ref
        L = C.CDLL(path)
    PP = C.POINTER(C.POINTER(C.c_double))
    L.ref_generate.restype = C.c_void_p
    L.ref_generate.argtypes = [C.c_int, C.c_int, C.c_int, PP, PP, PP]
    L.ref_nrow.restype = C.c_int
    L.ref_nrow.argtypes = [C.c_void_p]
    L.ref_total_nnz.restype = C.c_longlong
    L.ref_total_nnz.argtypes = [C.c_void_p]
    L.ref_to_csr.restype = C.c_longlong
    L.ref_to_csr.argtypes = [C.c_void_p, _lp, C.c_void_p, C.c_void_p]
    L.ref_from_csr.restype = C.c_void_p
    L.ref_from_csr.argtypes = [C.c_int, _lp, _ip, _dp]
    L.ref_hpccg.restype = C.c_int
    L.ref_hpccg.argtypes = [C.c_void_p, _dp, _dp, C.c_int, C.c_double, C.POINTER(C.c_int),
                            C.POINTER(C.c_double), _dp]
    L.ref_sparsemv.restype = C.c_int
    L.ref_sparsemv.argtypes = [C.c_void_p, _dp, _dp]
    L.ref_ddot.restype = C.c_double
    L.ref_ddot.argtypes = [C.c_int, _dp, _dp]
    L.ref_waxpby.restype = C.c_int
    L.ref_waxpby.argtypes = [C.c_int, C.c_double, _dp, C.c_double, _dp, _dp]
    L.ref_free.restype = None
    L.ref_free.argtypes = [C.c_void_p]
    L.ref_free_vec.restype = None
    L.ref_free_vec.argtypes = [C.POINTER(C.c_double)]
    if not omp:
        _ref = L
    return L


class RefMatrix:
    """Handle to a reference-built HPC_Sparse_Matrix (freed on close)."""

    def __init__(self, L, handle, n, b=None):
        self.L, self.h, self.nrow, self.b = L, handle, n, b

    def to_csr(self):
        rp = np.zeros(self.nrow + 1, np.int64)
        nnz = self.L.ref_to_csr(self.h, rp, None, None)
        cols = np.zeros(max(nnz, 1), np.int32)
        vals = np.zeros(max(nnz, 1), np.float64)
        self.L.ref_to_csr(self.h, rp, cols.ctypes.data_as(C.c_void_p),
                          vals.ctypes.data_as(C.c_void_p))
        return rp, cols[:nnz], vals[:nnz]

    def close(self):
        if self.h:
            self.L.ref_free(self.h)
            self.h = None


def ref_generate(nx, ny, nz, omp=False):
    """Reference generate_matrix() (serial: size=1, 27-pt, main.cpp:131-132)."""
    L = ref_lib(omp)
    xp = C.POINTER(C.c_double)()
    bp = C.POINTER(C.c_double)()
    ep = C.POINTER(C.c_double)()
    h = L.ref_generate(nx, ny, nz, C.byref(xp), C.byref(bp), C.byref(ep))
    n = L.ref_nrow(h)
    x = np.ctypeslib.as_array(xp, (n,)).copy()
    b = np.ctypeslib.as_array(bp, (n,)).copy()
    xe = np.ctypeslib.as_array(ep, (n,)).copy()
    for p in (xp, bp, ep):
        L.ref_free_vec(p)
    return RefMatrix(L, h, n, b), x, b, xe


def ref_from_csr(A: CSR, omp=False) -> RefMatrix:
    L = ref_lib(omp)
    h = L.ref_from_csr(A.nrow, A.row_ptr, A.cols, A.vals)
    return RefMatrix(L, h, A.nrow, A.b)


def ref_hpccg(M: RefMatrix, b, max_iter=500, tolerance=0.0, x=None):
    """Reference HPCCG() (prints its residual lines to fd 1)."""
    x = np.zeros(M.nrow) if x is None else x.copy()
    times = np.zeros(7)
    it = C.c_int(0)
    nr = C.c_double(0.0)
    M.L.ref_hpccg(M.h, np.ascontiguousarray(b), x, max_iter, tolerance, C.byref(it),
                  C.byref(nr), times)
    return {"niters": it.value, "normr": nr.value, "x": x, "times": times}
