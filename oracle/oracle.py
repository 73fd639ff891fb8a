"""ctypes front-end of the CPU oracle (oracle/ed_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product package dmft-ed_amd/.
Every wrapper names the reference routine restated in ed_oracle.c.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libedoracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        P = ctypes.c_void_p
        i64, i32, f64 = ctypes.c_int64, ctypes.c_int32, ctypes.c_double
        L.orc_ns.argtypes = [P]; L.orc_ns.restype = ctypes.c_int
        L.orc_build_sector.argtypes = [P, i32, i32, P]; L.orc_build_sector.restype = i64
        L.orc_build_csr.argtypes = [P, P, i64, P, P, P, i64]; L.orc_build_csr.restype = i64
        L.orc_build_csr_rows.argtypes = [P, P, i64, i64, i64, P, P, P, i64]
        L.orc_build_csr_rows.restype = i64
        L.orc_spmv.argtypes = [i64, P, P, P, P, P]; L.orc_spmv.restype = None
        L.orc_spmv_real.argtypes = [i64, P, P, P, P, P]; L.orc_spmv_real.restype = None
        L.orc_direct_hxv.argtypes = [P, P, i64, P, P]; L.orc_direct_hxv.restype = ctypes.c_int
        L.orc_lanc_tridiag.argtypes = [i64, P, P, P, P, ctypes.c_int, f64, P, P]
        L.orc_lanc_tridiag.restype = ctypes.c_int
        L.orc_lanc_eigh.argtypes = [i64, P, P, P, P, ctypes.c_int, f64, ctypes.c_int, P]
        L.orc_lanc_eigh.restype = ctypes.c_int
        L.orc_tql2.argtypes = [ctypes.c_int, P, P, P]; L.orc_tql2.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class Oracle:
    """Oracle bound to one EDConfig (the ctypes params are kept alive here)."""

    def __init__(self, cfg):
        self.cfg = cfg
        self.params = cfg.to_ctypes()
        self._pp = ctypes.cast(ctypes.pointer(self.params), ctypes.c_void_p)

    # build_sector ED_SETUP.f90:886-984
    def build_sector(self, q1, q2=0) -> np.ndarray:
        L = lib()
        dim = L.orc_build_sector(self._pp, q1, q2, None)
        m = np.zeros(dim, dtype=np.uint32)
        L.orc_build_sector(self._pp, q1, q2, _p(m))
        return m

    # ed_buildH_c ED_HAMILTONIAN_STORED_HxV.f90:28-113 (spH0 row-of-arrays order)
    def build_csr(self, hmap: np.ndarray):
        L = lib()
        dim = len(hmap)
        rowptr = np.zeros(dim + 1, dtype=np.int64)
        nnz = L.orc_build_csr(self._pp, _p(hmap), dim, _p(rowptr), None, None, 0)
        if nnz < 0:
            raise RuntimeError(f"orc_build_csr failed ({nnz})")
        cols = np.zeros(nnz, dtype=np.int32)
        vals = np.zeros(nnz, dtype=np.complex128)
        r = L.orc_build_csr(self._pp, _p(hmap), dim, _p(rowptr), _p(cols), _p(vals), nnz)
        assert r == nnz
        return rowptr, cols, vals

    # rows [row0, row0+nrows) of ed_buildH_c's CSR (ED_HAMILTONIAN_STORED_HxV.f90:28-113)
    def build_csr_rows(self, hmap: np.ndarray, row0: int, nrows: int):
        L = lib()
        dim = len(hmap)
        hmap = np.ascontiguousarray(hmap, dtype=np.uint32)
        rowptr = np.zeros(nrows + 1, dtype=np.int64)
        nnz = L.orc_build_csr_rows(self._pp, _p(hmap), dim, row0, nrows, _p(rowptr), None, None, 0)
        if nnz < 0:
            raise RuntimeError(f"orc_build_csr_rows failed ({nnz})")
        cols = np.zeros(nnz, dtype=np.int32)
        vals = np.zeros(nnz, dtype=np.complex128)
        r = L.orc_build_csr_rows(self._pp, _p(hmap), dim, row0, nrows, _p(rowptr), _p(cols), _p(vals), nnz)
        assert r == nnz
        return rowptr, cols, vals

    # directMatVec_cc ED_HAMILTONIAN_DIRECT_HxV.f90:21-92
    def direct_hxv(self, hmap, v):
        v = np.ascontiguousarray(v, dtype=np.complex128)
        hv = np.zeros_like(v)
        st = lib().orc_direct_hxv(self._pp, _p(hmap), len(hmap), _p(v), _p(hv))
        if st:
            raise RuntimeError(f"orc_direct_hxv failed ({st})")
        return hv


# spMatVec_cc ED_HAMILTONIAN_STORED_HxV.f90:132-143
def spmv(csr, v):
    rowptr, cols, vals = csr
    v = np.ascontiguousarray(v, dtype=np.complex128)
    hv = np.zeros_like(v)
    lib().orc_spmv(len(rowptr) - 1, _p(rowptr), _p(cols), _p(vals), _p(v), _p(hv))
    return hv


def spmv_real(csr, v):
    rowptr, cols, vals = csr
    vr = np.ascontiguousarray(np.real(vals), dtype=np.float64)
    v = np.ascontiguousarray(v, dtype=np.float64)
    hv = np.zeros_like(v)
    lib().orc_spmv_real(len(rowptr) - 1, _p(rowptr), _p(cols), _p(vr), _p(v), _p(hv))
    return hv


# lanczos_plain_tridiag_c .repo/PLAIN_LANCZOS.f90:154-180
def lanc_tridiag(csr, v0, nitermax, threshold=1e-13):
    rowptr, cols, vals = csr
    v0 = np.ascontiguousarray(v0, dtype=np.complex128)
    a = np.zeros(nitermax)
    b = np.zeros(nitermax)
    n = lib().orc_lanc_tridiag(len(rowptr) - 1, _p(rowptr), _p(cols), _p(vals), _p(v0),
                               nitermax, threshold, _p(a), _p(b))
    return a, b, n


# lanczos_plain_c .repo/PLAIN_LANCZOS.f90:286-385
def lanc_eigh(csr, v0, nitermax, threshold=1e-12, ncheck=10):
    rowptr, cols, vals = csr
    vect = np.array(v0, dtype=np.complex128, copy=True)
    egs = np.zeros(1)
    n = lib().orc_lanc_eigh(len(rowptr) - 1, _p(rowptr), _p(cols), _p(vals), _p(vect),
                            nitermax, threshold, ncheck, _p(egs))
    return float(egs[0]), vect, n


# tql2 .repo/PLAIN_LANCZOS.f90:427-565
def tql2(d, e):
    n = len(d)
    d = np.array(d, dtype=np.float64, copy=True)
    e = np.array(e, dtype=np.float64, copy=True)
    z = np.asfortranarray(np.eye(n))
    ierr = lib().orc_tql2(n, _p(d), _p(e), _p(z))
    return d, z, ierr


def start_vector(dim: int) -> np.ndarray:
    """The SpMV probe of SURVEY §8(d): x(i) = (sin i, cos 3i), i 1-based."""
    i = np.arange(1, dim + 1, dtype=np.float64)
    return np.sin(i) + 1j * np.cos(3.0 * i)
