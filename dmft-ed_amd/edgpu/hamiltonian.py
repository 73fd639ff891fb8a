"""Sector Hamiltonian on the MI355X: the host mirror of ED_HAMILTONIAN.

Reference interface mirrored (ED_HAMILTONIAN.f90:9-26):
  build_Hv_sector(isector)   -> builds the basis and the stored H (or selects
                                the matrix-free kernel) and binds spHtimesV_cc
  delete_Hv_sector()         -> frees it (safe after a direct build, which the
                                reference is not: ED_HAMILTONIAN.f90:111-119)
  vecDim_Hv_sector(isector)  -> local vector length (serial: the sector dim)
  spHtimesV_cc(Nloc, v, Hv)  -> cc_sparse_HxV (ED_VARS_GLOBAL.f90:48-54)

Everything computes on the GPU through libedgpu.so; host numpy arrays are
staged over PCIe (the drop-in level), torch device tensors are used in place.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _lib
from ._lib import ED_DIRECT, ED_KRON2_OFF, ED_KRON2_ON, ED_NO_PACK, ED_REAL, ED_STORED, OPTIONS, SectorInfo, check
from .params import EDConfig
from .sectors import Sector as SectorId
from .sectors import setup_pointers


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def _tptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _aptr(a):
    """Pointer of a host numpy array or a (contiguous) torch device tensor."""
    return _ptr(a) if isinstance(a, np.ndarray) else _tptr(a)


def _stream_ptr(stream):
    if stream is None:
        return None
    return ctypes.c_void_p(int(getattr(stream, "cuda_stream", stream)))


class Sector:
    """One symmetry sector resident on one GPU (handle API of include/ed_gpu.h)."""

    def __init__(self, cfg: EDConfig, q1: int, q2: int = 0, *, stored: bool = True,
                 direct: bool = False, real: bool = False, device: int = 0, rows=None,
                 pack: bool = True, kron2: Optional[bool] = None, split: Optional[bool] = None,
                 fused: Optional[bool] = None, options=(), stream=None):
        """rows=(row0, nrows): hold only those rows of H (ed_sector_create_rows,
        the reference's MPI row split); H·v then maps a whole-sector vector to
        the nrows local entries.  pack=False keeps the plain SELL arrays only;
        kron2 forces the two-pass Kronecker tables on (True) or off (False);
        split forces the two-segment stored form on (True, any size) or off
        (False; default: built for stored matrices beyond the Infinity Cache);
        fused likewise for the fused one-pass re-laid form (ed_fused.hpp);
        options: names of ED_OPT_* kernel alternatives (see set_options);
        stream: a torch.cuda.Stream (or raw hipStream_t) the sector runs its
        build and synchronous entry points on, kept by the caller and alive
        longer than the sector (default: a private stream per sector)."""
        lib = _lib.load()
        self.cfg = cfg
        self._params = cfg.to_ctypes()
        flags = (ED_STORED if stored else 0) | (ED_DIRECT if direct else 0) | (ED_REAL if real else 0)
        flags |= 0 if pack else ED_NO_PACK
        if kron2 is not None:
            flags |= ED_KRON2_ON if kron2 else ED_KRON2_OFF
        if split is not None:
            flags |= _lib.ED_SPLIT_ON if split else _lib.ED_NO_SPLIT
        if fused is not None:
            flags |= _lib.ED_FUSED_ON if fused else _lib.ED_NO_FUSED
        h = ctypes.c_void_p()
        if rows is None:
            check(lib.ed_sector_create(ctypes.byref(self._params), q1, q2, flags, device,
                                       _stream_ptr(stream), ctypes.byref(h)), "ed_sector_create")
        else:
            check(lib.ed_sector_create_rows(ctypes.byref(self._params), q1, q2, flags, int(rows[0]),
                                            int(rows[1]), device, _stream_ptr(stream), ctypes.byref(h)),
                  "ed_sector_create_rows")
        self._h = h
        self.device = device
        self.real = real
        info = SectorInfo()
        check(lib.ed_sector_get_info(self._h, ctypes.byref(info)), "ed_sector_get_info")
        self.info = info
        self.dim = int(info.dim)
        self.nnz = int(info.nnz)
        self.row0, self.nrows = int(info.row0), int(info.nrows)
        self.options = ()
        if options:
            self.set_options(*options)

    def set_options(self, *names: str) -> None:
        """Select kernel alternatives by name (ED_OPT_*: no_persist,
        persist_stored, no_preg, no_pkron, split_simple, no_batch,
        eigh_no_verify, trlan_unfused, trlan_nofold, no_graph, trlan_nolocal,
        trlan_nosolo, trlan_fullupd, stored_exact, eigh_fullprobe, no_fused, eigh_nohint;
        edgpu._lib.OPTIONS); no names
        restores the defaults."""
        bits = 0
        for n in names:
            if n not in OPTIONS:
                raise ValueError(f"unknown kernel option {n!r}")
            bits |= OPTIONS[n]
        check(_lib.load().ed_sector_set_options(self._h, bits), "ed_sector_set_options")
        self.options = tuple(names)

    # ------------------------------------------------------------------ life
    def close(self):
        if getattr(self, "_h", None):
            _lib.load().ed_sector_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    # -------------------------------------------------------------- queries
    def map(self) -> np.ndarray:
        """H%map (ED_SETUP.f90:886-984): the sector's Fock states, ascending."""
        m = np.zeros(self.dim, dtype=np.uint32)
        check(_lib.load().ed_sector_map(self._h, _ptr(m)), "ed_sector_map")
        return m

    def dump_csr(self):
        """spH0 in reference row order (sp_dump_matrix, ED_SPARSE_MATRIX.f90:331-388)."""
        rowptr = np.zeros(self.nrows + 1, dtype=np.int64)
        cols = np.zeros(self.nnz, dtype=np.int32)
        vals = np.zeros(self.nnz, dtype=np.complex128)
        check(_lib.load().ed_sector_dump_csr(self._h, _ptr(rowptr), _ptr(cols), _ptr(vals)),
              "ed_sector_dump_csr")
        return rowptr, cols, vals

    # ------------------------------------------------------------------ H·v
    def hxv(self, v: np.ndarray) -> np.ndarray:
        """cc_sparse_HxV on host complex(8) arrays (synchronous)."""
        v = np.ascontiguousarray(v, dtype=np.complex128)
        if v.shape != (self.dim,):
            raise ValueError("spHtimesV_cc: Nloc != dim(isector)")
        hv = np.empty_like(v)
        check(_lib.load().ed_sector_hxv(self._h, self.dim, _ptr(v), _ptr(hv)), "ed_sector_hxv")
        return hv

    def hxv_dev(self, v, hv, path: int = -1, stream=None) -> None:
        """H·v on torch device tensors (float64 or complex128), async on `stream`.

        path: -1 default, 0 stored SELL-64, 1 matrix-free generic, 2 matrix-free Kronecker.
        """
        import torch

        if v.dtype == torch.complex128:
            vt = 1
        elif v.dtype == torch.float64:
            vt = 0
        else:
            raise TypeError("vectors must be float64 or complex128")
        if hv.dtype != v.dtype or v.numel() != self.dim or hv.numel() != self.nrows:
            raise ValueError("shape/dtype mismatch")
        if not (v.is_contiguous() and hv.is_contiguous()):
            raise ValueError("vectors must be contiguous")
        if stream is None:
            stream = torch.cuda.current_stream(v.device)
        check(_lib.load().ed_sector_hxv_dev_path(self._h, path, vt, _tptr(v), _tptr(hv),
                                                 _stream_ptr(stream)), "ed_sector_hxv_dev")

    # -------------------------------------------------------------- Lanczos
    def lanc_tridiag(self, v0: Optional[np.ndarray], nitermax: int, threshold: float = 1e-13,
                     real: Optional[bool] = None):
        """sp_lanc_tridiag: (alfa, beta, nlanc) with beta[0]=0 (blanc(1) unused)."""
        vt, buf = self._vec_arg(v0, real)
        a = np.zeros(nitermax)
        b = np.zeros(nitermax)
        n = ctypes.c_int32()
        check(_lib.load().ed_sector_lanc_tridiag(self._h, vt, buf, nitermax, threshold, _ptr(a),
                                                 _ptr(b), ctypes.byref(n)), "lanc_tridiag")
        return a, b, int(n.value)

    def lanc_eigh(self, nitermax: int = 512, threshold: float = 1e-12, ncheck: int = 10,
                  v0: Optional[np.ndarray] = None, vector: bool = True,
                  real: Optional[bool] = None, on_device: bool = False):
        """sp_lanc_eigh: ground-state energy (and Ritz vector) by plain Lanczos.
        on_device: the Ritz vector stays in HBM (a torch tensor on this
        sector's GPU) instead of being copied to the host."""
        vt, buf = self._vec_arg(v0, real)
        egs = np.zeros(1)
        n = ctypes.c_int32()
        out = None
        if vector:
            out = self._out_array((self.dim,), vt, on_device)
        check(_lib.load().ed_sector_lanc_eigh(self._h, vt, buf, nitermax, threshold, ncheck,
                                              _ptr(egs), None if out is None else _aptr(out),
                                              ctypes.byref(n)), "lanc_eigh")
        return float(egs[0]), out, int(n.value)

    def lanc_run(self, niter: int, v0_dev=None, real: Optional[bool] = None):
        """Fixed-length device Lanczos (benchmark): returns (alpha, beta, ms).
        The vector type follows `real`, else the start vector's dtype (a
        complex tensor runs complex(8) vectors), else the sector's."""
        if real is None and v0_dev is not None:
            real = not v0_dev.is_complex()
        vt = 0 if (self.real if real is None else real) else 1
        if v0_dev is not None:
            if v0_dev.is_complex() != (vt == 1) or v0_dev.numel() != self.dim or not v0_dev.is_contiguous():
                raise ValueError("lanc_run: v0_dev must be a contiguous length-dim vector of the run's type")
        a = np.zeros(niter)
        b = np.zeros(niter)
        ms = ctypes.c_float()
        check(_lib.load().ed_sector_lanc_run(self._h, vt,
                                             None if v0_dev is None else _tptr(v0_dev), niter,
                                             _ptr(a), _ptr(b), ctypes.byref(ms), None),
              "lanc_run")
        return a, b, float(ms.value)

    def lanc_mode(self, real: Optional[bool] = None, path: int = -1) -> int:
        """Recurrence a Lanczos run would take: persistent mode 0 (stored, L2),
        1 (Kronecker tables in LDS), 2 (stored matrix in registers), or -1
        (graph-captured multi-kernel)."""
        vt, _ = self._vec_arg(None, real)
        return int(_lib.load().ed_sector_lanc_mode(self._h, vt, path))

    def eigh(self, neigen: int = 6, ncv: int = 23, maxit: int = 512, tol: float = 1e-12,
             v0: Optional[np.ndarray] = None, vectors: bool = True, real: Optional[bool] = None,
             on_device: bool = False):
        """sp_eigh (ARPACK, which="SR") replacement: thick-restart Lanczos with
        the Krylov basis in HBM.  Returns (eigenvalues, vectors (dim, neigen) or
        None, nconv, number of H·v products).  on_device: the eigenvectors stay
        in HBM (a (dim, neigen) view of a row-major (neigen, dim) torch tensor,
        so column i is contiguous) instead of being copied to the host."""
        vt, buf = self._vec_arg(v0, real)
        ev = np.zeros(neigen)
        out = None
        if vectors:
            out = self._out_array((neigen, self.dim), vt, on_device)
        nconv = ctypes.c_int32()
        nhv = ctypes.c_int32()
        check(_lib.load().ed_sector_eigh(self._h, vt, neigen, ncv, maxit, tol, buf, _ptr(ev),
                                         None if out is None else _aptr(out), ctypes.byref(nconv),
                                         ctypes.byref(nhv)), "ed_sector_eigh")
        return ev, (out.T if out is not None else None), int(nconv.value), int(nhv.value)

    def _out_array(self, shape, vt, on_device):
        if not on_device:
            return np.zeros(shape, dtype=np.complex128 if vt else np.float64)
        import torch

        return torch.empty(shape, dtype=torch.complex128 if vt else torch.float64,
                           device=torch.device("cuda", self.device))

    def _vec_arg(self, v0, real):
        use_real = self.real if real is None else real
        vt = 0 if use_real else 1
        if v0 is None:
            return vt, None
        arr = np.ascontiguousarray(v0, dtype=np.float64 if vt == 0 else np.complex128)
        if arr.shape != (self.dim,):
            raise ValueError("start vector length != dim")
        self._keep = arr
        return vt, _ptr(arr)


def eigh_batch(sectors, neigen: int = 6, ncv: int = 23, maxit=512, tol: float = 1e-12,
               v0s=None, vectors: bool = True, on_device: bool = False, stream=None,
               fallback: bool = True):
    """Sector.eigh (real vectors) for many sectors of one GPU at once
    (ed_sectors_eigh_batch): the small stored sectors' restart cycles share
    launches.  Returns one (eigenvalues, vectors (dim, neigen) or None, nconv,
    H·v products) per sector, and the number finished inside the batch.
    maxit: one Nitermax for all, or one per sector.  fallback=False: sectors
    the batch cannot take or finish come back with nconv == -1 (and no
    eigenvalues) for the caller to solve, instead of one after the other here."""
    n = len(sectors)
    if n == 0:
        return [], 0
    lib = _lib.load()
    hs = (ctypes.c_void_p * n)(*[s.handle for s in sectors])
    keep = []
    v0p = None
    if v0s is not None:
        v0p = (ctypes.c_void_p * n)()
        for i, (s, v) in enumerate(zip(sectors, v0s)):
            if v is None:
                continue
            a = np.ascontiguousarray(v, dtype=np.float64)
            if a.shape != (s.dim,):
                raise ValueError("start vector length != dim")
            keep.append(a)
            v0p[i] = a.ctypes.data
    ev = np.zeros((n, neigen))
    outs = [s._out_array((neigen, s.dim), 0, on_device) if vectors else None for s in sectors]
    ep = (ctypes.c_void_p * n)(*[(o.ctypes.data if isinstance(o, np.ndarray) else o.data_ptr())
                                 if o is not None else None for o in outs])
    nconv = np.zeros(n, dtype=np.int32)
    nhv = np.zeros(n, dtype=np.int32)
    nb = ctypes.c_int32()
    mx = np.ascontiguousarray(np.broadcast_to(np.asarray(maxit, dtype=np.int32), (n,)))
    check(lib.ed_sectors_eigh_batch(hs, n, neigen, ncv, _ptr(mx), tol, v0p, _ptr(ev), ep, _ptr(nconv), _ptr(nhv),
                                    ctypes.byref(nb), 0 if fallback else _lib.ED_BATCH_NO_FALLBACK,
                                    _stream_ptr(stream)), "ed_sectors_eigh_batch")
    res = [(ev[i].copy(), outs[i].T if outs[i] is not None else None, int(nconv[i]), int(nhv[i]))
           for i in range(n)]
    return res, int(nb.value)


# ------------------------------------------------------------ reference API
_current: Optional[Sector] = None


def build_Hv_sector(cfg: EDConfig, isector: int, *, sparse_H: bool = True,
                    real: bool = False, device: int = 0) -> Sector:
    """build_Hv_sector(isector) (ED_HAMILTONIAN.f90:42-103): ed_sparse_H selects
    stored (T) or matrix-free (F) H·v for the current sector."""
    global _current
    sec: SectorId = setup_pointers(cfg)[isector - 1]
    if _current is not None:
        _current.close()
    _current = Sector(cfg, sec.q1, sec.q2, stored=sparse_H, direct=not sparse_H, real=real,
                      device=device)
    return _current


def delete_Hv_sector() -> None:
    global _current
    if _current is not None:
        _current.close()
    _current = None


def vecDim_Hv_sector(cfg: EDConfig, isector: int) -> int:
    """Serial vecDim_Hv_sector: MpiQ=Dim, MpiR=0 (ED_HAMILTONIAN.f90:126-149)."""
    return setup_pointers(cfg)[isector - 1].dim


def spHtimesV_cc(Nloc: int, v: np.ndarray, Hv: np.ndarray) -> None:
    """The procedure bound by build_Hv_sector: Hv = H v, overwriting Hv."""
    if _current is None:
        raise RuntimeError("spHtimesV_cc ERROR: Hsector NOT set")
    if Nloc != _current.dim:
        raise ValueError("spHtimesV_cc ERROR: Nloc != dim(isector)")
    Hv[:] = _current.hxv(v)
