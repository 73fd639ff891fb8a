"""Impurity Green's function by Lanczos continued fraction, normal mode.

Mirrors build_gf_normal / lanc_build_gf_normal_c / add_to_lanczos_gf_normal
(ED_GF_NORMAL.f90:18-92, 116-260, 580-632) for the diagonal components
G_{aa,ss}.  Per kept state |gs> (energy E_i), orbital a, spin s:

  * seed  c+_{a s}|gs>  in sector getCDGsector(s, isector)  and
          c_{a s}|gs>   in sector getCsector(s, isector),
    built on the GPU (ed_sector_apply_op, the vvinit loop :159-174);
  * norm2 = <seed|seed>, seed /= sqrt(norm2);
  * nlanc = min(jdim, lanc_nGFiter) steps of sp_lanc_tridiag on the GPU
    (device-resident plain Lanczos from a device start vector);
  * poles: eigen-decomposition of the tridiagonal (diag alfa, subdiag beta(2:),
    LAPACK like the reference's eigh), weight norm2/Z * Z(1,j)^2,
    G(iw_n) += w/(iw_n - isign*(E_j - E_i)), G(w) += w/(w + i eps - isign*(E_j - E_i))
    with w_n = pi/beta (2n-1) and w = linspace(wini, wfin, Lreal)
    (allocate_grids, ED_AUX_FUNX.f90:449-461).
The pole sum runs in torch on the GPU when one is present (200 poles x 10^4
frequencies per seed), else in numpy.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

from . import _lib
from ._lib import check
from .diag import StateList
from .hamiltonian import Sector
from .params import EDConfig
from .sectors import c_sector, cdg_sector, setup_pointers


@dataclass
class GFOptions:
    """ED_INPUT_VARS defaults (ED_INPUT_VARS.f90:126-173)."""

    lanc_nGFiter: int = 200
    Lmats: int = 5000
    Lreal: int = 5000
    beta: float = 1000.0
    eps: float = 0.01
    wini: float = -5.0
    wfin: float = 5.0
    threshold: float = 1e-13      # sp_lanc_tridiag breakdown test (.repo/PLAIN_LANCZOS.f90:27)
    sparse_H: bool = True         # ed_sparse_H


def matsubara(beta: float, L: int) -> np.ndarray:
    return np.pi / beta * (2.0 * np.arange(1, L + 1) - 1.0)


def realaxis(wini: float, wfin: float, L: int) -> np.ndarray:
    return np.linspace(wini, wfin, L)


def tridiag_poles(alfa: np.ndarray, beta: np.ndarray, n: int) -> Tuple[np.ndarray, np.ndarray]:
    """Eigenvalues of tridiag(alfa(1:n), beta(2:n)) and squared first components."""
    from scipy.linalg import eigh_tridiagonal

    if n == 1:
        return np.array([alfa[0]]), np.array([1.0])
    w, z = eigh_tridiagonal(alfa[:n], beta[1:n])
    return w, z[0, :] ** 2


def add_poles(G_mats, G_real, peso_bz: float, Ei: float, E: np.ndarray, z2: np.ndarray,
              isign: int, wm: np.ndarray, wr: np.ndarray, eps: float) -> None:
    """add_to_lanczos_gf_normal inner loops (ED_GF_NORMAL.f90:620-631), vectorised."""
    de = E - Ei
    peso = peso_bz * z2
    try:
        import torch

        if torch.cuda.is_available():
            dev = "cuda"
            iw = torch.from_numpy(1j * wm).to(dev)
            rw = torch.from_numpy(wr + 1j * eps).to(dev)
            p = torch.from_numpy(peso.astype(np.complex128)).to(dev)
            d = torch.from_numpy((isign * de).astype(np.complex128)).to(dev)
            G_mats += (p[None, :] / (iw[:, None] - d[None, :])).sum(1).cpu().numpy()
            G_real += (p[None, :] / (rw[:, None] - d[None, :])).sum(1).cpu().numpy()
            return
    except Exception:
        pass
    G_mats += (peso[None, :] / ((1j * wm)[:, None] - isign * de[None, :])).sum(1)
    G_real += (peso[None, :] / ((wr + 1j * eps)[:, None] - isign * de[None, :])).sum(1)


def _seed(src: Sector, dst: Sector, op: int, level: int, vec: np.ndarray, real: bool):
    """apply c (op=0) / c+ (op=1) on the device; returns (normalised seed, norm2)."""
    import torch

    dt = torch.float64 if real else torch.complex128
    dev = f"cuda:{src.device}"
    x = torch.from_numpy(np.ascontiguousarray(vec.astype(np.float64 if real else np.complex128))).to(dev)
    y = torch.empty(dst.dim, dtype=dt, device=dev)
    st = torch.cuda.current_stream(x.device)
    check(_lib.load().ed_sector_apply_op(src.handle, dst.handle, op, level, 0 if real else 1,
                                         ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                                         ctypes.c_void_p(st.cuda_stream)), "ed_sector_apply_op")
    norm2 = float(torch.sum(y.abs() ** 2).item()) if not real else float(torch.dot(y, y).item())
    if norm2 > 0:
        y = y / np.sqrt(norm2)
    torch.cuda.synchronize(x.device)
    return y.contiguous(), norm2


def _tridiag_dev(S: Sector, seed, nlanc: int, real: bool, threshold: float):
    a = np.zeros(nlanc)
    b = np.zeros(nlanc)
    n = ctypes.c_int32()
    check(_lib.load().ed_sector_lanc_tridiag_dev(S.handle, 0 if real else 1,
                                                 ctypes.c_void_p(seed.data_ptr()), nlanc, threshold,
                                                 a.ctypes.data_as(ctypes.c_void_p),
                                                 b.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n)),
          "ed_sector_lanc_tridiag_dev")
    return a, b, int(n.value)


def build_gf_normal(cfg: EDConfig, states: StateList, gopt: Optional[GFOptions] = None,
                    device: int = 0, record: Optional[list] = None):
    """impGmats, impGreal of shape (Nspin, Nspin, Norb, Norb, L): diagonal part."""
    gopt = gopt or GFOptions()
    Ns, No, Nsp = cfg.Ns, cfg.Norb, cfg.Nspin
    wm = matsubara(gopt.beta, gopt.Lmats)
    wr = realaxis(gopt.wini, gopt.wfin, gopt.Lreal)
    Gm = np.zeros((Nsp, Nsp, No, No, gopt.Lmats), dtype=np.complex128)
    Gr = np.zeros((Nsp, Nsp, No, No, gopt.Lreal), dtype=np.complex128)
    real = cfg.is_real()
    secs = setup_pointers(cfg)
    zeta = float(states.size)                 # T=0: zeta_function = state_list%size (ED_DIAG.f90:411)
    for ispin in range(Nsp):
        for iorb in range(No):
            isite = iorb + ispin * Ns          # impIndex(iorb,ispin), 0-based bit
            for e_i, isec, vec in zip(states.energies, states.sectors, states.vectors):
                if vec is None:
                    raise ValueError("build_gf_normal needs the state vectors (keep_vectors=True)")
                sec = secs[isec - 1]
                with Sector(cfg, sec.q1, sec.q2, stored=False, direct=True, real=real,
                            device=device) as HI:
                    for op, isign, jsec in ((1, +1, cdg_sector(cfg, sec, ispin)),
                                            (0, -1, c_sector(cfg, sec, ispin))):
                        if jsec is None:
                            continue
                        with Sector(cfg, jsec.q1, jsec.q2, stored=gopt.sparse_H,
                                    direct=not gopt.sparse_H, real=real, device=device) as HJ:
                            seed, norm2 = _seed(HI, HJ, op, isite, vec, real)
                            if norm2 == 0.0:
                                continue
                            nlanc = min(HJ.dim, gopt.lanc_nGFiter)
                            a, b, n = _tridiag_dev(HJ, seed, nlanc, real, gopt.threshold)
                        # the reference diagonalises all nlanc entries (unset ones stay 0)
                        E, z2 = tridiag_poles(a, b, nlanc)
                        if record is not None:
                            record.append(dict(ispin=ispin, iorb=iorb, isector=isec, op=op,
                                               norm2=norm2, alfa=a, beta=b, nlanc=n))
                        add_poles(Gm[ispin, ispin, iorb, iorb], Gr[ispin, ispin, iorb, iorb],
                                  norm2 / zeta, e_i, E, z2, isign, wm, wr, gopt.eps)
    return Gm, Gr
