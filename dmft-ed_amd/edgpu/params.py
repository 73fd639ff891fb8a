"""Host-side model parameters: the ``ed_params`` C struct and the bath object.

Mirrors the reference's parameter plumbing for the H·v hot path:

* ``EDConfig``           <- input flags of ED_INPUT_VARS.f90:103-222 that enter H
* ``ed_setup_dimensions`` <- ED_SETUP.f90:96-143
* ``allocate_dmft_bath`` / ``init_dmft_bath`` <- ED_BATH/dmft_aux.f90:4-50, 78-256
  (flat bath; the ``hamiltonian.restart`` reader is out of scope)
* ``EdParams``           <- the C-ABI struct ``ed_params`` of include/ed_gpu.h

Arrays use the reference's index order with 0-based indices:
``imphloc[ispin, jspin, iorb, jorb]``, ``bath.e[ispin, iorb, k]`` ...
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

ED_MAX_NORB = 3
ED_MAX_NSPIN = 2
ED_MAX_NBATH = 32
ED_MAX_NS = 16

MODES = {"normal": 0, "superc": 1, "nonsu2": 2}
BATHS = {"normal": 0, "hybrid": 1, "replica": 2}

_c_double = ctypes.c_double
_c_int32 = ctypes.c_int32
_H4 = ED_MAX_NSPIN * ED_MAX_NSPIN * ED_MAX_NORB * ED_MAX_NORB
_B3 = ED_MAX_NSPIN * ED_MAX_NORB * ED_MAX_NBATH
_B5 = _H4 * ED_MAX_NBATH


class EdParams(ctypes.Structure):
    """ctypes mirror of ``ed_params`` (include/ed_gpu.h)."""

    _fields_ = [
        ("norb", _c_int32), ("nspin", _c_int32), ("nbath", _c_int32),
        ("ed_mode", _c_int32), ("bath_type", _c_int32), ("hfmode", _c_int32),
        ("uloc", _c_double * 3),
        ("ust", _c_double), ("jh", _c_double), ("jx", _c_double), ("jp", _c_double),
        ("xmu", _c_double),
        ("imphloc_re", _c_double * _H4), ("imphloc_im", _c_double * _H4),
        ("bath_e", _c_double * _B3), ("bath_v", _c_double * _B3),
        ("bath_u", _c_double * _B3), ("bath_d", _c_double * _B3),
        ("bath_h_re", _c_double * _B5), ("bath_h_im", _c_double * _B5),
        ("bath_vr_re", _c_double * ED_MAX_NBATH), ("bath_vr_im", _c_double * ED_MAX_NBATH),
        ("jz_basis", _c_int32), ("pad_", _c_int32),
    ]


@dataclass
class Bath:
    """``effective_bath`` (ED_VARS_GLOBAL.f90:12-22) with 0-based numpy arrays."""

    e: Optional[np.ndarray] = None   # (Nspin, Norb|1, Nbath) real
    v: Optional[np.ndarray] = None   # (Nspin, Norb, Nbath) real
    u: Optional[np.ndarray] = None   # (Nspin, Norb, Nbath) real (nonsu2)
    d: Optional[np.ndarray] = None   # (Nspin, Norb|1, Nbath) real (superc)
    h: Optional[np.ndarray] = None   # (Nspin, Nspin, Norb, Norb, Nbath) complex (replica)
    vr: Optional[np.ndarray] = None  # (Nbath,) complex (replica)


@dataclass
class EDConfig:
    """The input variables that define the sector Hamiltonian.

    Defaults are the reference defaults (ED_INPUT_VARS.f90:121-196).
    """

    Norb: int = 1
    Nbath: int = 6
    Nspin: int = 1
    ed_mode: str = "normal"
    bath_type: str = "normal"
    Uloc: tuple = (2.0, 0.0, 0.0)
    Ust: float = 0.0
    Jh: float = 0.0
    Jx: float = 0.0
    Jp: float = 0.0
    xmu: float = 0.0
    hfmode: bool = True
    deltasc: float = 0.02
    hwband: float = 2.0
    ed_vsf_ratio: float = 0.1
    ed_bath_noise_thr: float = 0.0
    impHloc: Optional[np.ndarray] = None  # (Nspin, Nspin, Norb, Norb) complex
    bath: Bath = field(default_factory=Bath)
    # nonsu2 sectors labelled (n, twoJz) (ED_INPUT_VARS.f90:78-80, 193-195)
    Jz_basis: bool = False
    Jz_max: bool = False
    Jz_max_value: float = 1000.0

    # --------------------------------------------------------------- derived
    @property
    def Ns(self) -> int:
        """Levels per spin, ed_setup_dimensions ED_SETUP.f90:98-105."""
        if self.bath_type == "hybrid":
            return self.Nbath + self.Norb
        return (self.Nbath + 1) * self.Norb

    @property
    def Nlevels(self) -> int:
        return 2 * self.Ns

    @property
    def jhflag(self) -> bool:
        """ED_SETUP.f90:289-290."""
        return self.Norb > 1 and (self.Jx != 0.0 or self.Jp != 0.0)

    def check(self) -> None:
        """ed_checks_global ED_SETUP.f90:51-87 (the parts that matter here)."""
        if self.Nspin > 2:
            raise ValueError("ED ERROR: Nspin > 2 is currently not supported")
        if self.Norb > 3:
            raise ValueError("ED ERROR: Norb > 3 is currently not supported")
        if self.ed_mode == "superc" and self.Nspin > 1:
            raise ValueError("ED ERROR: SC + AFM is currently not supported .")
        if self.ed_mode == "nonsu2" and self.Nspin != 2:
            raise ValueError("ED msg: ed_mode=nonSU2 with Nspin!=2 is not allowed.")
        if self.ed_mode not in MODES or self.bath_type not in BATHS:
            raise ValueError("unknown ed_mode / bath_type")
        if self.Jz_basis and (self.ed_mode != "nonsu2" or self.bath_type == "hybrid"):
            raise ValueError("Jz_basis needs ed_mode=nonsu2 and a normal/replica bath (Ns = Norb*(Nbath+1))")
        if self.Nbath > ED_MAX_NBATH or self.Ns > ED_MAX_NS:
            raise ValueError(f"Ns={self.Ns} exceeds the {ED_MAX_NS}-level limit of 32-bit states")

    def is_real(self) -> bool:
        """True when H is real: impHloc and the bath carry no imaginary part."""
        if self.impHloc is not None and np.any(np.imag(self.impHloc) != 0):
            return False
        b = self.bath
        for arr in (b.h, b.vr):
            if arr is not None and np.any(np.imag(arr) != 0):
                return False
        return True

    # ------------------------------------------------------------- to C-ABI
    def to_ctypes(self) -> EdParams:
        self.check()
        p = EdParams()
        p.norb, p.nspin, p.nbath = self.Norb, self.Nspin, self.Nbath
        p.ed_mode, p.bath_type = MODES[self.ed_mode], BATHS[self.bath_type]
        p.hfmode = int(bool(self.hfmode))
        for i in range(3):
            p.uloc[i] = float(self.Uloc[i])
        p.ust, p.jh, p.jx, p.jp, p.xmu = self.Ust, self.Jh, self.Jx, self.Jp, self.xmu

        def put(dst, shape, arr):
            view = np.frombuffer(dst, dtype=np.float64).reshape(shape)
            view[...] = 0.0
            if arr is not None:
                a = np.asarray(arr, dtype=np.float64)
                view[tuple(slice(0, s) for s in a.shape)] = a

        H4 = (ED_MAX_NSPIN, ED_MAX_NSPIN, ED_MAX_NORB, ED_MAX_NORB)
        B3 = (ED_MAX_NSPIN, ED_MAX_NORB, ED_MAX_NBATH)
        B5 = H4 + (ED_MAX_NBATH,)
        h = self.impHloc
        put(p.imphloc_re, H4, None if h is None else np.real(h))
        put(p.imphloc_im, H4, None if h is None else np.imag(h))
        b = self.bath
        put(p.bath_e, B3, b.e)
        put(p.bath_v, B3, b.v)
        put(p.bath_u, B3, b.u)
        put(p.bath_d, B3, b.d)
        put(p.bath_h_re, B5, None if b.h is None else np.real(b.h))
        put(p.bath_h_im, B5, None if b.h is None else np.imag(b.h))
        put(p.bath_vr_re, (ED_MAX_NBATH,), None if b.vr is None else np.real(b.vr))
        put(p.bath_vr_im, (ED_MAX_NBATH,), None if b.vr is None else np.imag(b.vr))
        p.jz_basis = int(bool(self.Jz_basis))
        return p


# ----------------------------------------------------------------------- bath
def allocate_dmft_bath(cfg: EDConfig) -> Bath:
    """ED_BATH/dmft_aux.f90:4-50."""
    Ns_, No, Nb = cfg.Nspin, cfg.Norb, cfg.Nbath
    b = Bath()
    if cfg.bath_type in ("normal", "hybrid"):
        ne = No if cfg.bath_type == "normal" else 1
        b.e = np.zeros((Ns_, ne, Nb))
        b.v = np.zeros((Ns_, No, Nb))
        if cfg.ed_mode == "superc":
            b.d = np.zeros((Ns_, ne, Nb))
        if cfg.ed_mode == "nonsu2":
            b.u = np.zeros((Ns_, No, Nb))
    else:
        b.h = np.zeros((Ns_, Ns_, No, No, Nb), dtype=np.complex128)
        b.vr = np.zeros((Nb,), dtype=np.complex128)
    return b


def init_dmft_bath(cfg: EDConfig, noise: Optional[np.ndarray] = None) -> Bath:
    """Flat initial bath, ED_BATH/dmft_aux.f90:78-150.

    ``noise`` plays the role of ``noise_b*ed_bath_noise_thr`` (default 0, the
    reference default ``ED_BATH_NOISE_THR=0``, ED_INPUT_VARS.f90:187).
    """
    b = allocate_dmft_bath(cfg)
    Nb = cfg.Nbath
    nb = np.zeros(Nb) if noise is None else np.asarray(noise, dtype=np.float64)
    hw = cfg.hwband
    if cfg.bath_type in ("normal", "hybrid"):
        # Fortran 1-based k -> index k-1
        b.e[:, :, 0] = -hw + nb[0]
        b.e[:, :, Nb - 1] = hw + nb[Nb - 1]
        Nh = Nb // 2
        if Nb % 2 == 0 and Nb >= 4:
            de = hw / max(Nh - 1, 1)
            b.e[:, :, Nh - 1] = -1.0e-3 + nb[Nh - 1]
            b.e[:, :, Nh] = 1.0e-3 + nb[Nh]
            for i in range(2, Nh):
                b.e[:, :, i - 1] = -hw + (i - 1) * de + nb[i - 1]
                b.e[:, :, Nb - i] = hw - (i - 1) * de + nb[Nb - i]
        elif Nb % 2 != 0 and Nb >= 3:
            de = hw / Nh
            b.e[:, :, Nh] = 0.0 + nb[Nh]
            for i in range(2, Nh + 1):
                b.e[:, :, i - 1] = -hw + (i - 1) * de + nb[i - 1]
                b.e[:, :, Nb - i] = hw - (i - 1) * de + nb[Nb - i]
        for i in range(Nb):
            b.v[:, :, i] = max(0.1, 1.0 / np.sqrt(float(Nb))) + nb[i]
        if cfg.ed_mode == "superc":
            b.d[...] = cfg.deltasc
        if cfg.ed_mode == "nonsu2":
            for i in range(Nb):
                b.u[:, :, i] = b.v[:, :, i] * cfg.ed_vsf_ratio + nb[i]
    else:
        himp = cfg.impHloc if cfg.impHloc is not None else np.zeros(
            (cfg.Nspin, cfg.Nspin, cfg.Norb, cfg.Norb), dtype=np.complex128)
        eye = np.zeros_like(himp)
        for s in range(cfg.Nspin):
            for o in range(cfg.Norb):
                eye[s, s, o, o] = 1.0
        for i in range(Nb):
            b.h[..., i] = himp - (cfg.xmu + nb[i]) * eye
            b.vr[i] = complex(0.5 + nb[i], 0.0)
    return b


def random_bath(cfg: EDConfig, seed: int = 20251015) -> Bath:
    """Synthetic random bath of SURVEY.md §8(d): e ~ U(-2,2) sorted, V ~ U(0.1,1)/sqrt(Nbath).

    Same values for both spins and every orbital's own energy list drawn
    independently.  nonsu2: u = ed_vsf_ratio * v; superc: d = deltasc.
    """
    rng = np.random.default_rng(seed)
    b = allocate_dmft_bath(cfg)
    Nb = cfg.Nbath
    if cfg.bath_type == "replica":
        for i in range(Nb):
            e = rng.uniform(-2.0, 2.0)
            for s in range(cfg.Nspin):
                for o in range(cfg.Norb):
                    b.h[s, s, o, o, i] = e
            b.vr[i] = rng.uniform(0.1, 1.0) / np.sqrt(Nb)
        return b
    ne = b.e.shape[1]
    for o in range(ne):
        b.e[:, o, :] = np.sort(rng.uniform(-2.0, 2.0, size=Nb))[None, :]
    for o in range(cfg.Norb):
        b.v[:, o, :] = (rng.uniform(0.1, 1.0, size=Nb) / np.sqrt(Nb))[None, :]
    if b.u is not None:
        b.u[...] = b.v * cfg.ed_vsf_ratio
    if b.d is not None:
        b.d[...] = cfg.deltasc
    return b


def make_config(Norb=1, Nbath=7, Nspin=1, ed_mode="normal", bath_type="normal",
                bath="flat", seed=20251015, **kw) -> EDConfig:
    """Convenience constructor: a config with its flat (reference default) or random bath."""
    cfg = EDConfig(Norb=Norb, Nbath=Nbath, Nspin=Nspin, ed_mode=ed_mode,
                   bath_type=bath_type, **kw)
    if cfg.impHloc is None:
        cfg.impHloc = np.zeros((Nspin, Nspin, Norb, Norb), dtype=np.complex128)
    cfg.check()
    if bath == "flat":
        cfg.bath = init_dmft_bath(cfg)
    elif bath == "random":
        cfg.bath = random_bath(cfg, seed)
    elif isinstance(bath, Bath):
        cfg.bath = bath
    else:
        raise ValueError(bath)
    return cfg
