"""Symmetry-sector bookkeeping (host side, tiny tables).

Mirrors ``setup_pointers_normal/superc/nonsu2`` (ED_SETUP.f90:372-808, incl.
the nonsu2 ``Jz_basis`` pointers :636-664, 769-805) and the sector dimension
functions (ED_SETUP.f90:809-876).  Sector ids are the reference's 1-based
``isector``.
"""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache
from math import comb
from typing import Dict, List, Tuple

import numpy as np

from .params import EDConfig


@dataclass(frozen=True)
class Sector:
    isector: int       # 1-based, reference order
    q1: int            # nup | sz | n
    q2: int            # ndw | 0  | 0 (twoJz for Jz_basis)
    dim: int


def binomial(n1: int, n2: int) -> int:
    """ED_SETUP.f90:1283-1300 (exact integer version; identical for n1 <= 32)."""
    if n2 < 0:
        return 0
    return comb(n1, n2) if n2 <= n1 else 0


LZDIAG = (-1, +1, 0)   # ED_VARS_GLOBAL.f90:207
SZDIAG = (+1, -1)      # ED_VARS_GLOBAL.f90:208


@lru_cache(maxsize=16)
def _jz_hist(Ns: int, Norb: int) -> np.ndarray:
    """Counts of Ns-bit patterns by (popcount, 2*Lz), 2*Lz offset by 2*Ns;
    level l belongs to orbital l mod Norb (ivec(iorb+Norb*ibath), ED_SETUP.f90:865)."""
    x = np.arange(1 << Ns, dtype=np.int64)
    bits = (x[:, None] >> np.arange(Ns)) & 1
    pc = bits.sum(1)
    lz2 = (bits * np.array([2 * LZDIAG[l % Norb] for l in range(Ns)])).sum(1)
    h = np.zeros((Ns + 1, 4 * Ns + 1), dtype=np.int64)
    np.add.at(h, (pc, lz2 + 2 * Ns), 1)
    return h


def sector_dim_jz(cfg: EDConfig, n: int, twoJz: int) -> int:
    """get_nonsu2_sector_dimension_Jz (ED_SETUP.f90:848-876): states with
    nup+ndw = n and (nup-ndw) + 2Lz(up) + 2Lz(dw) = twoJz."""
    Ns = cfg.Ns
    h = _jz_hist(Ns, cfg.Norb)
    off = 2 * Ns
    dim = 0
    for pd in range(Ns + 1):
        pu = n - pd
        if pu < 0 or pu > Ns:
            continue
        for ld in range(-off, off + 1):
            lu = twoJz - (pu - pd) - ld
            if -off <= lu <= off:
                dim += int(h[pd, ld + off]) * int(h[pu, lu + off])
    return dim


def max_two_jz(cfg: EDConfig, n: int) -> int:
    """Largest |twoJz| kept for n electrons (ED_SETUP.f90:638-648)."""
    Ns, Nbath = cfg.Ns, cfg.Nbath
    if n == 0 or n == 2 * Ns:
        return 0
    shift = 0
    if n <= Nbath + 1:
        shift = Nbath - n + 1
    if n >= 2 * Ns - Nbath:
        shift = Nbath - 2 * Ns + n + 1
    return 5 + 5 * Nbath - abs(n - Ns) - 2 * shift


def sector_dim(cfg: EDConfig, q1: int, q2: int = 0) -> int:
    Ns = cfg.Ns
    if cfg.ed_mode == "nonsu2" and cfg.Jz_basis:
        return sector_dim_jz(cfg, q1, q2)
    if cfg.ed_mode == "normal":
        return binomial(Ns, q1) * binomial(Ns, q2)
    if cfg.ed_mode == "superc":
        # count of (nup, ndw) with nup - ndw = sz
        return sum(binomial(Ns, ndw + q1) * binomial(Ns, ndw) for ndw in range(Ns + 1))
    return binomial(2 * Ns, q1)


_POINTERS: Dict[tuple, List[Sector]] = {}


def setup_pointers(cfg: EDConfig) -> List[Sector]:
    """Sector list in reference ``isector`` order (memoised per structure)."""
    key = (cfg.ed_mode, cfg.Ns, cfg.Norb, cfg.Nbath, bool(cfg.Jz_basis and cfg.ed_mode == "nonsu2"))
    if key not in _POINTERS:
        _POINTERS[key] = _setup_pointers(cfg)
    return list(_POINTERS[key])


def _setup_pointers(cfg: EDConfig) -> List[Sector]:
    Ns = cfg.Ns
    out: List[Sector] = []
    if cfg.ed_mode == "normal":
        for nup in range(Ns + 1):
            for ndw in range(Ns + 1):
                out.append(Sector(len(out) + 1, nup, ndw, sector_dim(cfg, nup, ndw)))
    elif cfg.ed_mode == "superc":
        for sz in range(-Ns, Ns + 1):
            out.append(Sector(len(out) + 1, sz, 0, sector_dim(cfg, sz)))
    elif cfg.Jz_basis:
        for n in range(2 * Ns + 1):                       # ED_SETUP.f90:637-664
            mx = max_two_jz(cfg, n)
            for k in range(mx + 1):
                tj = 0 if n in (0, 2 * Ns) else -mx + 2 * k
                out.append(Sector(len(out) + 1, n, tj, sector_dim_jz(cfg, n, tj)))
    else:
        for n in range(2 * Ns + 1):
            out.append(Sector(len(out) + 1, n, 0, sector_dim(cfg, n)))
    return out


def diag_sectors(cfg: EDConfig) -> List[Sector]:
    """The sectors ed_diag visits (ED_DIAG.f90:71-74): non-empty (Jz_basis
    lists empty (n, twoJz) sectors), |twoJz| <= 2*Jz_max_value if Jz_max."""
    out = []
    for s in setup_pointers(cfg):
        if s.dim == 0:
            continue
        if cfg.ed_mode == "nonsu2" and cfg.Jz_basis and cfg.Jz_max and abs(s.q2) > int(2 * cfg.Jz_max_value):
            continue
        out.append(s)
    return out


def get_sector(cfg: EDConfig) -> Dict[Tuple[int, int], Sector]:
    return {(s.q1, s.q2): s for s in setup_pointers(cfg)}


def _jz_target(cfg: EDConfig, sec: Sector, iorb: int, ispin: int, d: int):
    """getCsector_Jz / getCDGsector_Jz (ED_SETUP.f90:769-805): n+d electrons,
    twoJz + d*(2*Lzdiag(iorb) + Szdiag(ispin)); None (-1) if beyond maxtwoJz."""
    jn = sec.q1 + d
    if jn < 0 or jn > 2 * cfg.Ns:
        return None
    trgt = sec.q2 + d * (2 * LZDIAG[iorb] + SZDIAG[ispin])
    if abs(trgt) > max_two_jz(cfg, jn):
        return None
    return get_sector(cfg).get((jn, trgt))


def cdg_sector(cfg: EDConfig, sec: Sector, ispin: int, iorb: int = 0):
    """getCDGsector(ispin,isector) (ED_SETUP.f90:480-495 normal, :605-619 superc,
    :760-768 nonsu2; Jz_basis: getCDGsector_Jz(iorb,ispin,isector)); ``ispin``,
    ``iorb`` 0-based.  None where the reference stores 0 / -1."""
    Ns = cfg.Ns
    if cfg.ed_mode == "nonsu2" and cfg.Jz_basis:
        return _jz_target(cfg, sec, iorb, ispin, +1)
    if cfg.ed_mode == "normal":
        q = (sec.q1 + 1, sec.q2) if ispin == 0 else (sec.q1, sec.q2 + 1)
        return None if max(q) > Ns else get_sector(cfg)[q]
    if cfg.ed_mode == "superc":
        sz = sec.q1 + 1 if ispin == 0 else sec.q1 - 1
        return None if abs(sz) > Ns else get_sector(cfg)[(sz, 0)]
    n = sec.q1 + 1
    return None if n > 2 * Ns else get_sector(cfg)[(n, 0)]


def c_sector(cfg: EDConfig, sec: Sector, ispin: int, iorb: int = 0):
    """getCsector(ispin,isector) (ED_SETUP.f90:464-478 normal ...; Jz_basis:
    getCsector_Jz(iorb,ispin,isector))."""
    Ns = cfg.Ns
    if cfg.ed_mode == "nonsu2" and cfg.Jz_basis:
        return _jz_target(cfg, sec, iorb, ispin, -1)
    if cfg.ed_mode == "normal":
        q = (sec.q1 - 1, sec.q2) if ispin == 0 else (sec.q1, sec.q2 - 1)
        return None if min(q) < 0 else get_sector(cfg)[q]
    if cfg.ed_mode == "superc":
        sz = sec.q1 - 1 if ispin == 0 else sec.q1 + 1
        return None if abs(sz) > Ns else get_sector(cfg)[(sz, 0)]
    n = sec.q1 - 1
    return None if n < 0 else get_sector(cfg)[(n, 0)]
