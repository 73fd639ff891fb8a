"""Symmetry-sector bookkeeping (host side, tiny tables).

Mirrors ``setup_pointers_normal/superc/nonsu2`` (ED_SETUP.f90:372-808, Jz_basis=F)
and the sector dimension functions (ED_SETUP.f90:809-860).  Sector ids are the
reference's 1-based ``isector``.
"""
from __future__ import annotations

from dataclasses import dataclass
from math import comb
from typing import Dict, List, Tuple

from .params import EDConfig


@dataclass(frozen=True)
class Sector:
    isector: int       # 1-based, reference order
    q1: int            # nup | sz | n
    q2: int            # ndw | 0  | 0
    dim: int


def binomial(n1: int, n2: int) -> int:
    """ED_SETUP.f90:1283-1300 (exact integer version; identical for n1 <= 32)."""
    if n2 < 0:
        return 0
    return comb(n1, n2) if n2 <= n1 else 0


def sector_dim(cfg: EDConfig, q1: int, q2: int = 0) -> int:
    Ns = cfg.Ns
    if cfg.ed_mode == "normal":
        return binomial(Ns, q1) * binomial(Ns, q2)
    if cfg.ed_mode == "superc":
        # count of (nup, ndw) with nup - ndw = sz
        return sum(binomial(Ns, ndw + q1) * binomial(Ns, ndw) for ndw in range(Ns + 1))
    return binomial(2 * Ns, q1)


def setup_pointers(cfg: EDConfig) -> List[Sector]:
    """Sector list in reference ``isector`` order."""
    Ns = cfg.Ns
    out: List[Sector] = []
    if cfg.ed_mode == "normal":
        for nup in range(Ns + 1):
            for ndw in range(Ns + 1):
                out.append(Sector(len(out) + 1, nup, ndw, sector_dim(cfg, nup, ndw)))
    elif cfg.ed_mode == "superc":
        for sz in range(-Ns, Ns + 1):
            out.append(Sector(len(out) + 1, sz, 0, sector_dim(cfg, sz)))
    else:
        for n in range(2 * Ns + 1):
            out.append(Sector(len(out) + 1, n, 0, sector_dim(cfg, n)))
    return out


def get_sector(cfg: EDConfig) -> Dict[Tuple[int, int], Sector]:
    return {(s.q1, s.q2): s for s in setup_pointers(cfg)}


def cdg_sector(cfg: EDConfig, sec: Sector, ispin: int):
    """getCDGsector(ispin,isector) (ED_SETUP.f90:480-495 normal, :605-619 superc,
    :760-768 nonsu2); ``ispin`` 0-based.  None where the reference stores 0."""
    Ns = cfg.Ns
    if cfg.ed_mode == "normal":
        q = (sec.q1 + 1, sec.q2) if ispin == 0 else (sec.q1, sec.q2 + 1)
        return None if max(q) > Ns else get_sector(cfg)[q]
    if cfg.ed_mode == "superc":
        sz = sec.q1 + 1 if ispin == 0 else sec.q1 - 1
        return None if abs(sz) > Ns else get_sector(cfg)[(sz, 0)]
    n = sec.q1 + 1
    return None if n > 2 * Ns else get_sector(cfg)[(n, 0)]


def c_sector(cfg: EDConfig, sec: Sector, ispin: int):
    """getCsector(ispin,isector) (ED_SETUP.f90:464-478 normal ...)."""
    Ns = cfg.Ns
    if cfg.ed_mode == "normal":
        q = (sec.q1 - 1, sec.q2) if ispin == 0 else (sec.q1, sec.q2 - 1)
        return None if min(q) < 0 else get_sector(cfg)[q]
    if cfg.ed_mode == "superc":
        sz = sec.q1 - 1 if ispin == 0 else sec.q1 + 1
        return None if abs(sz) > Ns else get_sector(cfg)[(sz, 0)]
    n = sec.q1 - 1
    return None if n < 0 else get_sector(cfg)[(n, 0)]
