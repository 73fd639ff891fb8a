"""Independent second-quantised construction of the impurity Hamiltonian.

TEST INFRASTRUCTURE ONLY.  Builds H in the full Fock space of 2*Ns levels from
Jordan-Wigner matrices made by Kronecker products (no popcount sign logic, no
reference loop structure) and written as an operator sum:

  H = sum_ab h_ab c+_a c_b  (impHloc incl. nonSU2 spin flips, -xmu n_imp)
    + U n_up n_dw + Ust(...) + (Ust-Jh)(...) + Hartree terms   (ED_HAMILTONIAN/stored/Hint.f90)
    + Jx sum_{o!=q} c+_{o up} c+_{q dw} c_{o dw} c_{q up}
    + Jp sum_{o!=q} c+_{o up} c+_{o dw} c_{q dw} c_{q up}
    + sum e_k n_k  |  replica  sum_k h_k[ss'oo'] c+ c        (Hbath.f90)
    + d (c+_{k up} c+_{k dw} + c_{k dw} c_{k up})             (superc)
    + conj(V) c+_imp c_bath + V c+_bath c_imp                (Himp_bath.f90)
    + u (c+_{o up} c_{k dw} + h.c.) ...                      (nonSU2 spin flips)

and restricted to a sector's states.  It pins the oracle's element generator
(signs, conjugation convention, term set) by physics rather than by code
reading.  Only for tiny systems (2*Ns <= 14).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def _ops(nlev):
    """Annihilators c_p, p = bit p of the state integer (bit 0 = level 1)."""
    a = sp.csr_matrix(np.array([[0.0, 1.0], [0.0, 0.0]]))  # |1> -> |0> in basis (|0>,|1>)
    z = sp.csr_matrix(np.diag([1.0, -1.0]))
    eye = sp.identity(2, format="csr")
    ops = []
    for p in range(nlev):
        # kron ordering: the LAST factor is bit 0.  Bits above p: identity;
        # bit p: a; bits below p: Z (Jordan-Wigner string over lower levels).
        m = None
        for b in range(nlev - 1, -1, -1):
            f = eye if b > p else (a if b == p else z)
            m = f if m is None else sp.kron(m, f, format="csr")
        ops.append(m.astype(np.complex128))
    return ops


def full_hamiltonian(cfg):
    Ns, No, Nb = cfg.Ns, cfg.Norb, cfg.Nbath
    nlev = 2 * Ns
    c = _ops(nlev)
    cd = [m.getH() for m in c]
    n = [cd[p] @ c[p] for p in range(nlev)]
    dim = 2 ** nlev
    H = sp.csr_matrix((dim, dim), dtype=np.complex128)
    S = cfg.Nspin - 1

    def lev_imp(o, s):
        return o + s * Ns

    if cfg.bath_type == "hybrid":
        def lev_bath(o, k, s):
            return No + k + s * Ns
    elif cfg.bath_type == "replica":
        def lev_bath(o, k, s):
            return o + (k + 1) * No + s * Ns
    else:
        def lev_bath(o, k, s):
            return No + o * Nb + k + s * Ns

    h = cfg.impHloc
    spins = [(0, 0), (1, S)]  # (spin index in levels, spin index in arrays)
    # impurity one-body (same spin)
    for sl, sa in spins:
        for o in range(No):
            for q in range(No):
                if h[sa, sa, o, q] != 0:
                    H = H + h[sa, sa, o, q] * (cd[lev_imp(o, sl)] @ c[lev_imp(q, sl)])
    if cfg.ed_mode == "nonsu2":
        for si in range(2):
            sj = 1 - si
            for o in range(No):
                for q in range(No):
                    if h[si, sj, o, q] != 0:
                        H = H + h[si, sj, o, q] * (cd[lev_imp(o, si)] @ c[lev_imp(q, sj)])
    nimp = sum(n[lev_imp(o, s)] for o in range(No) for s in (0, 1))
    H = H - cfg.xmu * nimp
    # interaction
    U, Ust, Jh = cfg.Uloc, cfg.Ust, cfg.Jh
    nu = [n[lev_imp(o, 0)] for o in range(No)]
    nd = [n[lev_imp(o, 1)] for o in range(No)]
    for o in range(No):
        H = H + U[o] * (nu[o] @ nd[o])
    for o in range(No):
        for q in range(o + 1, No):
            H = H + Ust * (nu[o] @ nd[q] + nu[q] @ nd[o])
            H = H + (Ust - Jh) * (nu[o] @ nu[q] + nd[o] @ nd[q])
    if cfg.hfmode:
        I = sp.identity(dim, format="csr", dtype=np.complex128)
        for o in range(No):
            H = H - 0.5 * U[o] * (nu[o] + nd[o]) + 0.25 * U[o] * I
        for o in range(No):
            for q in range(o + 1, No):
                ntot = nu[o] + nd[o] + nu[q] + nd[q]
                H = H - 0.5 * Ust * ntot + 0.25 * Ust * I
                H = H - 0.5 * (Ust - Jh) * ntot + 0.25 * (Ust - Jh) * I
    if No > 1 and (cfg.Jx != 0 or cfg.Jp != 0):
        for o in range(No):
            for q in range(No):
                if o == q:
                    continue
                H = H + cfg.Jx * (cd[lev_imp(o, 0)] @ cd[lev_imp(q, 1)] @ c[lev_imp(o, 1)] @ c[lev_imp(q, 0)])
                H = H + cfg.Jp * (cd[lev_imp(o, 0)] @ cd[lev_imp(o, 1)] @ c[lev_imp(q, 1)] @ c[lev_imp(q, 0)])
    b = cfg.bath
    if cfg.bath_type != "replica":
        ne = b.e.shape[1]
        for sl, sa in spins:
            for o in range(ne):
                for k in range(Nb):
                    H = H + b.e[sa, o, k] * n[lev_bath(o, k, sl)]
        for sl, sa in spins:
            for o in range(No):
                for k in range(Nb):
                    V = b.v[sa, o, k]
                    if V != 0:
                        H = H + np.conj(V) * (cd[lev_imp(o, sl)] @ c[lev_bath(o, k, sl)])
                        H = H + V * (cd[lev_bath(o, k, sl)] @ c[lev_imp(o, sl)])
        if cfg.ed_mode == "nonsu2":
            for o in range(No):
                for k in range(Nb):
                    u1, u2 = b.u[0, o, k], b.u[S, o, k]
                    # imp up <-> bath dw (u(1)), imp dw <-> bath up (u(Nspin))
                    H = H + u1 * (cd[lev_bath(o, k, 1)] @ c[lev_imp(o, 0)] + cd[lev_imp(o, 0)] @ c[lev_bath(o, k, 1)])
                    H = H + u2 * (cd[lev_bath(o, k, 0)] @ c[lev_imp(o, 1)] + cd[lev_imp(o, 1)] @ c[lev_bath(o, k, 0)])
        if cfg.ed_mode == "superc":
            for o in range(ne):
                for k in range(Nb):
                    d = b.d[0, o, k]
                    up, dw = lev_bath(o, k, 0), lev_bath(o, k, 1)
                    H = H + d * (cd[up] @ cd[dw] + c[dw] @ c[up])
    else:
        for k in range(Nb):
            for sl, sa in spins:
                for o in range(No):
                    for q in range(No):
                        if b.h[sa, sa, o, q, k] != 0:
                            H = H + b.h[sa, sa, o, q, k] * (cd[lev_bath(o, k, sl)] @ c[lev_bath(q, k, sl)])
            if cfg.ed_mode == "nonsu2":
                for si in range(2):
                    for o in range(No):
                        for q in range(No):
                            if b.h[si, 1 - si, o, q, k] != 0:
                                H = H + b.h[si, 1 - si, o, q, k] * (cd[lev_bath(o, k, si)] @ c[lev_bath(q, k, 1 - si)])
            vr = b.vr[k]
            if vr != 0:
                for sl, sa in spins:
                    for o in range(No):
                        H = H + np.conj(vr) * (cd[lev_imp(o, sl)] @ c[lev_bath(o, k, sl)])
                        H = H + vr * (cd[lev_bath(o, k, sl)] @ c[lev_imp(o, sl)])
    return H.tocsr()


def sector_matrix(cfg, hmap):
    H = full_hamiltonian(cfg)
    idx = np.asarray(hmap, dtype=np.int64)
    return H[idx][:, idx].toarray()
