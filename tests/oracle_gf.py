"""CPU Green's function from the oracle pieces (test infrastructure): seeds by
the reference's vvinit loop (ED_GF_NORMAL.f90:159-174, binary search on the
target H%map), tridiagonalisation by the oracle's lanczos_plain_tridiag_c,
poles as add_to_lanczos_gf_normal (:580-632)."""
import numpy as np

from edgpu.diag import to_host
from edgpu.gf import matsubara, realaxis
from edgpu.sectors import c_sector, cdg_sector, setup_pointers
from oracle.oracle import Oracle, lanc_tridiag


def tridiag_poles(alfa, beta, n):
    """Oracle poles for the normal-mode GF: LAPACK dstev (the eigh of
    add_to_lanczos_gf_normal, ED_GF_NORMAL.f90:612-618), full eigenvectors."""
    from scipy.linalg import eigh_tridiagonal

    if n == 1:
        return np.array([alfa[0]]), np.array([1.0])
    w, z = eigh_tridiagonal(alfa[:n], beta[1:n], lapack_driver="stev")
    return w, z[0, :] ** 2


def _popcount_below(states, level):
    m = states & np.uint32((1 << level) - 1)
    c = np.zeros_like(m, dtype=np.int64)
    for b in range(level):
        c += (m >> np.uint32(b)) & np.uint32(1)
    return c


def seed(orc, hmap_i, jsec, op, level, vec):
    hmap_j = orc.build_sector(jsec.q1, jsec.q2)
    occ = (hmap_i >> np.uint32(level)) & np.uint32(1)
    sel = (occ == 0) if op == 1 else (occ == 1)
    st = hmap_i[sel]
    sg = 1.0 - 2.0 * (_popcount_below(st, level) % 2)
    tgt = st ^ np.uint32(1 << level)
    j = np.searchsorted(hmap_j, tgt)
    assert np.all(hmap_j[j] == tgt)
    v = np.zeros(len(hmap_j), dtype=np.complex128)
    v[j] = sg * vec[sel]
    return hmap_j, v


def build_gf_normal_oracle(cfg, states, gopt):
    orc = Oracle(cfg)
    Ns, No, Nsp = cfg.Ns, cfg.Norb, cfg.Nspin
    wm = matsubara(gopt.beta, gopt.Lmats)
    wr = realaxis(gopt.wini, gopt.wfin, gopt.Lreal)
    Gm = np.zeros((Nsp, Nsp, No, No, gopt.Lmats), dtype=np.complex128)
    Gr = np.zeros((Nsp, Nsp, No, No, gopt.Lreal), dtype=np.complex128)
    secs = setup_pointers(cfg)
    zeta = float(len(states.energies))
    rec = []
    for ispin in range(Nsp):
        for iorb in range(No):
            isite = iorb + ispin * Ns
            for e_i, isec, vec in zip(states.energies, states.sectors, map(to_host, states.vectors)):
                sec = secs[isec - 1]
                hmap_i = orc.build_sector(sec.q1, sec.q2)
                for op, isign, jsec in ((1, 1, cdg_sector(cfg, sec, ispin)), (0, -1, c_sector(cfg, sec, ispin))):
                    if jsec is None:
                        continue
                    hmap_j, v = seed(orc, hmap_i, jsec, op, isite, vec)
                    norm2 = float(np.vdot(v, v).real)
                    if norm2 == 0.0:
                        continue
                    v = v / np.sqrt(norm2)
                    csr = orc.build_csr(hmap_j)
                    nlanc = min(len(hmap_j), gopt.lanc_nGFiter)
                    a, b, n = lanc_tridiag(csr, v, nlanc, gopt.threshold)
                    E, z2 = tridiag_poles(a, b, nlanc)
                    rec.append(dict(ispin=ispin, iorb=iorb, isector=isec, op=op, norm2=norm2,
                                    alfa=a, beta=b, nlanc=n))
                    de = E - e_i
                    peso = norm2 / zeta * z2
                    Gm[ispin, ispin, iorb, iorb] += (peso[None] / ((1j * wm)[:, None] - isign * de[None])).sum(1)
                    Gr[ispin, ispin, iorb, iorb] += (peso[None] / ((wr + 1j * gopt.eps)[:, None] - isign * de[None])).sum(1)
    return Gm, Gr, rec


def seed_combo(orc, hmap_i, jsec, op, terms, vec):
    """sum_t coef_t op_{level_t}|vec> (ED_GF_NONSU2.f90 vvinit loops)."""
    v = None
    for level, coef in terms:
        hmap_j, w = seed(orc, hmap_i, jsec, op, level, vec)
        v = coef * w if v is None else v + coef * w
    return hmap_j, v


def build_gf_oracle(cfg, states, gopt):
    """build_gf_normal / build_gf_nonsu2 (normal bath) from oracle pieces;
    nonSU2 poles from the oracle's tql2 like add_to_lanczos_gf_nonsu2
    (ED_GF_NONSU2.f90:936)."""
    from oracle.oracle import tql2

    orc = Oracle(cfg)
    Ns, No, Nsp = cfg.Ns, cfg.Norb, cfg.Nspin
    wm = matsubara(gopt.beta, gopt.Lmats)
    wr = realaxis(gopt.wini, gopt.wfin, gopt.Lreal)
    Gm = np.zeros((Nsp, Nsp, No, No, gopt.Lmats), dtype=np.complex128)
    Gr = np.zeros((Nsp, Nsp, No, No, gopt.Lreal), dtype=np.complex128)
    secs = setup_pointers(cfg)
    zeta = float(len(states.energies))
    site = lambda o, s: o + s * Ns

    def channel(idx, specs):
        for e_i, isec, vec in zip(states.energies, states.sectors, map(to_host, states.vectors)):
            sec = secs[isec - 1]
            hmap_i = orc.build_sector(sec.q1, sec.q2)
            for op, isign, ispin, terms, weight in specs:
                jsec = cdg_sector(cfg, sec, ispin, idx[2]) if op == 1 else c_sector(cfg, sec, ispin, idx[2])
                if jsec is None:
                    continue
                hmap_j, v = seed_combo(orc, hmap_i, jsec, op, terms, vec.astype(np.complex128))
                norm2 = float(np.vdot(v, v).real)
                if norm2 == 0.0:
                    continue
                v = v / np.sqrt(norm2)
                csr = orc.build_csr(hmap_j)
                nlanc = min(len(hmap_j), gopt.lanc_nGFiter)
                a, b, n = lanc_tridiag(csr, v, nlanc, gopt.threshold)
                if cfg.ed_mode == "nonsu2":
                    E, Z, ierr = tql2(a[:nlanc], np.concatenate([[0.0], b[1:nlanc]]))
                    z2 = Z[0, :] ** 2
                else:
                    E, z2 = tridiag_poles(a, b, nlanc)
                de = E - e_i
                peso = weight * norm2 / zeta * z2
                Gm[idx] += (peso[None] / ((1j * wm)[:, None] - isign * de[None])).sum(1)
                Gr[idx] += (peso[None] / ((wr + 1j * gopt.eps)[:, None] - isign * de[None])).sum(1)

    for ispin in range(Nsp):
        for iorb in range(No):
            i = site(iorb, ispin)
            channel((ispin, ispin, iorb, iorb), [(1, 1, ispin, [(i, 1)], 1.0), (0, -1, ispin, [(i, 1)], 1.0)])
    if cfg.ed_mode == "nonsu2":
        pairs = [(s1, s2, o) for s1 in range(Nsp) for s2 in range(Nsp) for o in range(No) if s1 != s2
                 and (cfg.bath_type != "replica"      # dmft_bath%mask, ED_BATH/dmft_aux.f90:283-295
                      or abs(cfg.impHloc[s1, s2, o, o].real) > 1e-6 or abs(cfg.impHloc[s1, s2, o, o].imag) > 1e-6)]
        for ispin, jspin, iorb in pairs:
            i, j = site(iorb, ispin), site(iorb, jspin)
            channel((ispin, jspin, iorb, iorb), [
                (1, 1, ispin, [(i, 1), (j, 1)], 1.0), (0, -1, ispin, [(i, 1), (j, 1)], 1.0),
                (1, 1, ispin, [(i, 1), (j, 1j)], 1j), (0, -1, ispin, [(i, 1), (j, -1j)], 1j)])
        for ispin, jspin, iorb in pairs:
            for G in (Gm, Gr):
                G[ispin, jspin, iorb, iorb] = 0.5 * (G[ispin, jspin, iorb, iorb]
                                                     - (1 + 1j) * G[ispin, ispin, iorb, iorb]
                                                     - (1 + 1j) * G[jspin, jspin, iorb, iorb])
    return Gm, Gr


def oracle_job_runner(cfg, states, gopt, job, wm, wr, G_m, G_r, zeta):
    """edgpu.gf.build_gf job (one seed of one kept state) from oracle pieces,
    for the CPU (gloo) seed-farm tests."""
    from oracle.oracle import tql2

    comp, tag, k, (op, isign, ispin, terms, weight), sec, jsec = job
    orc = Oracle(cfg)
    hmap_i = orc.build_sector(sec.q1, sec.q2)
    hmap_j, v = seed_combo(orc, hmap_i, jsec, op, terms, np.asarray(to_host(states.vectors[k])).astype(np.complex128))
    norm2 = float(np.vdot(v, v).real)
    if norm2 == 0.0:
        return
    v = v / np.sqrt(norm2)
    nlanc = min(len(hmap_j), gopt.lanc_nGFiter)
    a, b, n = lanc_tridiag(orc.build_csr(hmap_j), v, nlanc, gopt.threshold)
    if cfg.ed_mode == "nonsu2":
        E, Z, ierr = tql2(a[:nlanc], np.concatenate([[0.0], b[1:nlanc]]))
        z2 = Z[0, :] ** 2
    else:
        E, z2 = tridiag_poles(a, b, nlanc)
    de = E - states.energies[k]
    peso = weight * norm2 / zeta * z2
    G_m += (peso[None] / ((1j * wm)[:, None] - isign * de[None])).sum(1)
    G_r += (peso[None] / ((wr + 1j * gopt.eps)[:, None] - isign * de[None])).sum(1)
