"""Generate the committed golden fixtures for BASELINE configs[3] and configs[4]
from the CPU oracle (oracle/ed_oracle.c: restated ED_SETUP build_sector,
ed_buildH_c, lanczos_plain_tridiag_c, tql2) and scipy.

TEST INFRASTRUCTURE ONLY — run in the CPU container, never on the GPU box:
    python tests/golden/make_golden.py [c4] [c5]

configs[3]  (ED_DIAG.f90:71-249, ed_hm_2bands_bethe): Norb=2, Nbath=5
  (Nlevels=24), Uloc=(2,2,0), Ust=1, Jh=0.5, flat bath and the
  bench's seeded random bath: for every one of the 169 (nup,ndw) sectors its
  Neigen = min(dim, 6) lowest eigenvalues with their multiplicities (dense
  LAPACK for dim <= 4096, else ARPACK eigsh of the lowest 12 to machine
  precision on the oracle's CSR, merged over the isospectral spin-partner
  sector; see _solve), and the T=0 state list (gs_threshold window,
  ED_DIAG.f90:224-235).
configs[4]  (ED_GF_NONSU2.f90:28-55): nonSU2, Norb=1, Nbath=6 (Nlevels=14),
  same baths: all 15 sectors' lowest eigenvalues, the state list, and the
  Green's function G(iw_n) (diagonal and spin-mixed components, 200-step
  Lanczos per seed, tql2 poles, Lmats=5000) from the oracle pipeline
  (tests/oracle_gf.py), thinned to every 50th Matsubara frequency.
"""
from __future__ import annotations

import json
import os
import sys
import time
from multiprocessing import Pool

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as sla

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "dmft-ed_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

from edgpu.diag import DiagOptions, SectorResult, lanczos_params, state_list  # noqa: E402
from edgpu.sectors import diag_sectors  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

from golden.golden_configs import C2_KW, C4_KW, C5_KW, SEED, c2_config, c4_config, c5_config  # noqa: E402

GF_THIN = 50


DENSE_MAX = 4096   # exact LAPACK spectrum up to this dimension
KEXTRA = 12        # ARPACK: the lowest 12 (multiplicities of the lowest 6 resolved)


def _solve(args):
    """One sector: its lowest eigenvalues from the oracle CSR — Neigen (with
    vectors if asked) for the state list, and up to KEXTRA for the
    multiplicity check.  A single-vector Krylov method (ARPACK, the device
    thick-restart Lanczos) sees one direction of a degenerate eigenspace and
    finds the other copies only through rounding, so the fixture resolves
    multiplicities: exact dense spectra up to DENSE_MAX, else the lowest 12 by
    ARPACK merged across the isospectral (nup,ndw)/(ndw,nup) pair (make_c4)."""
    cfg, sec, keep = args[:3]
    kx = args[3] if len(args) > 3 else 0
    opt = DiagOptions()
    orc = Oracle(cfg)
    hmap = orc.build_sector(sec.q1, sec.q2)
    rp, cols, vals = orc.build_csr(hmap)
    dim = len(hmap)
    neigen, _, _ = lanczos_params(dim, opt)
    real = cfg.is_real()
    A = sp.csr_matrix((vals.real if real else vals, cols, rp), shape=(dim, dim))
    if neigen == dim or dim <= max(opt.lanc_dim_threshold, opt.mpi_size, DENSE_MAX if kx else 0):
        w, v = np.linalg.eigh(A.toarray())
        w = w[: max(neigen, kx)]
        return sec.isector, (sec.q1, sec.q2), dim, w, (v[:, :neigen] if keep else None), "dense"
    i = np.arange(1, dim + 1, dtype=np.float64)
    v0 = np.sin(i) if real else np.sin(i) + 1j * np.cos(3.0 * i)
    k = max(neigen, kx)
    w, v = sla.eigsh(A, k=k, which="SA", tol=0.0, v0=v0, ncv=min(dim, max(2 * k + 1, 24, 3 * k)))
    o = np.argsort(w)
    return sec.isector, (sec.q1, sec.q2), dim, w[o], (v[:, o[:neigen]] if keep else None), "eigsh"


def diag_all(cfg, keep=False, procs=6, kx=0):
    secs = diag_sectors(cfg)
    order = sorted(secs, key=lambda s: -s.dim)
    with Pool(procs) as pool:
        out = pool.map(_solve, [(cfg, s, keep, kx) for s in order], chunksize=1)
    opt = DiagOptions()
    res = [SectorResult(k, q, d, w, lanczos_params(d, opt)[0], v, m) for (k, q, d, w, v, m) in out]
    return sorted(res, key=lambda r: r.isector)


def merge_spin_partners(res, tol=1e-9):
    """Normal mode with spin-independent parameters: (nup,ndw) and (ndw,nup)
    are isospectral.  Each eigenvalue cluster gets the larger multiplicity the
    two ARPACK runs found; the merged list replaces both sectors' lowest."""
    by_q = {r.q: r for r in res}
    for r in res:
        p = by_q[(r.q[1], r.q[0])]
        if r.method == "dense" or p is r:
            continue
        vals = []
        a, b = list(r.eigenvalues), list(p.eigenvalues)
        while a or b:
            x = min(a[0] if a else np.inf, b[0] if b else np.inf)
            ca = [y for y in a if abs(y - x) <= tol]
            cb = [y for y in b if abs(y - x) <= tol]
            vals += ca if len(ca) >= len(cb) else cb
            a = [y for y in a if abs(y - x) > tol]
            b = [y for y in b if abs(y - x) > tol]
        r.merged = np.asarray(vals)
    for r in res:
        if hasattr(r, "merged"):
            r.eigenvalues = r.merged[: len(r.eigenvalues)]
    return res


def _sector_table(res):
    return {str(r.isector): {"q": list(r.q), "dim": r.dim, "method": r.method,
                             "eigenvalues": [float(x) for x in r.eigenvalues[: r.neigen]],
                             "lowest": [float(x) for x in r.eigenvalues]} for r in res}


def make_c4():
    for bath in ("flat", "random"):
        t0 = time.time()
        cfg = c4_config(bath)
        res = merge_spin_partners(diag_all(cfg, kx=KEXTRA))
        sl = state_list(res, DiagOptions())
        out = {"config": {**{k: (list(v) if isinstance(v, tuple) else v) for k, v in C4_KW.items()},
                          "bath": bath, "seed": SEED},
               "source": "oracle CSR (ed_buildH_c restatement) + LAPACK eigh (dim<=4096) / ARPACK eigsh k=12 tol=0 merged over (nup,ndw)<->(ndw,nup)",
               "E0": sl.emin, "states": {"energies": sl.energies, "sectors": sl.sectors},
               "sectors": _sector_table(res)}
        path = os.path.join(HERE, f"c4_diag_{bath}.json")
        with open(path, "w") as fh:
            json.dump(out, fh, indent=0)
        print(f"c4 {bath}: {len(res)} sectors, E0={sl.emin:.12f}, states={sl.size} in {time.time()-t0:.1f}s",
              flush=True)


def make_c5():
    from edgpu.gf import GFOptions
    from oracle_gf import build_gf_oracle

    for bath in ("flat", "random"):
        t0 = time.time()
        cfg = c5_config(bath)
        res = diag_all(cfg, keep=True, kx=KEXTRA)
        sl = state_list(res, DiagOptions())
        gopt = GFOptions()
        Gm, _ = build_gf_oracle(cfg, sl, gopt)
        idx = np.arange(0, gopt.Lmats, GF_THIN)
        np.savez(os.path.join(HERE, f"c5_gf_{bath}.npz"), iw_index=idx, Gm=Gm[..., idx],
                 E0=np.float64(sl.emin), energies=np.asarray(sl.energies), sectors=np.asarray(sl.sectors),
                 beta=np.float64(gopt.beta), Lmats=np.int64(gopt.Lmats), nGFiter=np.int64(gopt.lanc_nGFiter))
        with open(os.path.join(HERE, f"c5_diag_{bath}.json"), "w") as fh:
            json.dump({"config": {**C5_KW, "bath": bath, "seed": SEED}, "E0": sl.emin,
                       "states": {"energies": sl.energies, "sectors": sl.sectors},
                       "sectors": _sector_table(res)}, fh, indent=0)
        print(f"c5 {bath}: E0={sl.emin:.12f} states={sl.size} |G(iw0)|={abs(Gm[0,0,0,0,0]):.6f} "
              f"in {time.time()-t0:.1f}s", flush=True)


def make_c2():
    """configs[1] sector (4,4) with the bench's random bath (seed SEED + rank
    for ranks 0..7): the ground-state energy the bench's timed 512-step
    Lanczos run must reproduce (oracle plain Lanczos, .repo/PLAIN_LANCZOS.f90
    :286-385, cross-checked by dense LAPACK)."""
    from oracle.oracle import lanc_eigh

    out = {}
    for rank in range(8):
        cfg = c2_config("random", SEED + rank)
        orc = Oracle(cfg)
        hmap = orc.build_sector(4, 4)
        csr = orc.build_csr(hmap)
        i = np.arange(1, len(hmap) + 1, dtype=np.float64)
        e_l, _, n = lanc_eigh(csr, np.sin(i) + 0j, 512, 1e-14)
        w = np.linalg.eigvalsh(sp.csr_matrix((csr[2].real, csr[1], csr[0])).toarray())
        assert abs(e_l - w[0]) < 1e-10 * abs(w[0]), (e_l, w[0])
        out[str(SEED + rank)] = {"E0": float(w[0]), "E0_lanczos": e_l, "lanczos_steps": n, "dim": len(hmap)}
        print(f"c2 seed {SEED + rank}: E0={w[0]:.12f}", flush=True)
    with open(os.path.join(HERE, "c2_e0.json"), "w") as fh:
        json.dump({"config": {**C2_KW, "bath": "random", "sector": [4, 4]}, "by_seed": out}, fh, indent=1)


if __name__ == "__main__":
    what = sys.argv[1:] or ["c2", "c5", "c4"]
    if "c2" in what:
        make_c2()
    if "c5" in what:
        make_c5()
    if "c4" in what:
        make_c4()
