"""Generate tests/golden/adversarial_probe.json: near-cut degenerate sectors
for the degeneracy probe of the device eigensolver (ed_lib.hip trlan_run /
probe_screen; reference call site ED_DIAG.f90:88-101, Neigen=6).

TEST INFRASTRUCTURE ONLY — run in the CPU container:
    python tests/golden/make_adversarial.py

Model: golden_configs.adv_config(ed) — configs[3] (Norb=2, Nbath=5) with the
second orbital's bath equal to the first's and impurity level `ed` on both
orbitals; sector (nup, ndw) = (1, 3), dim 2,640.  Each orbital's particle
number per spin is conserved (density-density interaction, orbital-diagonal
hybridisation; levels are [imp_0, imp_1, bath_0[0..4], bath_1[0..4]]), so H is
block diagonal in (n_0up, n_0dw) and the orbital swap maps block (a, b) onto
(1 - a, 3 - b): every level is an exact pair.  The second-lowest pairs of the
swap classes {(0,2), (1,1)} and {(0,1), (1,2)} cross near ed = 0.061; `ed` is
solved so that their gap is delta_rel * |E|.

Why this is adversarial: with Neigen = 6 the true lowest six are
[P1, P1, P2, P2, lo, lo].  A single-vector Krylov solve sees one direction of
each pair and returns [P1, P2, lo, hi, ...]; the probe recovers P1's and P2's
copies and then faces cut = hi - margin with the complement holding lo's
missed copy |delta| below hi — right under the cut — and hi's own copy just
above it (the two-level cluster straddles the cut).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "dmft-ed_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

from oracle.oracle import Oracle  # noqa: E402

from golden.golden_configs import ADV_SECTOR, adv_config  # noqa: E402

DELTAS = (-1e-8, -3e-9, -3e-10, 3e-10, 3e-9, 1e-8)
NKEEP = 10


def sector_H(ed):
    cfg = adv_config(ed)
    orc = Oracle(cfg)
    hmap = orc.build_sector(*ADV_SECTOR)
    rp, cols, vals = orc.build_csr(hmap)
    assert np.all(vals.imag == 0)
    H = sp.csr_matrix((vals.real, cols, rp), shape=(len(hmap), len(hmap)))
    return cfg, hmap, H


def block_keys(cfg, hmap):
    """(n_0up, n_0dw): orbital 0 = impurity level 0 + bath levels Norb..Norb+Nbath-1."""
    ns = cfg.Ns
    m0 = 1 | sum(1 << (cfg.Norb + k) for k in range(cfg.Nbath))
    up = hmap & ((1 << ns) - 1)
    dw = hmap >> ns
    pc = np.vectorize(lambda x: bin(int(x)).count("1"))
    return pc(up & m0) * 100 + pc(dw & m0)


def gap(ed):
    """E_2nd(block (0,2)) - E_2nd(block (0,1)) and the former."""
    cfg, hmap, H = sector_H(ed)
    key = block_keys(cfg, hmap)
    ev = {}
    for k in (1, 2):
        idx = np.where(key == k)[0]
        ev[k] = np.linalg.eigvalsh(H[idx][:, idx].toarray())
    return ev[2][1] - ev[1][1], ev[2][1]


def solve_ed(delta_rel, lo=0.05, hi=0.07):
    ga, _ = gap(lo)
    gb, _ = gap(hi)
    m = lo
    for _ in range(80):
        _, e = gap(m)
        tgt = delta_rel * abs(e)
        m = lo + (tgt - ga) * (hi - lo) / (gb - ga)
        gm, _ = gap(m)
        if abs(gm - tgt) <= 1e-4 * abs(tgt):
            return m, gm
        if (gm - tgt) * (ga - tgt) < 0:
            hi, gb = m, gm
        else:
            lo, ga = m, gm
    raise RuntimeError("no convergence")


def main():
    cases = []
    for d in DELTAS:
        ed, g = solve_ed(d)
        cfg, hmap, H = sector_H(ed)
        # block-diagonal check: no element between different (n_0up, n_0dw)
        key = block_keys(cfg, hmap)
        Hc = H.tocoo()
        assert np.all(key[Hc.row] == key[Hc.col])
        w = np.linalg.eigvalsh(H.toarray())[:NKEEP]
        e = abs(w[0])
        # exact pairs, and the crossing pair at the requested distance
        assert np.all(np.abs(w[0:NKEEP:2] - w[1:NKEEP:2]) < 1e-12 * e)
        assert abs((w[6] - w[4]) - abs(g)) < 1e-3 * abs(g) + 1e-13 * e
        cases.append({"ed": float(ed), "delta_rel": d, "gap": float(g), "eigenvalues": [float(x) for x in w]})
        print(f"delta_rel {d:+.0e}: ed = {ed!r}, gap {g:.3e}, E = {w[:8]}", flush=True)
    out = {"sector": list(ADV_SECTOR), "dim": int(H.shape[0]), "neigen": 6, "cases": cases}
    with open(os.path.join(HERE, "adversarial_probe.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
