"""The degeneracy probe's screening decision (probe_screen, ed_lib.hip) in a
numpy restatement, on the adversarial near-cut sectors of
tests/golden/adversarial_probe.json (make_adversarial.py; ED_DIAG.f90:88-101
Neigen=6).

The screen runs a plain Lanczos recurrence on the orthogonal complement of
the locked (found) eigenvectors — orthogonalised against the locked columns
and the two-column window only, as on the device — and every 10 steps forms
the lowest Ritz value theta of the tridiagonal and its residual bound
r = |beta_k s_k|.  It answers "below" when theta < cut (a certificate: a Ritz
value is a Rayleigh quotient, so >= the complement's lowest eigenvalue),
"none" when theta is converged to 1e-5 AND theta - r > cut (round 6), else
"undecided" after 400 steps.  cut = ev[5] - 1e-11 |ev[5]|.

Situation tested: the last probe round of a single-vector solve that missed
one copy of the pair `lo` whose partner pair `hi` lies |delta| = 1.8e-9 ..
6e-8 above it: locked = [P1, P1, P2, P2, lo, hi], the complement holds lo's
missed copy just under the cut and hi's copy just above it.  The screen must
flag it; with every true vector locked it must not.  The round-5 rule (a
1e-9 margin, "none" on the residual interval alone after 30 steps) answers
"none" on the 3e-10 cases, i.e. it would return hi in place of lo: 2.8e-10
of |E0| off, beyond the 1e-10 bar.
"""
import json
import os

import numpy as np
import pytest
import scipy.sparse as sp

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def screen(H, locked, cut, rule, tol=1e-5, maxsteps=400, chunk=10, seed=1):
    n = H.shape[0]
    rng = np.random.default_rng(seed)
    v = rng.uniform(-1.0, 1.0, n)
    v -= locked @ (locked.T @ v)
    v /= np.linalg.norm(v)
    vp = np.zeros(n)
    b = 0.0
    al, be = [], []
    for k in range(maxsteps):
        w = H @ v - b * vp
        w -= locked @ (locked.T @ w)
        a = v @ w
        w -= a * v
        w -= (vp @ w) * vp
        b = np.linalg.norm(w)
        al.append(a)
        be.append(b)
        vp, v = v, w / b
        if (k + 1) % chunk:
            continue
        T = np.diag(al) + np.diag(be[:-1], 1) + np.diag(be[:-1], -1)
        e, Z = np.linalg.eigh(T)
        theta, r = e[0], abs(be[-1] * Z[-1, 0])
        if theta < cut:
            return "below"
        conv = r <= tol * max(3.6e-11, abs(theta))
        if rule == "r6" and conv and theta - r > cut:
            return "none"
        if rule == "r5" and (conv or (k + 1 >= 30 and theta - r > cut)):
            return "none"
    return "undecided"


@pytest.mark.parametrize("case", [0, 2, 3, 5], ids=["-1e-8", "-3e-10", "+3e-10", "+1e-8"])
def test_screen_flags_near_cut_missed_copy(case):
    from golden.golden_configs import ADV_SECTOR, adv_config
    from oracle.oracle import Oracle

    with open(os.path.join(GOLD, "adversarial_probe.json")) as fh:
        c = json.load(fh)["cases"][case]
    orc = Oracle(adv_config(c["ed"]))
    hmap = orc.build_sector(*ADV_SECTOR)
    rp, cols, vals = orc.build_csr(hmap)
    H = sp.csr_matrix((vals.real, cols, rp), shape=(len(hmap), len(hmap)))
    w, X = np.linalg.eigh(H.toarray())
    np.testing.assert_allclose(w[:10], c["eigenvalues"], rtol=0, atol=1e-12 * abs(w[0]))
    # last probe round of a solve that missed lo's second copy (index 5)
    found = X[:, [0, 1, 2, 3, 4, 6]]
    hi = w[6]
    assert screen(H, found, hi - 1e-11 * abs(hi), "r6") == "below"
    # every true vector locked: nothing below the cut
    assert screen(H, X[:, :6], w[5] - 1e-11 * abs(w[5]), "r6") != "below"
    # the round-5 rule and margin on the same complement
    r5 = screen(H, found, hi - 1e-9 * abs(hi), "r5")
    if abs(c["delta_rel"]) < 1e-9:
        assert r5 == "none"     # the copy sits inside the old margin: missed
