"""Batched thick-restart Lanczos (ed_sectors_eigh_batch) against the
per-sector solver, the dense configs[3] fixtures and the adversarial
degeneracy fixture.

The batch runs trlan_run's algorithm (ED_DIAG.f90:145-167's sp_eigh
replacement) for many sectors at once: one workgroup per sector and one
launch per restart cycle up to 2,640 rows (ed_trlbatch.hpp), every step of
the larger ones in shared launches (ed_trlmulti.hpp); sectors it cannot
finish fall back to the per-sector path, so the results must meet the same
1e-10 bar either way.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
NEV, NCV = 6, 23


def _small_sectors(cfg, opt, lo=257, hi=15360):
    from edgpu.diag import batchable
    from edgpu.sectors import diag_sectors

    return [s for s in diag_sectors(cfg) if lo <= s.dim <= hi and batchable(cfg, s, opt)]


@pytest.mark.parametrize("bath", ["random", "flat"])
def test_batch_matches_fixture_and_single(bath):
    """Every configs[3] Lanczos sector of 495-14,520 rows in one batch call
    (up to 2,640 rows one workgroup each, the larger ones in lockstep):
    eigenvalues within 1e-10 of |E0| of the dense fixture, and of the
    per-sector solver (ed_sector_eigh); eigenvectors orthonormal with H v =
    w v; the random bath finishes (nearly) every sector inside the batch, the
    flat bath sends the sectors with a missed degenerate copy to the
    per-sector probe."""
    from edgpu.diag import DiagOptions, _start_vector, lanczos_params
    from edgpu.hamiltonian import Sector, eigh_batch
    from golden.golden_configs import c4_config

    with open(os.path.join(GOLD, f"c4_diag_{bath}.json")) as fh:
        gold = json.load(fh)
    cfg = c4_config(bath)
    opt = DiagOptions()
    secs = [s for s in _small_sectors(cfg, opt) if lanczos_params(s.dim, opt)[1] == 512]
    assert len(secs) > 20
    hs = [Sector(cfg, s.q1, s.q2, stored=True, real=True) for s in secs]
    try:
        res, nb = eigh_batch(hs, NEV, NCV, 512, 1e-12, [_start_vector(h.dim, False) for h in hs],
                             vectors=True, on_device=False)
        scale = abs(gold["E0"])
        worst, worst_single = 0.0, 0.0
        for s, h, (w, v, nconv, nhv) in zip(secs, hs, res):
            ref = np.asarray(gold["sectors"][str(s.isector)]["eigenvalues"][:NEV])
            worst = max(worst, float(np.max(np.abs(w - ref))) / scale)
            assert nconv == NEV and nhv > 0
            # eigenvectors: H v = w v to the solver's tolerance, orthonormal
            hv = np.stack([h.hxv(v[:, k]).real for k in range(NEV)], axis=1)
            r = np.abs(hv - v * w[None, :]).max()
            assert r < 1e-8 * max(1.0, float(np.abs(w).max())), (s.isector, r)
            np.testing.assert_allclose(v.T @ v, np.eye(NEV), atol=1e-10)
        for s, h, (w, _, _, _) in list(zip(secs, hs, res))[:: max(1, len(secs) // 8)]:
            w1, _, _, _ = h.eigh(neigen=NEV, ncv=NCV, maxit=512, tol=1e-12, v0=_start_vector(h.dim, False),
                                 vectors=False)
            worst_single = max(worst_single, float(np.max(np.abs(w - w1))) / scale)
    finally:
        for h in hs:
            h.close()
    print(f"c4 {bath}: {len(secs)} sectors, {nb} finished in the batch, worst vs fixture {worst:.1e}, "
          f"vs single {worst_single:.1e}")
    assert worst < 1e-10 and worst_single < 1e-10
    if bath == "random":
        assert nb >= len(secs) - 2


def test_batch_adversarial_and_lockstep():
    """The six adversarial near-cut degenerate sectors (tests/golden/
    make_adversarial.py) in one batch (one workgroup each), together with a
    sector beyond the one-workgroup size (the lockstep path): all within 1e-10
    of the dense spectra / the per-sector solve."""
    from edgpu.hamiltonian import Sector, eigh_batch
    from golden.golden_configs import ADV_SECTOR, adv_config, c4_config

    with open(os.path.join(GOLD, "adversarial_probe.json")) as fh:
        fx = json.load(fh)
    hs = [Sector(adv_config(c["ed"]), *ADV_SECTOR, stored=True, real=True) for c in fx["cases"]]
    big = Sector(c4_config("random"), 3, 4, stored=True, real=True)   # 32,670 rows
    try:
        assert big.dim > 2640
        res, nb = eigh_batch(hs + [big], NEV, NCV, 512, 1e-12, None, vectors=False)
        for c, (w, _, nconv, _) in zip(fx["cases"], res):
            ref = np.asarray(c["eigenvalues"][:NEV])
            scale = max(1.0, float(np.max(np.abs(ref))))
            assert nconv == NEV
            assert float(np.max(np.abs(w - ref))) / scale < 1e-10, (c["delta_rel"], w - ref)
        w1, _, _, _ = big.eigh(neigen=NEV, ncv=NCV, maxit=512, tol=1e-12, vectors=False)
        np.testing.assert_allclose(res[-1][0], w1, rtol=0, atol=1e-10 * abs(w1[0]))
        assert nb >= 1    # (the lockstep sector; the adversarial ones go on to the probe)
    finally:
        for h in hs + [big]:
            h.close()
    print(f"adversarial + lockstep: {nb} of {len(hs) + 1} finished in the batch")


def test_farm_batch_on_and_off_agree():
    """farm_diag with the batch (default: every Lanczos sector, one workgroup
    each up to 2,640 rows, the rest in lockstep) and without
    (batch_max_dim=0): identical state lists, sector eigenvalues within 1e-10
    of |E0|."""
    from edgpu.diag import DiagOptions
    from edgpu.farm import farm_diag
    from golden.golden_configs import c4_config

    cfg = c4_config("random")
    a = farm_diag(cfg, DiagOptions())
    b = farm_diag(cfg, DiagOptions(batch_max_dim=0))
    scale = abs(a.states.emin)
    for k, ev in a.eigenvalues.items():
        assert np.max(np.abs(np.asarray(ev) - np.asarray(b.eigenvalues[k]))) < 1e-10 * scale, k
    assert a.states.sectors == b.states.sectors
