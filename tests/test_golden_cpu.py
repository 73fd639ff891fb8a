"""The committed configs[3] / configs[4] fixtures (tests/golden/make_golden.py)
checked on CPU: pinned to the survey's reference-run values where they
overlap, internally consistent, and reproduced by the oracle on a sample of
sectors (the full regeneration takes minutes: `python tests/golden/make_golden.py`)."""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    with open(os.path.join(GOLD, name)) as fh:
        return json.load(fh)


def test_c5_flat_e0_matches_survey_pin():
    """configs[4] flat bath: E0 = -7.56253778 measured on the reference's own
    hot-path Fortran during the survey (survey_pins.json)."""
    pins = _load("survey_pins.json")
    pin = [p for p in pins["sectors"] if p["name"].startswith("c5")][0]
    d = _load("c5_diag_flat.json")
    assert abs(d["E0"] - pin["e0"]) < 5e-9


@pytest.mark.parametrize("bath", ["flat", "random"])
def test_c4_fixture_consistent(bath):
    from edgpu.diag import DiagOptions, SectorResult, state_list
    from edgpu.sectors import diag_sectors
    from golden.golden_configs import c4_config

    d = _load(f"c4_diag_{bath}.json")
    secs = diag_sectors(c4_config(bath))
    assert len(secs) == len(d["sectors"]) == 169
    for s in secs:
        g = d["sectors"][str(s.isector)]
        assert g["q"] == [s.q1, s.q2] and g["dim"] == s.dim
        assert len(g["eigenvalues"]) == min(s.dim, 6)
        assert np.all(np.diff(g["eigenvalues"]) >= 0)
    # spin symmetry of the normal-mode model: (nup,ndw) and (ndw,nup) share a spectrum
    by_q = {tuple(g["q"]): np.asarray(g["eigenvalues"]) for g in d["sectors"].values()}
    for (a, b), ev in by_q.items():
        np.testing.assert_allclose(ev, by_q[(b, a)], rtol=0, atol=1e-10)
    # the state list replays from the per-sector eigenvalues
    res = [SectorResult(int(k), tuple(g["q"]), g["dim"], np.asarray(g["eigenvalues"]),
                        len(g["eigenvalues"])) for k, g in d["sectors"].items()]
    sl = state_list(res, DiagOptions())
    assert sl.sectors == d["states"]["sectors"] and sl.energies == d["states"]["energies"]


@pytest.mark.parametrize("bath", ["flat", "random"])
def test_c4_fixture_reproduced_by_oracle_sample(bath):
    """Regenerate a few sectors (dense and ARPACK branches) from the oracle."""
    from edgpu.sectors import diag_sectors
    from golden.golden_configs import c4_config
    from golden.make_golden import _solve

    d = _load(f"c4_diag_{bath}.json")
    cfg = c4_config(bath)
    secs = {s.isector: s for s in diag_sectors(cfg)}
    sample = [k for k, g in d["sectors"].items() if g["dim"] <= 256][:3] + \
             [k for k, g in d["sectors"].items() if 256 < g["dim"] <= 3000][:3]
    for k in sample:
        _, _, _, w, _, _ = _solve((cfg, secs[int(k)], False))
        np.testing.assert_allclose(w, d["sectors"][k]["eigenvalues"], rtol=0, atol=1e-11)


def test_c5_gf_fixture_shape():
    for bath in ("flat", "random"):
        g = np.load(os.path.join(GOLD, f"c5_gf_{bath}.npz"))
        assert g["Gm"].shape == (2, 2, 1, 1, 100) and g["iw_index"][1] == 50
        # causality: Im G_ss(iw_n) < 0 on the positive Matsubara axis
        assert np.all(g["Gm"][0, 0, 0, 0].imag < 0) and np.all(g["Gm"][1, 1, 0, 0].imag < 0)


@pytest.mark.parametrize("case", [0, 3])
def test_adversarial_probe_fixture(case):
    """tests/golden/adversarial_probe.json: the dense spectrum of the tuned
    sector is reproduced from the oracle's CSR, every level is an exact pair,
    and the pairs at positions 4-5 and 6-7 lie the fixture's gap apart."""
    import scipy.sparse as sp

    from golden.golden_configs import ADV_SECTOR, adv_config
    from oracle.oracle import Oracle

    d = _load("adversarial_probe.json")
    c = d["cases"][case]
    orc = Oracle(adv_config(c["ed"]))
    hmap = orc.build_sector(*ADV_SECTOR)
    rp, cols, vals = orc.build_csr(hmap)
    H = sp.csr_matrix((vals.real, cols, rp), shape=(len(hmap), len(hmap)))
    w = np.linalg.eigvalsh(H.toarray())[:10]
    ref = np.asarray(c["eigenvalues"])
    e = abs(ref[0])
    assert np.max(np.abs(w - ref)) < 1e-12 * e
    assert np.max(np.abs(ref[0::2] - ref[1::2])) < 1e-12 * e
    assert abs((ref[6] - ref[4]) - abs(c["gap"])) < 1e-3 * abs(c["gap"])
    assert abs(c["gap"]) <= 1.01e-8 * e
