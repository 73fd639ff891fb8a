"""BASELINE configs[3] and configs[4] at their full size on the GPU against the
committed oracle fixtures (tests/golden/make_golden.py).

configs[3]: all 169 (nup,ndw) sectors of Norb=2 Nbath=5 through ed_diag's
default path (dense for dim <= 256, device thick-restart Lanczos for the 6
lowest otherwise; ED_DIAG.f90:71-249): every sector's eigenvalues and the
T=0 state list within 1e-10 (north_star Ritz-value bar).
configs[4]: nonSU2 Norb=1 Nbath=6: ground state over all sectors and the
Green's function (12 seeds, 200 Lanczos steps each, L=5000;
ED_GF_NONSU2.f90:28-55) on every 50th Matsubara frequency within 1e-10
relative (north_star G(iw) bar).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    with open(os.path.join(GOLD, name)) as fh:
        return json.load(fh)


@pytest.mark.parametrize("bath,kopts", [("flat", ()), ("random", ()), ("random", ("trlan_unfused",)),
                                        ("random", ("trlan_nolocal", "trlan_nosolo"))],
                         ids=["flat", "random", "random-unfused", "random-plain-step"])
def test_c4_all_sectors_match_fixture(bath, kopts):
    """All 169 configs[3] sectors through the farm against the dense fixture
    (1e-10 of |E0|); also with the always-two-pass CGS2 (ED_OPT_TRLAN_UNFUSED,
    DiagOptions.kernel_options) against the default DGKS-conditional pass."""
    from edgpu.diag import DiagOptions
    from edgpu.farm import farm_diag
    from golden.golden_configs import c4_config

    gold = _load(f"c4_diag_{bath}.json")
    cfg = c4_config(bath)
    res = farm_diag(cfg, DiagOptions(kernel_options=kopts))
    assert len(res.eigenvalues) == len(gold["sectors"]) == 169
    scale = abs(gold["E0"])
    worst = 0.0
    for k, g in gold["sectors"].items():
        ev = np.asarray(res.eigenvalues[int(k)])[: len(g["eigenvalues"])]
        worst = max(worst, float(np.max(np.abs(ev - np.asarray(g["eigenvalues"])))) / scale)
    print(f"c4 {bath}: worst sector eigenvalue deviation {worst:.2e} (relative to |E0|)")
    assert worst < 1e-10
    assert res.states.sectors == gold["states"]["sectors"]
    np.testing.assert_allclose(res.states.energies, gold["states"]["energies"], rtol=1e-10, atol=0)


@pytest.mark.parametrize("bath", ["flat", "random"])
def test_c5_gf_matches_fixture(bath):
    from edgpu.diag import DiagOptions
    from edgpu.farm import farm_diag
    from edgpu.gf import GFOptions, build_gf
    from golden.golden_configs import c5_config

    gold = np.load(os.path.join(GOLD, f"c5_gf_{bath}.npz"))
    cfg = c5_config(bath)
    res = farm_diag(cfg, DiagOptions())
    assert abs(res.states.emin - float(gold["E0"])) <= 1e-10 * abs(float(gold["E0"]))
    assert res.states.sectors == [int(s) for s in gold["sectors"]]
    Gm, _ = build_gf(cfg, res.states, GFOptions(), owners=res.owners)
    got = Gm[..., gold["iw_index"]]
    ref = gold["Gm"]
    rel = float(np.max(np.abs(got - ref)) / np.max(np.abs(ref)))
    print(f"c5 {bath}: G(iw) max relative deviation {rel:.2e}")
    assert rel < 1e-10
    assert np.max(np.abs(ref[0, 1, 0, 0])) > 1e-8 * np.max(np.abs(ref))   # spin-mixed part present


def test_c4_flat_probe_recovers_missed_copies():
    """The degeneracy probe on the sectors where it matters: with the flat
    bath, a single-vector Krylov solve (ED_OPT_EIGH_NO_VERIFY: no probe)
    misses degenerate copies in some configs[3] sectors — it returns a
    spectrum that differs from the dense fixture there — and the default
    solve (screen with the residual-interval exit, then the thick-restart
    probe on the flagged complement) matches the fixture on every one of
    those sectors."""
    from edgpu.diag import DiagOptions
    from edgpu.farm import farm_diag
    from golden.golden_configs import c4_config

    gold = _load("c4_diag_flat.json")
    cfg = c4_config("flat")
    nov = farm_diag(cfg, DiagOptions(kernel_options=("eigh_no_verify",)))
    dflt = farm_diag(cfg, DiagOptions())
    scale = abs(gold["E0"])
    missed = []
    for k, g in gold["sectors"].items():
        ref = np.asarray(g["eigenvalues"])
        a = np.asarray(nov.eigenvalues[int(k)])[: len(ref)]
        if np.max(np.abs(a - ref)) / scale > 1e-10:
            missed.append(int(k))
    assert missed, "no sector with a missed degenerate copy: the probe is untested here"
    for k in missed:
        ref = np.asarray(gold["sectors"][str(k)]["eigenvalues"])
        b = np.asarray(dflt.eigenvalues[k])[: len(ref)]
        assert np.max(np.abs(b - ref)) / scale < 1e-10, k
    print(f"c4 flat: {len(missed)} sectors with missed copies without the probe, all recovered")
