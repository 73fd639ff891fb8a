"""Jz_basis sectors (nonsu2, ED_SETUP.f90:636-664, 769-805, 940-965) on the GPU:
the (n, twoJz) split of the t2g spin-orbit case against the oracle and
against the same Hamiltonian in the plain n basis."""
import copy

import numpy as np
import pytest

from cases import nonsu2_jz
from edgpu.diag import DiagOptions, ed_diag

pytestmark = pytest.mark.gpu


def _n_basis(cfg):
    c = copy.deepcopy(cfg)
    c.Jz_basis = False
    return c


def test_jz_ground_state_equals_n_basis():
    """Same H, two sector labellings: the T=0 state list (energies, count)
    agrees; the Jz basis finds the degenerate partners in separate sectors."""
    cfg = nonsu2_jz()
    _, sl = ed_diag(cfg, DiagOptions())
    _, sn = ed_diag(_n_basis(cfg), DiagOptions())
    assert len(sl.energies) == len(sn.energies)
    np.testing.assert_allclose(sorted(sl.energies), sorted(sn.energies), rtol=1e-10, atol=1e-10)


def test_jz_gf_matches_oracle_and_n_basis():
    from edgpu.gf import GFOptions, build_gf
    from oracle_gf import build_gf_oracle

    cfg = nonsu2_jz()
    _, sl = ed_diag(cfg, DiagOptions())
    gopt = GFOptions(Lmats=300, Lreal=300)
    Gm, Gr = build_gf(cfg, sl, gopt)
    Gm0, Gr0 = build_gf_oracle(cfg, sl, gopt)
    scale = np.max(np.abs(Gm0))
    assert np.max(np.abs(Gm - Gm0)) / scale < 1e-10
    # the n basis: same Krylov spaces (H conserves Jz), summed over the same
    # degenerate ground states -> the same G_ii(iw) up to rounding
    cn = _n_basis(cfg)
    _, sn = ed_diag(cn, DiagOptions())
    Gn, _ = build_gf(cn, sn, gopt)
    assert np.max(np.abs(Gm - Gn)) / scale < 1e-8


def test_jz_non_conserving_h_is_rejected():
    from edgpu._lib import EDGPUError
    from edgpu.hamiltonian import Sector

    cfg = nonsu2_jz()
    cfg.impHloc[0, 1, 0, 0] = cfg.impHloc[1, 0, 0, 0] = 0.1    # spin flip at fixed Lz
    with pytest.raises(EDGPUError, match="Jz"):
        Sector(cfg, 6, 0, stored=True)
