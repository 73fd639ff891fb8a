"""CPU tests of the oracle (no GPU): pinned against the reference outputs
recorded in SURVEY.md (tests/golden/survey_pins.json) and against an
independent second-quantised construction (oracle/jw_dense.py).
"""
import json
import os

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as sla

from cases import CASES
from edgpu.params import make_config
from oracle.jw_dense import sector_matrix
from oracle.oracle import Oracle, lanc_eigh, lanc_tridiag, spmv, start_vector, tql2

HERE = os.path.dirname(os.path.abspath(__file__))
PINS = json.load(open(os.path.join(HERE, "golden", "survey_pins.json")))


def _csr_dense(csr, dim):
    return sp.csr_matrix((csr[2], csr[1], csr[0]), shape=(dim, dim)).toarray()


@pytest.mark.parametrize("pin", [p for p in PINS["sectors"] if not p.get("gpu_only")],
                         ids=[p["name"] for p in PINS["sectors"] if not p.get("gpu_only")])
def test_survey_pins(pin):
    """dim, nnz and E0 of the reference run recorded in SURVEY.md §6/§8a."""
    cfg = make_config(**pin["config"])
    orc = Oracle(cfg)
    hmap = orc.build_sector(*pin["sector"])
    assert len(hmap) == pin["dim"]
    csr = orc.build_csr(hmap)
    assert len(csr[1]) == pin["nnz"]
    if "e0" in pin:
        A = sp.csr_matrix((csr[2], csr[1], csr[0]), shape=(len(hmap),) * 2)
        e0 = sla.eigsh(A, k=1, which="SA", tol=1e-13)[0][0]
        assert round(e0, 8) == pin["e0"]


@pytest.mark.parametrize("name,factory,sectors", CASES, ids=[c[0] for c in CASES])
def test_oracle_vs_second_quantisation(name, factory, sectors):
    cfg = factory()
    orc = Oracle(cfg)
    for q1, q2 in sectors:
        hmap = orc.build_sector(q1, q2)
        csr = orc.build_csr(hmap)
        A = _csr_dense(csr, len(hmap))
        B = sector_matrix(cfg, hmap)
        assert np.max(np.abs(A - B)) < 1e-13
        # hermiticity and stored == direct (reference's own two paths)
        assert np.max(np.abs(A - A.conj().T)) == 0.0
        x = start_vector(len(hmap))
        hv = spmv(csr, x)
        assert np.max(np.abs(orc.direct_hxv(hmap, x) - hv)) <= 1e-13 * np.max(np.abs(hv))


def test_sector_enumeration_matches_dimension_formulas():
    from edgpu.sectors import setup_pointers

    from cases import nonsu2_jz

    for cfg in (make_config(Norb=1, Nbath=4), make_config(Norb=1, Nbath=3, Nspin=2, ed_mode="nonsu2"),
                make_config(Norb=1, Nbath=3, ed_mode="superc"), nonsu2_jz()):
        orc = Oracle(cfg)
        for s in setup_pointers(cfg):
            assert len(orc.build_sector(s.q1, s.q2)) == s.dim


def test_binary_search_order():
    """H%map strictly ascending (binary_search precondition, ED_SETUP.f90:1307)."""
    cfg = make_config(Norb=1, Nbath=5, Nspin=2, ed_mode="nonsu2")
    m = Oracle(cfg).build_sector(6, 0)
    assert np.all(np.diff(m.astype(np.int64)) > 0)


def test_tql2_matches_lapack():
    rng = np.random.default_rng(0)
    d = rng.normal(size=30)
    e = np.concatenate([[0.0], rng.normal(size=29)])
    w, z, ierr = tql2(d, e)
    assert ierr == 0
    T = np.diag(d) + np.diag(e[1:], 1) + np.diag(e[1:], -1)
    ref, V = np.linalg.eigh(T)
    np.testing.assert_allclose(w, ref, rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(np.abs(z[0]), np.abs(V[0]), atol=1e-10)


def test_plain_lanczos_restatement():
    """lanczos_plain_c converges to the exact ground state; tridiag reproduces
    the Krylov spectrum's extremes."""
    cfg = make_config(Norb=1, Nbath=5)
    orc = Oracle(cfg)
    hmap = orc.build_sector(3, 3)
    csr = orc.build_csr(hmap)
    A = _csr_dense(csr, len(hmap))
    exact = np.linalg.eigvalsh(A)[0]
    e0, vec, n = lanc_eigh(csr, start_vector(len(hmap)), 200)
    assert abs(e0 - exact) < 1e-10
    assert np.linalg.norm(A @ vec - e0 * vec) < 1e-6
    a, b, nl = lanc_tridiag(csr, start_vector(len(hmap)), 60)
    T = np.diag(a[:nl]) + np.diag(b[1:nl], 1) + np.diag(b[1:nl], -1)
    assert abs(np.linalg.eigvalsh(T)[0] - exact) < 1e-10


def test_complex_vr_reference_quirk():
    """Complex replica vr: stored H has conj(vr) on both (i,j) and (j,i) of a
    hybridisation pair (stored/Himp_bath.f90:20,32) -> symmetric, not
    Hermitian, in that block.  The oracle reproduces the stored semantics."""
    from cases import replica_cplx_vr

    cfg = replica_cplx_vr()
    orc = Oracle(cfg)
    hmap = orc.build_sector(3, 3)
    A = _csr_dense(orc.build_csr(hmap), len(hmap))
    B = sector_matrix(cfg, hmap)        # Hermitian construction
    D = A - B
    assert np.max(np.abs(D)) > 0.1      # differs exactly in the vr block
    mask = np.abs(D) > 1e-12
    # in the vr block the stored value is the conjugate of the Hermitian one ...
    assert np.max(np.abs(A[mask] - np.conj(B[mask]))) < 1e-13
    # ... and everything else is the Hermitian operator
    assert np.max(np.abs(D[~mask])) < 1e-13


def test_jz_sectors_partition_and_targets():
    """Jz_basis (ED_SETUP.f90:636-664, 769-805, 940-965): the (n, twoJz)
    sectors of the t2g case tile the whole Fock space, each n-sector is the
    disjoint union of its Jz sectors (same states as the n basis), and
    c+/c of (iorb, ispin) move twoJz by +-(2*Lzdiag(iorb) + Szdiag(ispin))."""
    from cases import nonsu2_jz
    from edgpu.sectors import cdg_sector, c_sector, setup_pointers

    cfg = nonsu2_jz()
    secs = setup_pointers(cfg)
    assert sum(s.dim for s in secs) == 4 ** cfg.Ns
    orc = Oracle(cfg)
    import copy

    cn = copy.deepcopy(cfg)
    cn.Jz_basis = False
    on = Oracle(cn)
    for n in (5, 6):
        whole = set(on.build_sector(n, 0).tolist())
        parts = [set(orc.build_sector(s.q1, s.q2).tolist()) for s in secs if s.q1 == n]
        assert sum(len(p) for p in parts) == len(whole) and set().union(*parts) == whole
    lz = (-1, 1, 0)
    sec = [s for s in secs if (s.q1, s.q2) == (6, 0)][0]
    for iorb in range(3):
        for ispin, sz in ((0, 1), (1, -1)):
            t = cdg_sector(cfg, sec, ispin, iorb)
            assert (t.q1, t.q2) == (7, 2 * lz[iorb] + sz)
            t = c_sector(cfg, sec, ispin, iorb)
            assert (t.q1, t.q2) == (5, -(2 * lz[iorb] + sz))


def test_build_csr_rows_and_sampled_check():
    """orc_build_csr_rows equals the matching slice of orc_build_csr, and the
    sampled-row check of the full-size GPU tests (tests/sampled_rows.py)
    accepts spMatVec_cc's own result and rejects a perturbed one."""
    from cases import CASES
    from oracle.oracle import spmv
    from sampled_rows import check_rows, sample_starts

    cfg = CASES[0][1]()
    orc = Oracle(cfg)
    hmap = orc.build_sector(*CASES[0][2][0])
    csr = orc.build_csr(hmap)
    rp, cols, vals = csr
    r0, n = 37, 101
    rp2, c2, v2 = orc.build_csr_rows(hmap, r0, n)
    np.testing.assert_array_equal(rp2, rp[r0:r0 + n + 1] - rp[r0])
    np.testing.assert_array_equal(c2, cols[rp[r0]:rp[r0 + n]])
    np.testing.assert_array_equal(v2, vals[rp[r0]:rp[r0 + n]])
    x = start_vector(len(hmap))
    y = spmv(csr, x)
    starts = sample_starts(len(hmap), nblocks=16, block=640)
    assert check_rows(orc, hmap, x, y, starts, block=640) <= 1e-15
    y[starts[3] + 5] += 1e-6
    with pytest.raises(AssertionError):
        check_rows(orc, hmap, x, y, starts, block=640)
