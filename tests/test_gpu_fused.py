"""Fused one-pass re-laid stored H·v (ed_fused.hpp) against the oracle,
through the C-ABI.

The fused form re-lays the packed stored matrix losslessly into 64-row units
of one idw block: in-block elements as per-lane words (A), cross-block
elements that every row of the unit holds with the same {column offset,
value} once per unit (U), the rest per lane (L); one sweep in row order sums
diagonal, A, U, L — a reordering of spMatVec_cc's row sum
(ED_HAMILTONIAN_STORED_HxV.f90:132-143).  Bars:
  * H·v per element within 1e-13 of the oracle's spMatVec_cc relative to the
    row's sum_j |H_ij x_j| (the rounding bound of any summation order), every
    case of tests/cases.py (real and complex H, real and complex vectors);
  * the Lanczos (EpiLancA) and thick-restart (EpiTrlLoc) epilogues on the
    fused kernel: alpha/beta and E0 at 1e-10 vs the oracle recurrence,
    eigenvalues at 1e-10 vs dense eigh;
  * at Nlevels=26/28 size (built by default): the oracle on >= 16,384 sampled
    rows (tests/sampled_rows.py), real and complex vectors, complex(8) H, a
    nonSU2 sector (spin flips in L words), and <z, Hx> = <Hz, x>.
"""
import numpy as np
import pytest

from cases import CASES
from oracle.oracle import Oracle, lanc_tridiag, spmv, spmv_real, start_vector

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def _abs_rows(csr, x):
    rp, cols, vals = csr
    out = np.zeros(len(rp) - 1)
    np.add.at(out, np.repeat(np.arange(len(rp) - 1), np.diff(rp)), np.abs(vals) * np.abs(x[cols]))
    return out


def _check_rows(y, ref, bound, tol=1e-13):
    err = np.abs(y - ref)
    worst = float(np.max(err / np.maximum(bound, 1e-300)))
    assert np.all(err <= tol * bound + 1e-300), worst
    return worst


@pytest.mark.parametrize("name,factory,sectors", CASES, ids=[c[0] for c in CASES])
def test_fused_hxv_matches_oracle(name, factory, sectors):
    from edgpu.hamiltonian import Sector

    cfg = factory()
    orc = Oracle(cfg)
    for q1, q2 in sectors:
        hmap = orc.build_sector(q1, q2)
        csr = orc.build_csr(hmap)
        reals = (True, False) if cfg.is_real() else (False,)
        for real in reals:
            with Sector(cfg, q1, q2, stored=True, real=real, fused=True) as S:
                if not S.info.packed:
                    continue     # (a sector without off-diagonal elements keeps the plain kernel)
                assert S.info.fused == 1, "fused form not built"
                assert 0 <= S.info.fused_far_uniform <= S.info.fused_far <= S.nnz - S.dim
                i = np.arange(1, S.dim + 1, dtype=np.float64)
                xs = [start_vector(S.dim)]
                if real:
                    xs.append(np.sin(i))
                for x in xs:
                    ref = spmv_real(csr, x) if np.isrealobj(x) else spmv(csr, x)
                    bound = _abs_rows(csr, x)
                    xd = _dev(x)
                    y = torch.empty_like(xd)
                    S.hxv_dev(xd, y, path=0)
                    torch.cuda.synchronize()
                    _check_rows(y.cpu().numpy(), ref, bound)
                    S.set_options("stored_exact")        # one-pass kernel: bit-exact
                    S.hxv_dev(xd, y, path=0)
                    torch.cuda.synchronize()
                    np.testing.assert_array_equal(y.cpu().numpy(), ref)
                    S.set_options()


def test_fused_uniform_fraction_normal_mode():
    """Normal mode without Jx/Jp: every cross-block element (a down-spin hop)
    is the same {column offset, value} on every row of a unit, so all of them
    are U entries; nonSU2 spin flips are not (they stay L words)."""
    from edgpu.hamiltonian import Sector
    from cases import c2, c5

    with Sector(c2(), 4, 4, stored=True, real=True, fused=True) as S:
        assert S.info.fused_far > 0
        assert S.info.fused_far_uniform == S.info.fused_far
    with Sector(c5(), 6, 0, stored=True, real=True, fused=True) as S:
        assert 0 < S.info.fused_far_uniform < S.info.fused_far


@pytest.mark.parametrize("real", [True, False], ids=["real_vec", "complex_vec"])
def test_fused_lanczos_matches_oracle(real):
    """Lanczos epilogue (EpiLancA) on the fused kernel, multi-kernel
    recurrence: alpha/beta (15 steps) and E0 at 1e-10 vs the oracle."""
    from edgpu.hamiltonian import Sector
    from oracle.oracle import lanc_eigh
    from cases import normal_jh

    cfg = normal_jh()
    orc = Oracle(cfg)
    hmap = orc.build_sector(3, 3)
    csr = orc.build_csr(hmap)
    v0 = start_vector(len(hmap))
    if real:
        v0 = v0.real.copy()
    ar, br, _ = lanc_tridiag(csr, v0 + 0j, 60)
    with Sector(cfg, 3, 3, stored=True, real=True, fused=True, options=("no_persist",)) as S:
        assert S.info.fused == 1
        a, b, _ = S.lanc_tridiag(v0, 60, real=real)
        np.testing.assert_allclose(a[:15], ar[:15], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(b[:15], br[:15], rtol=1e-10, atol=1e-12)
        e0, _, _ = S.lanc_eigh(nitermax=512, threshold=1e-12, v0=v0, real=real, vector=False)
        eref, _, _ = lanc_eigh(csr, v0 + 0j, 512)
        assert abs(e0 - eref) <= 1e-10 * abs(eref)


@pytest.mark.parametrize("real", [True, False], ids=["real_vec", "complex_vec"])
def test_fused_eigh_matches_dense(real):
    """Thick-restart eigh (shifted three-term epilogue) on a fused nonSU2
    sector with spin flips (L words beside the U entries): the 6 lowest
    eigenvalues at 1e-10 vs dense eigh."""
    from edgpu.hamiltonian import Sector
    from cases import c5

    cfg = c5()
    orc = Oracle(cfg)
    hmap = orc.build_sector(6, 0)
    rp, cols, vals = orc.build_csr(hmap)
    n = len(hmap)
    H = np.zeros((n, n), dtype=np.complex128)
    for r in range(n):
        for k in range(rp[r], rp[r + 1]):
            H[r, cols[k]] += vals[k]
    w = np.linalg.eigvalsh(H)
    with Sector(cfg, 6, 0, stored=True, real=True, fused=True) as S:
        assert S.info.fused == 1
        ev, _, nconv, _ = S.eigh(neigen=6, ncv=23, maxit=300, tol=1e-12, vectors=False, real=real)
        assert nconv == 6
        np.testing.assert_allclose(ev, w[:6], rtol=1e-10, atol=1e-10)


def _big(name):
    from edgpu.params import make_config

    if name == "n28":
        return make_config(Norb=1, Nbath=13, bath="random", seed=3), (7, 7), True
    if name == "n28_cplxH":      # complex(8) H values (the reference's storage), complex dictionary
        return make_config(Norb=1, Nbath=13, bath="random", seed=3), (7, 7), False
    if name == "n26s":           # nonSU2: spin flips (L words)
        return make_config(Norb=1, Nbath=12, Nspin=2, ed_mode="nonsu2", bath="random", seed=3), (13, 0), True
    raise KeyError(name)


@pytest.mark.parametrize("name,cplx", [("n28", False), ("n28", True), ("n28_cplxH", True),
                                       ("n26s", False), ("n26s", True)],
                         ids=["n28-real", "n28-complex", "n28-complexH", "n26s-real", "n26s-complex"])
def test_fused_full_size_sampled_rows(name, cplx):
    """HBM-sized sectors (the fused form is built by default there, forced
    on the nonSU2 one): the fused H·v (real vectors: with the two-segment form
    not built, so that the fused kernel serves them) against the oracle on
    >= 16,384 sampled rows, 1e-13 of each row's sum_j |H_ij x_j|, and
    symmetric to rounding."""
    from edgpu.hamiltonian import Sector
    from sampled_rows import check_rows, sample_starts

    cfg, q, real_h = _big(name)
    orc = Oracle(cfg)
    hmap = orc.build_sector(*q)
    g = torch.Generator(device="cuda:0").manual_seed(11)
    # (nonSU2: 41 % of the cross-block elements in U, below the default
    # policy's 90 %: forced here, the one-pass kernel is that sector's default)
    forced = True if name == "n26s" else None
    with Sector(cfg, *q, stored=True, real=real_h, fused=forced, split=False) as S:
        assert S.dim == len(hmap)
        assert S.info.fused == 1
        dt = torch.complex128 if cplx else torch.float64
        x = torch.rand(S.dim, dtype=dt, device="cuda:0", generator=g) - 0.5
        y = torch.empty_like(x)
        S.hxv_dev(x, y, path=0)
        worst = check_rows(orc, hmap, x.cpu().numpy(), y.cpu().numpy(), sample_starts(S.dim, seed=2))
        print(f"{name} {'complex' if cplx else 'real'} vectors: fused worst sampled-row error {worst:.1e}, "
              f"U share {S.info.fused_far_uniform / max(S.info.fused_far, 1):.3f}")
        z = torch.rand(S.dim, dtype=dt, device="cuda:0", generator=g) - 0.5
        hz = torch.empty_like(z)
        S.hxv_dev(z, hz, path=0)
        a = torch.vdot(z, y).item()
        b = torch.vdot(hz, x).item()
        assert abs(a - b) <= 1e-12 * abs(a)
