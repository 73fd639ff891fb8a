"""Two-segment stored H·v (ed_split.hpp) against the oracle, through the C-ABI.

The two-segment form re-lays the stored matrix losslessly (every element once,
the stored double) and sums each row as diagonal + in-block elements, then the
cross-block elements: a reordering of spMatVec_cc's row sum
(ED_HAMILTONIAN_STORED_HxV.f90:132-143).  Bars:
  * H·v per element within 1e-13 of the oracle's spMatVec_cc, relative to the
    row's absolute sum sum_j |H_ij x_j| (the rounding bound of any summation
    order), and the one-pass kernel (ED_OPT_STORED_EXACT) still bit-exact;
  * Lanczos alpha/beta (first 15 steps) at 1e-10 and E0 at 1e-10 against the
    oracle recurrence; thick-restart eigenvalues at 1e-10 vs dense eigh;
  * at BASELINE's Nlevels=28 size (split built by default): against the
    one-pass kernel at 1e-13 (row abs-sum bound), symmetry <y, Hx> = <Hy, x>.
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
    prod = np.abs(vals) * np.abs(x[cols])
    np.add.at(out, np.repeat(np.arange(len(rp) - 1), np.diff(rp)), prod)
    return out


def _check_rows(y, ref, bound, tol=1e-13):
    err = np.abs(y - ref)
    assert np.all(err <= tol * bound + 1e-300), float(np.max(err / np.maximum(bound, 1e-300)))


@pytest.mark.parametrize("name,factory,sectors", CASES, ids=[c[0] for c in CASES])
def test_split_hxv_matches_oracle(name, factory, sectors):
    from edgpu.hamiltonian import Sector

    cfg = factory()
    orc = Oracle(cfg)
    for q1, q2 in sectors:
        hmap = orc.build_sector(q1, q2)
        csr = orc.build_csr(hmap)
        reals = (True, False) if cfg.is_real() else (False,)
        for real in reals:
            with Sector(cfg, q1, q2, stored=True, real=real, split=True) as S:
                # (a sector without off-diagonal elements has no packed words
                # and keeps the one-pass kernel; complex(8) H keeps it too:
                # the two-segment form serves real H on real vectors)
                assert S.info.packed == (1 if S.nnz > S.dim else 0)
                assert S.info.split == (S.info.packed if real else 0), "two-segment form not built"
                assert 0 <= S.info.split_far_uniform <= S.info.split_far <= S.nnz - S.dim
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
                    if np.isrealobj(x):
                        _check_rows(y.cpu().numpy(), ref, bound)
                    else:  # complex vectors: the one-pass kernel, bit-exact
                        np.testing.assert_array_equal(y.cpu().numpy(), ref)
                    S.set_options("stored_exact")                  # one-pass kernel: bit-exact
                    S.hxv_dev(xd, y, path=0)
                    torch.cuda.synchronize()
                    np.testing.assert_array_equal(y.cpu().numpy(), ref)
                    S.set_options()


def test_split_uniform_fraction_normal_mode():
    """Normal mode without Jx/Jp: every cross-block element is a down-spin hop
    with the same column offset and value across a block's rows, so the B
    slices hold them all as U entries (no per-lane words)."""
    from edgpu.hamiltonian import Sector
    from cases import c2

    with Sector(c2(), 4, 4, stored=True, real=True, split=True) as S:
        assert S.info.split_far > 0
        assert S.info.split_far_uniform == S.info.split_far


@pytest.mark.parametrize("real", [True, False], ids=["real_vec", "complex_vec"])
def test_split_lanczos_matches_oracle(real):
    """The Lanczos epilogues run in segment B: multi-kernel recurrence on the
    split sector vs the oracle's recurrence (alpha/beta 1e-10, E0 1e-10)."""
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
    ar, br, nr = lanc_tridiag(csr, v0 + 0j, 60)
    with Sector(cfg, 3, 3, stored=True, real=True, split=True, options=("no_persist",)) as S:
        assert S.info.split == 1
        a, b, n = S.lanc_tridiag(v0, 60, real=real)
        np.testing.assert_allclose(a[:15], ar[:15], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(b[:15], br[:15], rtol=1e-10, atol=1e-12)
        e0, _, _ = S.lanc_eigh(nitermax=512, threshold=1e-12, v0=v0, real=real, vector=False)
        eref, _, _ = lanc_eigh(csr, v0 + 0j, 512)
        assert abs(e0 - eref) <= 1e-10 * abs(eref)


def test_split_eigh_matches_dense():
    """Thick-restart eigh (shifted three-term epilogue in segment B) on a
    split nonSU2 sector (spin flips: per-lane L words beside the U entries):
    the 6 lowest eigenvalues at 1e-10 vs dense eigh."""
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
    with Sector(cfg, 6, 0, stored=True, real=True, split=True) as S:
        assert S.info.split == 1
        assert S.info.split_far > S.info.split_far_uniform  # (spin flips: L words)
        ev, _, nconv, _ = S.eigh(neigen=6, ncv=23, maxit=300, tol=1e-12, vectors=False, real=True)
        assert nconv == 6
        np.testing.assert_allclose(ev, w[:6], rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("cplx", [False, True], ids=["real", "complex"])
def test_n28_split_default(cplx):
    """Nlevels=28 (7,7), the roofline sector: the default stored H·v (the
    two-segment form where it is built) against the oracle on >= 16,384
    sampled rows (tests/sampled_rows.py: orc_build_csr_rows, 1e-13 of each
    row's sum_j |H_ij x_j|), the one-pass kernel (ED_OPT_STORED_EXACT) on the
    same rows, every cross-block element uniform, and <z, Hx> = <Hz, x>."""
    from edgpu.hamiltonian import Sector
    from edgpu.params import make_config
    from sampled_rows import check_rows, sample_starts

    cfg = make_config(Norb=1, Nbath=13, bath="random", seed=3)
    orc = Oracle(cfg)
    hmap = orc.build_sector(7, 7)
    g = torch.Generator(device="cuda:0").manual_seed(5)
    with Sector(cfg, 7, 7, stored=True, real=not cplx) as S:
        assert S.dim == len(hmap)
        if S.info.split:
            assert S.info.split_far_uniform == S.info.split_far > 0
        else:
            assert cplx, "two-segment form not built for the real(8) sector"
        dt = torch.complex128 if cplx else torch.float64
        x = torch.rand(S.dim, dtype=dt, device="cuda:0", generator=g) - 0.5
        y1, y2 = torch.empty_like(x), torch.empty_like(x)
        S.hxv_dev(x, y1, path=0)
        S.set_options("stored_exact")
        S.hxv_dev(x, y2, path=0)
        S.set_options()
        xh = x.cpu().numpy()
        starts = sample_starts(S.dim)
        w1 = check_rows(orc, hmap, xh, y1.cpu().numpy(), starts)
        w2 = check_rows(orc, hmap, xh, y2.cpu().numpy(), starts)
        print(f"N28 {'complex' if cplx else 'real'} split={S.info.split}: worst sampled-row error "
              f"{w1:.1e} (default), {w2:.1e} (one-pass) of sum|H_ij x_j|")
        z = torch.rand(S.dim, dtype=dt, device="cuda:0", generator=g) - 0.5
        hz = torch.empty_like(z)
        S.hxv_dev(z, hz, path=0)
        a = torch.vdot(z, y1).item()
        b = torch.vdot(hz, x).item()
        assert abs(a - b) <= 1e-12 * abs(a)


def test_split_offset_views_take_one_pass():
    """8-byte aligned vector views (a torch slice at an odd offset): segment
    B's 16-byte pair loads/stores need 16-byte aligned x and y, so such a call
    takes the one-pass kernel — bit-exact with spMatVec_cc — and aligned
    views keep the two-segment form (1e-13 of the row's |H||x|)."""
    from edgpu.hamiltonian import Sector
    from cases import c2

    cfg = c2()
    orc = Oracle(cfg)
    hmap = orc.build_sector(4, 4)
    csr = orc.build_csr(hmap)
    with Sector(cfg, 4, 4, stored=True, real=True, split=True) as S:
        assert S.info.split == 1
        x = np.sin(np.arange(1, S.dim + 1, dtype=np.float64))
        ref = spmv_real(csr, x)
        bound = _abs_rows(csr, x)
        xb = torch.zeros(S.dim + 2, dtype=torch.float64, device="cuda:0")
        yb = torch.zeros(S.dim + 2, dtype=torch.float64, device="cuda:0")
        for ox, oy in ((1, 1), (1, 0), (0, 1), (0, 0)):
            xv = xb[ox:ox + S.dim]
            xv.copy_(_dev(x))
            yv = yb[oy:oy + S.dim]
            S.hxv_dev(xv, yv, path=0)
            torch.cuda.synchronize()
            got = yv.cpu().numpy()
            if ox or oy:
                np.testing.assert_array_equal(got, ref)
            else:
                _check_rows(got, ref, bound)
