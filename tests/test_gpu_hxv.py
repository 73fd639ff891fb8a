"""GPU parity of the H·v hot path against the CPU oracle (through the C-ABI).

Bars (stated per assertion):
  * basis H%map, stored-H columns and values: bit-exact (integer/index work, and
    the diagonal is accumulated in reference order without FMA contraction);
  * stored H·v: bit-exact vs the oracle's spMatVec_cc (same per-row summation
    order, no contraction);
  * matrix-free generic kernel: bit-exact vs the stored kernel (same row order);
  * matrix-free Kronecker kernel and the reference's scatter-form
    directMatVec_cc: 1e-13 relative (different summation order).
"""
import numpy as np
import pytest

from cases import CASES
from oracle.oracle import Oracle, spmv, spmv_real, start_vector

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.mark.parametrize("name,factory,sectors", CASES, ids=[c[0] for c in CASES])
def test_stored_and_direct_match_oracle(name, factory, sectors):
    from edgpu.hamiltonian import Sector

    cfg = factory()
    orc = Oracle(cfg)
    for q1, q2 in sectors:
        hmap = orc.build_sector(q1, q2)
        csr = orc.build_csr(hmap)
        with Sector(cfg, q1, q2, stored=True, direct=True) as S:
            assert S.dim == len(hmap)
            assert S.nnz == len(csr[1])
            np.testing.assert_array_equal(S.map(), hmap)          # bit-exact
            rp, cols, vals = S.dump_csr()
            np.testing.assert_array_equal(rp, csr[0])
            np.testing.assert_array_equal(cols, csr[1])
            np.testing.assert_array_equal(vals, csr[2])            # bit-exact values
            x = start_vector(S.dim)
            ref = spmv(csr, x)
            hv = S.hxv(x)
            np.testing.assert_array_equal(hv, ref)                 # bit-exact H·v
            xd = _dev(x)
            out = torch.empty_like(xd)
            S.hxv_dev(xd, out, path=1)                              # generic matrix-free
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy(), ref)
            if S.info.kron:
                S.hxv_dev(xd, out, path=2)                          # Kronecker matrix-free
                torch.cuda.synchronize()
                assert _rel(out.cpu().numpy(), ref) < 1e-13
            # the reference's own scatter-form direct product agrees to rounding
            assert _rel(orc.direct_hxv(hmap, x), ref) < 1e-13


@pytest.mark.parametrize("name,factory,sectors", [c for c in CASES if c[1]().is_real()],
                         ids=[c[0] for c in CASES if c[1]().is_real()])
def test_real_variant(name, factory, sectors):
    """real(8) storage (configs[1] is quoted in real(8)): values and H·v."""
    from edgpu.hamiltonian import Sector

    cfg = factory()
    orc = Oracle(cfg)
    q1, q2 = sectors[0]
    hmap = orc.build_sector(q1, q2)
    csr = orc.build_csr(hmap)
    with Sector(cfg, q1, q2, stored=True, direct=True, real=True) as S:
        rp, cols, vals = S.dump_csr()
        np.testing.assert_array_equal(cols, csr[1])
        np.testing.assert_array_equal(vals, csr[2])
        x = np.sin(np.arange(1, S.dim + 1, dtype=np.float64))
        ref = spmv_real(csr, x)
        xd = _dev(x)
        out = torch.empty_like(xd)
        for path in (0, 1):
            S.hxv_dev(xd, out, path=path)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy(), ref)
        if S.info.kron:
            S.hxv_dev(xd, out, path=2)
            torch.cuda.synchronize()
            assert _rel(out.cpu().numpy(), ref) < 1e-13
        # real H applied to complex vectors (the reference's complex interface)
        z = start_vector(S.dim)
        assert _rel(S.hxv(z), spmv(csr, z)) == 0.0


def test_errors_are_loud():
    from edgpu._lib import EDGPUError
    from edgpu.hamiltonian import Sector
    from cases import replica_cplx

    cfg = replica_cplx()
    with pytest.raises(EDGPUError):
        Sector(cfg, 3, 3, real=True)          # complex bath cannot be stored real
    with Sector(cfg, 3, 3) as S:
        with pytest.raises(ValueError):
            S.hxv(np.zeros(S.dim + 1, dtype=np.complex128))


def test_complex_vr_stored_semantics():
    """Complex replica vr (non-Hermitian in the reference's stored H): the GPU
    reproduces the stored semantics bit-exactly on every path."""
    from edgpu.hamiltonian import Sector
    from cases import replica_cplx_vr

    cfg = replica_cplx_vr()
    orc = Oracle(cfg)
    hmap = orc.build_sector(3, 3)
    csr = orc.build_csr(hmap)
    with Sector(cfg, 3, 3, stored=True, direct=True) as S:
        np.testing.assert_array_equal(S.dump_csr()[2], csr[2])
        x = start_vector(S.dim)
        ref = spmv(csr, x)
        np.testing.assert_array_equal(S.hxv(x), ref)
        xd = _dev(x)
        out = torch.empty_like(xd)
        S.hxv_dev(xd, out, path=1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), ref)
        S.hxv_dev(xd, out, path=2)
        torch.cuda.synchronize()
        assert _rel(out.cpu().numpy(), ref) < 1e-13


@pytest.mark.parametrize("pin", ["n28_norb1", "n28_norb2"])
def test_full_size_roofline_sectors(pin):
    """Nlevels=28 (7,7) sectors at full size (dim 11,778,624): nnz pins of the
    reference run, the default stored H·v against the oracle on >= 16,384
    sampled rows (1e-13 of the row's absolute sum, tests/sampled_rows.py),
    size-independent properties: hermiticity <x,Hy> = <Hx,y>,
    the one-pass stored kernel (ED_OPT_STORED_EXACT) == generic matrix-free
    bit for bit, the default two-segment stored kernel and Kronecker to 1e-13."""
    import json
    import os

    from edgpu.hamiltonian import Sector
    from edgpu.params import make_config

    pins = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "survey_pins.json")))
    p = [x for x in pins["sectors"] if x["name"] == pin][0]
    cfg = make_config(bath="random", seed=1, **p["config"])
    from sampled_rows import check_rows, sample_starts

    orc = Oracle(cfg)
    hmap = orc.build_sector(*p["sector"])
    with Sector(cfg, *p["sector"], stored=True, direct=True, real=True) as S:
        assert S.dim == p["dim"] and S.nnz == p["nnz"]
        g = torch.Generator(device="cuda:0").manual_seed(0)
        x = torch.rand(S.dim, dtype=torch.float64, device="cuda:0", generator=g)
        y = torch.rand(S.dim, dtype=torch.float64, device="cuda:0", generator=g)
        hx, hy = torch.empty_like(x), torch.empty_like(x)
        S.hxv_dev(x, hx, path=0)
        S.hxv_dev(y, hy, path=0)
        # the default (two-segment) stored H·v against the oracle's rows
        worst = check_rows(orc, hmap, x.cpu().numpy(), hx.cpu().numpy(), sample_starts(S.dim, seed=1))
        print(f"{pin}: worst sampled-row error {worst:.1e} of sum|H_ij x_j|")
        a, b = torch.dot(y, hx).item(), torch.dot(hy, x).item()
        assert abs(a - b) <= 1e-12 * abs(a)
        h1 = torch.empty_like(x)
        assert S.info.split == 1              # HBM-sized: the two-segment form is the default
        S.set_options("stored_exact")
        he = torch.empty_like(x)
        S.hxv_dev(x, he, path=0)
        S.set_options()
        assert (he - hx).abs().max().item() <= 1e-13 * hx.abs().max().item()
        S.hxv_dev(x, h1, path=1)
        assert torch.equal(h1, he)
        S.hxv_dev(x, h1, path=2)
        assert (h1 - hx).abs().max().item() <= 1e-13 * hx.abs().max().item()


@pytest.mark.parametrize("name,factory,sectors", CASES, ids=[c[0] for c in CASES])
def test_packed_matches_plain_sell(name, factory, sectors):
    """Packed stored H ({col|value index} words over the distinct values) gives
    bit-identical H·v to the plain SELL arrays: real(8) H with real and complex
    vectors, and complex(8) H (the reference's arithmetic, dictionary of
    (re, im) pairs) with complex vectors."""
    from edgpu.hamiltonian import Sector

    cfg = factory()
    q1, q2 = sectors[0]
    for real in ((True, False) if cfg.is_real() else (False,)):
        with Sector(cfg, q1, q2, stored=True, real=real) as S:
            with Sector(cfg, q1, q2, stored=True, real=real, pack=False) as P:
                assert P.info.packed == 0
                assert S.info.packed == 1 and 1 <= S.info.npdict <= 256
                i = np.arange(1, S.dim + 1, dtype=np.float64)
                xs = (np.sin(i), np.sin(i) + 1j * np.cos(3 * i)) if real else (np.sin(i) + 1j * np.cos(3 * i),)
                for x in xs:
                    xd = _dev(x)
                    y1 = torch.empty_like(xd)
                    y2 = torch.empty_like(xd)
                    S.hxv_dev(xd, y1, path=0)
                    P.hxv_dev(xd, y2, path=0)
                    torch.cuda.synchronize()
                    assert torch.equal(y1, y2)


@pytest.mark.parametrize("cplx", [False, True])
def test_n28_packed_matches_plain(cplx):
    """Nlevels=28 sector (matrix beyond the MALL: non-temporal matrix loads,
    XCD-remapped block order on the packed kernel): the one-pass packed real /
    complex H (ED_OPT_STORED_EXACT: the two-segment form is this sector's
    default) gives H·v identical to the plain SELL arrays."""
    from edgpu.hamiltonian import Sector
    from edgpu.params import make_config

    cfg = make_config(Norb=1, Nbath=13, bath="random", seed=3)
    g = torch.Generator(device="cuda:0").manual_seed(1)
    with Sector(cfg, 7, 7, stored=True, real=not cplx, options=("stored_exact",)) as S:
        with Sector(cfg, 7, 7, stored=True, real=not cplx, pack=False) as P:
            assert S.info.packed == 1 and P.info.packed == 0
            dt = torch.complex128 if cplx else torch.float64
            x = torch.rand(S.dim, dtype=dt, device="cuda:0", generator=g)
            y1, y2 = torch.empty_like(x), torch.empty_like(x)
            S.hxv_dev(x, y1, path=0)
            P.hxv_dev(x, y2, path=0)
            torch.cuda.synchronize()
            assert torch.equal(y1, y2)
