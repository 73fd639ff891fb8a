"""Two-pass matrix-free Kronecker H·v (k_kron_up + k_kron_dw, ed_kernels.hpp)
against the one-pass k_kron and the oracle.

The two-pass form keeps k_kron's term order per element (diagonal, up hops,
down hops, each in slot order), so its H·v is bit-identical to k_kron's; the
Lanczos epilogue reduces over a different grid, so alpha/beta agree to
rounding (1e-12 relative).  Sector(kron2=True) forces the two-pass form on
small sectors (by default it serves sectors of dim >= 2^19), kron2=False
disables it.
"""
import numpy as np
import pytest

from cases import CASES
from oracle.oracle import Oracle, spmv, start_vector

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _both(cfg, q, real, options=()):
    from edgpu.hamiltonian import Sector

    A = Sector(cfg, q[0], q[1], stored=False, direct=True, real=real, kron2=True, options=options)
    B = Sector(cfg, q[0], q[1], stored=False, direct=True, real=real, kron2=False)
    return A, B


@pytest.mark.parametrize("name,factory,sectors", CASES, ids=[c[0] for c in CASES])
def test_two_pass_bit_identical(name, factory, sectors):
    cfg = factory()
    orc = Oracle(cfg)
    for q in sectors:
        A, B = _both(cfg, q, real=False)
        with A, B:
            if not A.info.kron:
                pytest.skip("no Kronecker form (Jx/Jp or not normal mode)")
            x = start_vector(A.dim)
            xd = torch.from_numpy(x).to("cuda:0")
            ya, yb = torch.empty_like(xd), torch.empty_like(xd)
            A.hxv_dev(xd, ya, path=2)
            B.hxv_dev(xd, yb, path=2)
            torch.cuda.synchronize()
            assert torch.equal(ya, yb)                          # bit-identical to k_kron
            ref = spmv(orc.build_csr(orc.build_sector(*q)), x)
            got = ya.cpu().numpy()
            assert np.max(np.abs(got - ref)) <= 1e-13 * np.max(np.abs(ref))


@pytest.mark.parametrize("cfg_kw,q", [
    (dict(Norb=1, Nbath=7), (4, 4)),                                     # configs[1] sector
    (dict(Norb=2, Nbath=5, bath="random", seed=20251015), (6, 6)),       # configs[3] largest
    (dict(Norb=2, Nbath=4, bath="random", seed=4), (3, 6)),              # du != dd
    (dict(Norb=1, Nbath=6, bath="random", seed=6), (3, 4)),              # odd DimUp (35)
])
@pytest.mark.parametrize("offset", [False, True], ids=["aligned", "offset8"])
def test_two_pass_real_vectors_and_lanczos(cfg_kw, q, offset):
    """Pass D takes two columns per lane at even DimUp and 16-byte aligned
    vectors (odd DimUp, or input / output 8 bytes off a 16-byte boundary: one
    column per lane on the same grid) — the same H·v bit for bit."""
    from edgpu.params import make_config

    cfg = make_config(**cfg_kw)
    A, B = _both(cfg, q, real=True)
    with A, B:
        i = torch.arange(1, A.dim + 1, dtype=torch.float64, device="cuda:0")
        x = torch.sin(i)
        ya, yb = torch.empty_like(x), torch.empty_like(x)
        B.hxv_dev(x, yb, path=2)   # one-pass k_kron: the reference sums
        if offset:   # views one element into larger buffers: 8-byte aligned only
            xb = torch.zeros(A.dim + 1, dtype=torch.float64, device="cuda:0")
            xb[1:] = x
            yo = torch.empty(A.dim + 1, dtype=torch.float64, device="cuda:0")
            A.hxv_dev(xb[1:], yo[1:], path=2)
            ya = yo[1:]
        else:
            A.hxv_dev(x, ya, path=2)
        torch.cuda.synchronize()
        assert torch.equal(ya, yb)
        # the Lanczos epilogue (w = Hv/b - b p, alpha) in pass D: multi-kernel
        # recurrence on a sector too large for the persistent kernels, or the
        # same sector when it is small (then both take the persistent path)
        a1, b1, n1 = A.lanc_tridiag(x.cpu().numpy(), 24, 0.0)
        a2, b2, n2 = B.lanc_tridiag(x.cpu().numpy(), 24, 0.0)
        assert n1 == n2 == 24
        np.testing.assert_allclose(a1, a2, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(b1, b2, rtol=1e-12, atol=1e-12)

