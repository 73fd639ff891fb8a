"""GPU device-resident Lanczos against the oracle's restatement of
.repo/PLAIN_LANCZOS.f90 and against scipy's ARPACK on the oracle matrix.

Bars: Ritz values / ground-state energies within 1e-10 relative (north_star);
alpha/beta of the first 15 steps within 1e-10 (summation order differs, so
beyond a few tens of steps the unreorthogonalised recurrences drift apart;
SURVEY §7 hard part 4).
"""
import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as sla

from cases import CASES
from oracle.oracle import Oracle, lanc_eigh, lanc_tridiag, start_vector

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _e0_scipy(csr, dim):
    A = sp.csr_matrix((csr[2], csr[1], csr[0]), shape=(dim, dim))
    if dim <= 400:
        return float(np.linalg.eigvalsh(A.toarray())[0])
    return float(sla.eigsh(A, k=1, which="SA", tol=1e-14)[0][0])


@pytest.mark.parametrize("persist", ["default", "l2", "lds", "multi"],
                         ids=["persistent", "persist_l2", "persist_lds", "multikernel"])
@pytest.mark.parametrize("name,factory,sectors", CASES, ids=[c[0] for c in CASES])
def test_tridiag_and_ground_state(name, factory, sectors, persist):
    """Every device recurrence: the one-workgroup persistent kernel (default for
    sectors that fit one CU: stored matrix in registers / Kronecker tables in
    LDS), its opt-in L2-streaming stored mode, and the graph-captured
    two-kernel one."""
    from edgpu.hamiltonian import Sector

    opts = {"default": (), "multi": ("no_persist",), "l2": ("persist_stored",),
            "lds": ("no_preg",)}[persist]                # no_preg: Kronecker tables in LDS (MODE 1)

    cfg = factory()
    orc = Oracle(cfg)
    q1, q2 = sectors[0]
    hmap = orc.build_sector(q1, q2)
    csr = orc.build_csr(hmap)
    dim = len(hmap)
    v0 = start_vector(dim)
    n = min(dim, 40)
    ar, br, nr = lanc_tridiag(csr, v0, n)
    for direct in (False, True):
        with Sector(cfg, q1, q2, stored=not direct, direct=direct, options=opts) as S:
            a, b, ng = S.lanc_tridiag(v0, n)
            assert ng == nr
            k = min(15, nr)
            np.testing.assert_allclose(a[:k], ar[:k], rtol=1e-10, atol=1e-12)
            np.testing.assert_allclose(b[:k], br[:k], rtol=1e-10, atol=1e-12)
            assert b[0] == 0.0
            e0, vec, nl = S.lanc_eigh(nitermax=min(dim, 512), threshold=1e-12, v0=v0)
            eref, _, _ = lanc_eigh(csr, v0, min(dim, 512))
            exact = _e0_scipy(csr, dim)
            assert abs(e0 - eref) <= 1e-10 * abs(eref)
            assert abs(e0 - exact) <= 1e-9 * abs(exact)
            # Ritz vector: unit norm and small residual
            assert abs(np.linalg.norm(vec) - 1.0) < 1e-10
            res = S.hxv(vec) - e0 * vec if not S.real else None
            assert np.linalg.norm(res) < 1e-5


def test_real_lanczos_c2():
    """configs[1] in real(8): the Lanczos ground state of the half-filled sector."""
    from edgpu.hamiltonian import Sector
    from cases import c2

    cfg = c2()
    with Sector(cfg, 4, 4, stored=True, real=True) as S:
        e0, vec, nl = S.lanc_eigh(nitermax=512, threshold=1e-12)
        assert abs(e0 - (-9.36173525)) < 5e-9          # SURVEY §6 pin (reference run)
        assert vec.dtype == np.float64
    with Sector(cfg, 4, 4, stored=False, direct=True, real=True) as S:
        e1, _, _ = S.lanc_eigh(nitermax=512, threshold=1e-12, vector=False)
        assert abs(e1 - e0) <= 1e-10 * abs(e0)


@pytest.mark.parametrize("path", ["stored_l2", "stored_reg", "stored_kr", "kron_lds", "kron_reg", "kron_kr"])
def test_persistent_matches_multikernel(path):
    """Same start vector, same sector: the two recurrences agree step by step
    (first 40 steps to 1e-9; only the reduction order differs)."""
    from edgpu.hamiltonian import Sector
    from cases import c2

    cfg = c2()
    kw = dict(stored=False, direct=True) if path.startswith("kron") else dict(stored=True)
    opts = {"stored_l2": ("persist_stored",), "kron_lds": ("no_preg",), "stored_reg": ("no_pkron",),
            "kron_reg": ("no_pkron",)}.get(path, ())
    with Sector(cfg, 4, 4, real=True, options=opts, **kw) as S:
        want = {"stored_l2": 0, "stored_reg": 2, "stored_kr": 4, "kron_lds": 1, "kron_reg": 3,
                "kron_kr": 4}[path]
        assert S.lanc_mode(real=True) == want
        v0 = np.sin(np.arange(1, S.dim + 1, dtype=np.float64))
        a1, b1, n1 = S.lanc_tridiag(v0, 60)
        S.set_options(*opts, "no_persist")
        a2, b2, n2 = S.lanc_tridiag(v0, 60)
    assert n1 == n2 == 60
    np.testing.assert_allclose(a1[:40], a2[:40], rtol=1e-9, atol=1e-11)
    np.testing.assert_allclose(b1[:40], b2[:40], rtol=1e-9, atol=1e-11)


def test_c4_half_filled_ground_state_pin():
    """configs[3] half-filled sector at full size: nnz and E0 of the reference
    run through the large-grid (two-pass reduction) recurrence."""
    from edgpu.hamiltonian import Sector
    from edgpu.params import make_config

    cfg = make_config(Norb=2, Nbath=5)
    for kw in (dict(stored=True), dict(stored=False, direct=True)):
        with Sector(cfg, 6, 6, real=True, **kw) as S:
            assert S.dim == 853776
            if kw.get("stored"):
                assert S.nnz == 10167696
            e0, vec, n = S.lanc_eigh(nitermax=512, threshold=1e-12)
            assert abs(e0 - (-14.70964221)) < 5e-9
            assert abs(np.linalg.norm(vec) - 1.0) < 1e-10


@pytest.mark.parametrize("direct", [False, True], ids=["stored", "direct"])
def test_complex_vectors_kronecker_register_layout(direct):
    """The reference's arithmetic — complex(8) vectors — on a real H through
    the Kronecker register layout (persistent MODE 4, 512-thread form):
    alpha/beta (first 15 steps) and E0 against the oracle's complex
    recurrence at 1e-10, and 40 steps against the multi-kernel one at 1e-9."""
    from edgpu.hamiltonian import Sector
    from cases import c2

    cfg = c2()
    orc = Oracle(cfg)
    hmap = orc.build_sector(4, 4)
    csr = orc.build_csr(hmap)
    v0 = start_vector(len(hmap))
    ar, br, nr = lanc_tridiag(csr, v0, 60)
    kw = dict(stored=False, direct=True) if direct else dict(stored=True)
    with Sector(cfg, 4, 4, real=True, **kw) as S:
        assert S.lanc_mode(real=False) == 4
        a, b, n = S.lanc_tridiag(v0, 60, real=False)
        assert n == nr == 60
        np.testing.assert_allclose(a[:15], ar[:15], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(b[:15], br[:15], rtol=1e-10, atol=1e-12)
        e0, vec, _ = S.lanc_eigh(nitermax=512, threshold=1e-12, v0=v0, real=False)
        eref, _, _ = lanc_eigh(csr, v0, 512)
        assert abs(e0 - eref) <= 1e-10 * abs(eref)
        assert vec.dtype == np.complex128 and abs(np.linalg.norm(vec) - 1.0) < 1e-10
        S.set_options("no_persist")
        a2, b2, n2 = S.lanc_tridiag(v0, 60, real=False)
    np.testing.assert_allclose(a[:40], a2[:40], rtol=1e-9, atol=1e-11)
    np.testing.assert_allclose(b[:40], b2[:40], rtol=1e-9, atol=1e-11)


def test_complex_vectors_batched_mode4():
    """Batched complex runs (one workgroup per start vector, MODE 4 complex
    layout) give each run's single-launch alpha/beta."""
    from edgpu.gf import _tridiag_batch
    from edgpu.hamiltonian import Sector
    from cases import c2

    with Sector(c2(), 4, 4, real=True, stored=True) as S:
        assert S.lanc_mode(real=False) == 4
        i = torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda:0")
        seeds = torch.stack([torch.complex(torch.sin(k * i), torch.cos(3 * k * i)) for k in (1, 2, 3)])
        seeds = seeds / seeds.abs().pow(2).sum(1, keepdim=True).sqrt()
        torch.cuda.synchronize()
        a, b, n = _tridiag_batch(S, seeds.contiguous(), 50, False, 0.0)
        for k in range(3):
            a1, b1, n1 = S.lanc_tridiag(seeds[k].cpu().numpy(), 50, 0.0, real=False)
            assert n[k] == n1
            np.testing.assert_array_equal(a[k], a1)
            np.testing.assert_array_equal(b[k], b1)
