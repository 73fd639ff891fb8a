"""Within-sector split H·v (ed_sector_kron_rows/_cols + all-to-all transposes,
edgpu.dist) on the GPU against the single-GPU Kronecker kernel: 1e-13
relative (only the association of the up and down partial sums differs)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from edgpu.params import make_config

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max())


@pytest.mark.parametrize("kw,q", [
    (dict(Norb=1, Nbath=7, bath="random", seed=5), (4, 4)),
    (dict(Norb=1, Nbath=9, bath="random", seed=4), (5, 5)),
    (dict(Norb=2, Nbath=3, Uloc=(2.0, 1.5, 0.0), Ust=1.0, Jh=0.3, bath="random", seed=7), (4, 3)),
])
@pytest.mark.parametrize("cplx", [False, True])
def test_split_serial_matches_kron(kw, q, cplx):
    from edgpu.dist import DistKronSector, dist_lanczos
    from edgpu.hamiltonian import Sector

    cfg = make_config(**kw)
    ds = DistKronSector(cfg, *q)
    with Sector(cfg, *q, stored=False, direct=True, real=True) as S:
        n = S.dim
        i = torch.arange(1, n + 1, dtype=torch.float64, device="cuda")
        x = torch.complex(torch.sin(i), torch.cos(3 * i)) if cplx else torch.sin(i)
        y0 = torch.empty_like(x)
        S.hxv_dev(x, y0, path=2)
        y = ds.hxv(x)
        torch.cuda.synchronize()
        assert _rel(y, y0) < 1e-13
        if not cplx:
            a, b, nl = dist_lanczos(ds, x, 30)
            ar, br, nr = S.lanc_tridiag(x.cpu().numpy(), 30)
            assert nl == nr
            np.testing.assert_allclose(a[:20], ar[:20], rtol=1e-10, atol=1e-12)
    ds.close()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "dmft-ed_amd")]
    import torch.distributed as dist
    from edgpu.dist import DistKronSector
    from edgpu.hamiltonian import Sector

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)                       # both ranks share the box's one GPU
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = make_config(Norb=1, Nbath=9, bath="random", seed=4)
    ds = DistKronSector(cfg, 5, 5)
    with Sector(cfg, 5, 5, stored=False, direct=True, real=True) as S:
        i = torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda")
        x = torch.sin(i)
        y0 = torch.empty_like(x)
        S.hxv_dev(x, y0, path=2)
        y = ds.gather(ds.hxv(ds.scatter(x)))
        torch.cuda.synchronize()
        q.put((rank, _rel(y, y0), ds.local_dim))
    ds.close()
    dist.barrier()
    dist.destroy_process_group()


def test_split_two_ranks_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sum(o[2] for o in out) == 252 * 252
    assert all(o[1] < 1e-13 for o in out)


# ---------------------------------------------------------------- row split
@pytest.mark.parametrize("name", ["nonsu2_rand", "superc_2orb", "normal_jh", "nonsu2_jz"])
@pytest.mark.parametrize("stored", [True, False])
def test_row_sectors_match_oracle(name, stored):
    """ed_sector_create_rows: every row block of H·v equals the oracle's
    spMatVec_cc rows bit for bit (stored) / to 1e-13 (matrix-free generic)."""
    import cases
    from edgpu.dist import mpi_split
    from edgpu.hamiltonian import Sector
    from oracle.oracle import Oracle, spmv, start_vector

    cfg = getattr(cases, name)()
    q = [c for c in cases.CASES if c[0] == name][0][2][0]
    orc = Oracle(cfg)
    hmap = orc.build_sector(*q)
    csr = orc.build_csr(hmap)
    n = len(hmap)
    x = start_vector(n)
    ref = spmv(csr, x)
    xd = torch.from_numpy(x).cuda()
    r0, cnt = mpi_split(n, 3)
    parts = []
    for a, c in zip(r0, cnt):
        with Sector(cfg, *q, stored=stored, direct=not stored, rows=(a, c)) as S:
            assert (S.row0, S.nrows, S.dim) == (a, c, n)
            y = torch.empty(c, dtype=torch.complex128, device="cuda")
            S.hxv_dev(xd, y)
            if stored:
                rp, cols, vals = S.dump_csr()
                assert rp[-1] == csr[0][a + c] - csr[0][a]
                assert np.array_equal(cols, csr[1][csr[0][a]:csr[0][a + c]])
            parts.append(y.cpu().numpy())
    y = np.concatenate(parts)
    if stored:
        assert np.array_equal(y, ref)
    else:
        assert np.max(np.abs(y - ref)) <= 1e-13 * np.max(np.abs(ref))


def test_row_sector_refuses_whole_sector_calls():
    from edgpu._lib import EDGPUError
    from edgpu.hamiltonian import Sector

    cfg = make_config(Norb=1, Nbath=5)
    with Sector(cfg, 3, 3, stored=True, rows=(0, 100)) as S:
        with pytest.raises(EDGPUError, match="row-split"):
            S.lanc_eigh(nitermax=50, threshold=1e-12)


def _row_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "dmft-ed_amd"), os.path.join(root, "tests")]
    import torch.distributed as dist
    from cases import nonsu2_rand
    from edgpu.dist import DistRowSector, dist_lanczos
    from oracle.oracle import Oracle, lanc_tridiag, spmv, start_vector

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)                       # both ranks share the box's one GPU
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = nonsu2_rand()
    ds = DistRowSector(cfg, 6, 0)
    orc = Oracle(cfg)
    csr = orc.build_csr(orc.build_sector(6, 0))
    x = start_vector(ds.dim)
    y = ds.gather(ds.hxv(ds.scatter(torch.from_numpy(x).cuda())))
    exact = bool(np.array_equal(y.cpu().numpy(), spmv(csr, x)))
    a, b, nl = dist_lanczos(ds, ds.scatter(torch.from_numpy(x).cuda()), 30)
    ar, br, nr = lanc_tridiag(csr, x, 30)
    q.put((rank, exact, float(np.max(np.abs(a[:20] - ar[:20]))), nl, nr, ds.local_dim))
    ds.close()
    dist.barrier()
    dist.destroy_process_group()


def test_row_split_two_ranks_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_row_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, exact, da, nl, nr, _ in out:
        assert exact and nl == nr == 30 and da < 1e-10


def test_empty_row_range():
    """A rank with no rows (dim < MpiSize in build_Hv_sector's split): the
    sector builds, vecDim is 0 and H·v is a no-op (spMatVec_mpi_cc with Nloc=0)."""
    import torch

    from edgpu.hamiltonian import Sector
    from edgpu.params import make_config

    cfg = make_config(Norb=1, Nbath=3)
    for stored in (True, False):
        with Sector(cfg, 0, 0, stored=stored, direct=not stored, rows=(0, 0)) as S:
            assert S.nrows == 0 and S.dim == 1
            x = torch.ones(S.dim, dtype=torch.complex128, device="cuda:0")
            y = torch.empty(0, dtype=torch.complex128, device="cuda:0")
            S.hxv_dev(x, y)
            torch.cuda.synchronize()
            if stored:
                rp, cols, vals = S.dump_csr()
                assert list(rp) == [0] and len(cols) == 0
