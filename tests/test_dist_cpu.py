"""Within-sector split (edgpu.dist) on CPU: the all-to-all transposes and the
split Lanczos on 1/2/3 gloo ranks against the oracle's full-sector CSR."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from edgpu.params import make_config


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cfg():
    return make_config(Norb=1, Nbath=7, bath="random", seed=5)    # c2 family, (4,4): 70 x 70


def test_factors_reproduce_sector():
    from oracle_kron import oracle_factors

    H, D, Hup, Hdw, du, dd = oracle_factors(_cfg(), 4, 4)
    x = np.sin(np.arange(1, du * dd + 1)) + 1j * np.cos(3 * np.arange(1, du * dd + 1))
    X = x.reshape(dd, du)
    y = (D * X + (Hup @ X.T).T + Hdw @ X).reshape(-1)
    assert np.max(np.abs(y - H @ x)) < 1e-12


def test_split_serial_equals_full():
    from oracle_kron import NumpyKronOps, oracle_factors
    from edgpu.dist import DistKronSector

    H, D, Hup, Hdw, du, dd = oracle_factors(_cfg(), 4, 4)
    ds = DistKronSector(ops=NumpyKronOps(D, Hup, Hdw, du, dd))
    x = torch.from_numpy(np.sin(np.arange(1, du * dd + 1)) + 1j * np.cos(3 * np.arange(1, du * dd + 1)))
    y = ds.hxv(x)
    assert np.max(np.abs(y.numpy() - H @ x.numpy())) < 1e-12


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from oracle_kron import NumpyKronOps, oracle_factors
    from edgpu.dist import DistKronSector, dist_lanczos
    from oracle.oracle import lanc_tridiag, Oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = _cfg()
    H, D, Hup, Hdw, du, dd = oracle_factors(cfg, 4, 4)
    ds = DistKronSector(ops=NumpyKronOps(D, Hup, Hdw, du, dd))
    n = du * dd
    i = np.arange(1, n + 1, dtype=np.float64)
    x = torch.from_numpy(np.sin(i) + 1j * np.cos(3 * i))
    y = ds.gather(ds.hxv(ds.scatter(x)))
    err = float(np.max(np.abs(y.numpy() - H @ x.numpy())))
    a, b, nl = dist_lanczos(ds, ds.scatter(x), 40)
    orc = Oracle(cfg)
    hmap = orc.build_sector(4, 4)
    ar, br, nr = lanc_tridiag(orc.build_csr(hmap), x.numpy(), 40)
    q.put((rank, err, float(np.max(np.abs(a[:30] - ar[:30]))), float(np.max(np.abs(b[:30] - br[:30]))), nl, nr,
           ds.local_dim))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_split_matches_full(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sum(o[6] for o in out) == 4900          # the blocks tile the sector
    for rank, err, da, db, nl, nr, _ in out:
        assert err < 1e-12
        assert nl == nr == 40
        assert da < 1e-10 and db < 1e-10


# ---------------------------------------------------------------- row split
def _row_cfg():
    from cases import nonsu2_rand

    return nonsu2_rand()                 # nonsu2 with Jx/Jp and spin flips: no Kronecker form


def test_mpi_split_matches_reference_rule():
    """build_Hv_sector: mpiQ = dim/size rows per rank, remainder on the last
    rank (ED_HAMILTONIAN.f90:55-62)."""
    from edgpu.dist import mpi_split

    assert mpi_split(10, 3) == ([0, 3, 6], [3, 3, 4])
    assert mpi_split(4900, 8)[1][-1] == 4900 // 8 + 4900 % 8


def _row_worker(rank, world, port, q):
    import torch.distributed as dist
    from edgpu.dist import DistRowSector, dist_lanczos
    from oracle.oracle import Oracle, lanc_tridiag

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = _row_cfg()
    orc = Oracle(cfg)
    hmap = orc.build_sector(6, 0)
    rp, cols, vals = orc.build_csr(hmap)
    import scipy.sparse as sp

    n = len(hmap)
    H = sp.csr_matrix((vals, cols, rp), shape=(n, n))
    from edgpu.dist import mpi_split

    r0, cnt = mpi_split(n, world)
    Hloc = H[r0[rank]:r0[rank] + cnt[rank]]
    rows = lambda v: torch.from_numpy(Hloc @ v.numpy())    # noqa: E731
    ds = DistRowSector(hxv_rows=rows, dim=n, cols_needed=Hloc.indices)            # halo exchange
    full = DistRowSector(hxv_rows=rows, dim=n, halo=False)                        # Allgatherv
    i = np.arange(1, n + 1, dtype=np.float64)
    x = torch.from_numpy(np.sin(i) + 1j * np.cos(3 * i))
    yl = ds.hxv(ds.scatter(x))
    assert torch.equal(yl, full.hxv(full.scatter(x)))        # bit-identical to the Allgatherv product
    assert ds.halo_size < n - cnt[rank]                      # fewer entries than the whole vector
    y = ds.gather(yl)
    err = float(np.max(np.abs(y.numpy() - H @ x.numpy())))
    a, b, nl = dist_lanczos(ds, ds.scatter(x), 40)
    ar, br, nr = lanc_tridiag((rp, cols, vals), x.numpy(), 40)
    q.put((rank, err, float(np.max(np.abs(a[:30] - ar[:30]))), float(np.max(np.abs(b[:30] - br[:30]))), nl, nr,
           ds.local_dim))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_row_split_matches_full(world):
    """spMatVec_mpi_cc semantics on `world` gloo ranks: local rows, the halo
    exchange (bit-identical to the Allgatherv of the vector), distributed plain
    Lanczos."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_row_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle.oracle import Oracle

    dim = len(Oracle(_row_cfg()).build_sector(6, 0))
    assert sum(o[6] for o in out) == dim
    for rank, err, da, db, nl, nr, _ in out:
        assert err < 1e-12
        assert nl == nr == 40
        assert da < 1e-10 and db < 1e-10
