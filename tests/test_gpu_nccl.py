"""The RCCL (backend "nccl") branches of the multi-GPU code, run for real.

The box has one GPU and RCCL refuses two ranks on one device, so this runs a
world_size-1 process group over RCCL: every collective the farms and the
within-sector split issue (all_gather_object, broadcast of device tensors,
all_to_all_single, all_gather, all_reduce) goes through RCCL with the device
tensors, dtypes and shapes the N-GPU run uses, and each result must equal the
run without a process group (the gloo world_size-2 tests cover the data
movement between ranks).  Reference: ED_DIAG.f90:71-249 (sector loop),
ED_GF_NORMAL.f90:132-258 / ED_GF_NONSU2.f90:28-55 (seeds),
ED_HAMILTONIAN_STORED_HxV.f90:147-197 (row split + Allgatherv).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


def _worker(port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "dmft-ed_amd"), os.path.join(root, "tests")]
    import torch.distributed as dist
    from edgpu.diag import DiagOptions, to_host
    from edgpu.dist import DistKronSector, DistRowSector, dist_lanczos
    from edgpu.farm import broadcast_vector, farm_diag
    from edgpu.gf import GFOptions, build_gf
    from edgpu.hamiltonian import Sector
    from edgpu.params import make_config

    out = {}
    torch.cuda.set_device(0)
    # serial results first (no process group)
    cfgs = {"normal": make_config(Norb=1, Nbath=5, bath="random", seed=5),
            "nonsu2": make_config(Norb=1, Nbath=3, Nspin=2, ed_mode="nonsu2", bath="random", seed=2)}
    gopt = GFOptions(Lmats=64, Lreal=64)
    serial = {}
    for k, cfg in cfgs.items():
        res = farm_diag(cfg, DiagOptions(lanc_method="lanczos"))
        Gm, Gr = build_gf(cfg, res.states, gopt)
        serial[k] = (res.states.energies, res.states.sectors, to_host(res.states.vectors[0]), Gm, Gr)
    kcfg = make_config(Norb=1, Nbath=9, bath="random", seed=4)
    with Sector(kcfg, 5, 5, stored=False, direct=True, real=True) as S:
        i = torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda")
        xk = torch.sin(i)
        yk = torch.empty_like(xk)
        S.hxv_dev(xk, yk, path=2)
        ak, bk, nk = S.lanc_tridiag(xk.cpu().numpy(), 30)
    rcfg = cfgs["nonsu2"]
    with Sector(rcfg, 6, 0, stored=True, real=rcfg.is_real()) as S:
        i = torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda")
        xr = torch.complex(torch.sin(i), torch.cos(3 * i))
        yr = torch.empty_like(xr)
        S.hxv_dev(xr, yr)

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    out["backend"] = dist.get_backend()
    for k, cfg in cfgs.items():
        res = farm_diag(cfg, DiagOptions(lanc_method="lanczos"))
        en, secs, v0, Gm0, Gr0 = serial[k]
        vb = broadcast_vector(res.states.vectors[0], res.owners[0], len(v0), bool(np.iscomplexobj(v0)))
        Gm, Gr = build_gf(cfg, res.states, gopt, owners=res.owners)
        out[k] = {"secs": res.states.sectors == secs,
                  "en": float(np.max(np.abs(np.asarray(res.states.energies) - np.asarray(en)))),
                  "vb_dev": bool(torch.is_tensor(vb) and vb.is_cuda),
                  "vb": float(np.max(np.abs(vb.cpu().numpy() - v0))),
                  "gm": _rel(Gm, Gm0), "gr": _rel(Gr, Gr0)}
    ds = DistKronSector(kcfg, 5, 5)
    y = ds.gather(ds.hxv(ds.scatter(xk)))
    a, b, n = dist_lanczos(ds, ds.scatter(xk), 30)
    out["kron"] = {"rel": float((y - yk).abs().max() / yk.abs().max()), "n": n == nk,
                   "alpha": float(np.max(np.abs(np.asarray(a[:20]) - ak[:20])))}
    ds.close()
    dr = DistRowSector(rcfg, 6, 0)
    y = dr.gather(dr.hxv(dr.scatter(xr)))
    out["rows"] = {"exact": bool(torch.equal(y, yr))}
    dr.close()
    dist.barrier()
    dist.destroy_process_group()
    q.put(out)


def test_rccl_world1_paths_match_serial():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_port(), q))
    p.start()
    out = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert out["backend"] == "nccl"
    for k in ("normal", "nonsu2"):
        r = out[k]
        assert r["secs"] and r["en"] <= 1e-12, r
        assert r["vb_dev"] and r["vb"] == 0.0, r          # device tensor, delivered unchanged
        assert r["gm"] < 1e-12 and r["gr"] < 1e-12, r
    assert out["kron"]["rel"] < 1e-13 and out["kron"]["n"] and out["kron"]["alpha"] < 1e-10, out["kron"]
    assert out["rows"]["exact"], out["rows"]
