"""Benchmark of the Lanczos H·v hot path (BASELINE.json metric:
"Lanczos SpMV GB/s + ground-state iters/s, Ns=16 half-filled sector, 1/2/4/8 GPU").

Workload (configs[1]): Norb=1, Nbath=7 (reference Nlevels=16), half-filled
sector (nup,ndw)=(4,4), dim 4,900, stored H in real(8), synthetic random bath
(seeded per rank).  One step = one device-resident plain-Lanczos run of
`--niter` iterations (lanc_niter=512 by default) from a fixed start vector.
value = Lanczos iterations/s summed over all ranks (weak scaling: every rank
runs its own sector replica; sectors are independent, no collective in the
data path).

Also reported (rank 0):
  * spmv_gbs: stored SpMV GB/s on the c2 sector (algorithmic bytes, L2-resident);
  * roofline: stored SpMV on the Nlevels=28 (7,7) sector (dim 11,778,624,
    nnz 176,679,360, real(8)) — the only size where HBM is the bound
     — timed with HIP events on the launch stream;
  * cpu_baseline: the oracle's row-gather CSR SpMV + plain recurrence
    (restated reference algorithm), 1 host core, bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "dmft-ed_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def spmv_bytes_real(nnz, dim):
    """Algorithmic bytes of one real(8) stored SpMV in the reference's CSR form
    (SURVEY §8d): 12 nnz + 8 (dim+1) + 16 dim."""
    return 12 * nnz + 8 * (dim + 1) + 16 * dim


def spmv_bytes_packed(padded, dim):
    """Algorithmic bytes of one packed SELL-64 SpMV (k_spmv_pk): 4-B words per
    slot, slice pointers, real(8) diagonal, read v, write Hv."""
    nslice = (dim + 63) // 64
    return 4 * padded + 8 * (nslice + 1) + 8 * dim + 16 * dim


def time_kernel(fn, iters, stream):
    """Average device time (ms) of fn() over iters launches, HIP events on `stream`."""
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def measure_spmv(Sector, cfg, q, iters, warm=5, info=None):
    with Sector(cfg, q[0], q[1], stored=True, direct=False, real=True) as S:
        dim, nnz = S.dim, S.nnz
        if info is not None:
            info.update(packed=int(S.info.packed), padded=int(S.info.padded), npdict=int(S.info.npdict))
        x = torch.sin(torch.arange(1, dim + 1, dtype=torch.float64, device="cuda")).contiguous()
        y = torch.empty_like(x)
        st = torch.cuda.current_stream()
        for _ in range(warm):
            S.hxv_dev(x, y, path=0, stream=st)
        ms = time_kernel(lambda: S.hxv_dev(x, y, path=0, stream=st), iters, st)
        return dim, nnz, ms


def cpu_baseline(budget_s=10.0):
    """Oracle (restated reference loops) on 1 host core: plain Lanczos iters/s on c2."""
    from edgpu.params import make_config
    from oracle.oracle import Oracle, lanc_tridiag, start_vector

    cfg = make_config(Norb=1, Nbath=7, bath="random", seed=20251015)
    orc = Oracle(cfg)
    hmap = orc.build_sector(4, 4)
    csr = orc.build_csr(hmap)
    v0 = start_vector(len(hmap))
    n = 200
    t0 = time.perf_counter()
    runs = 0
    while time.perf_counter() - t0 < budget_s:
        lanc_tridiag(csr, v0, n, threshold=0.0)
        runs += 1
    dt = time.perf_counter() - t0
    return {"value": runs * n / dt, "unit": "Lanczos iters/s", "cores": 1, "kind": "port",
            "sample": f"{runs} x {n}-step plain-Lanczos runs (complex(8), row-gather CSR, "
                      f"c2 (4,4) sector, random bath) in {dt:.1f}s on 1 core"}


def _timed(dist, fn):
    """Barrier-bracketed wall time of fn(), max over ranks."""
    import torch.distributed as tdist

    def barrier():
        if dist:
            tdist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    r = fn()
    barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = float(t.item())
    return dt, r


def bench_farm(dist, world, dev):
    """configs[3]: all 169 (Nup,Ndw) sectors of Norb=2 Nbath=5 (Nlevels=24) through
    ed_diag's default path (dense <= 256, device thick-restart Lanczos for the 6
    lowest otherwise), sectors farmed over the ranks (LPT), one all_gather of
    eigenvalues.  Strong scaling: the same job on 1/2/4/8 GPUs."""
    from edgpu.diag import DiagOptions
    from edgpu.farm import farm_diag
    from edgpu.params import make_config

    cfg = make_config(Norb=2, Nbath=5, bath="random", seed=20251015)
    opt = DiagOptions()
    farm_diag(cfg, opt, device=dev)        # warm-up (code objects, allocator)
    dt, res = _timed(dist, lambda: farm_diag(cfg, opt, device=dev))
    nloc = len(res.local)
    return {"wall_s": round(dt, 4), "sectors": len(res.eigenvalues), "n_gpus": world,
            "E0": round(float(res.states.emin), 10), "gs_states": res.states.size,
            "rank0_sectors": nloc, "scaling": "strong",
            "workload": "configs[3]: Norb=2 Nbath=5 random bath, all sectors, lanc_method=arpack "
                        "(Neigen=6, ncv=23) on device"}


def bench_nonsu2(dist, world, dev):
    """configs[4]: nonSU2 Norb=1 Nbath=6 (Nlevels=14): complex ground state over
    all sectors + the Green's function (diagonal + spin-mixed seeds, 200-step
    Lanczos each, Lmats=Lreal=5000), seeds farmed over the ranks."""
    from edgpu.diag import DiagOptions
    from edgpu.farm import farm_diag
    from edgpu.gf import GFOptions, _job_list, build_gf
    from edgpu.params import make_config

    cfg = make_config(Norb=1, Nbath=6, Nspin=2, ed_mode="nonsu2", bath="random", seed=20251015)
    opt = DiagOptions()
    gopt = GFOptions()
    res = farm_diag(cfg, opt, device=dev)
    build_gf(cfg, res.states, gopt, device=dev, owners=res.owners)   # warm-up
    t_diag, res = _timed(dist, lambda: farm_diag(cfg, opt, device=dev))
    t_gf, (Gm, _) = _timed(dist, lambda: build_gf(cfg, res.states, gopt, device=dev, owners=res.owners))
    return {"diag_s": round(t_diag, 4), "gf_s": round(t_gf, 4), "n_gpus": world,
            "gf_seeds": len(_job_list(cfg, res.states)[0]), "E0": round(float(res.states.emin), 10),
            "G_iw0_00": [round(float(Gm[0, 0, 0, 0, 0].real), 10), round(float(Gm[0, 0, 0, 0, 0].imag), 10)],
            "workload": "configs[4]: nonSU2 Norb=1 Nbath=6 random bath, default (arpack) GS over all sectors "
                        "+ build_gf (diag + mixed seeds, nGFiter=200, L=5000)"}


def bench_split(dist, world, dev, iters=10):
    """one Nlevels=28 (7,7) sector split by down rows over all
    ranks; H·v = local Kronecker rows + all-to-all transpose + columns +
    all-to-all back (edgpu.dist).  Strong scaling of a single H·v."""
    from edgpu.dist import DistKronSector
    from edgpu.params import make_config

    cfg = make_config(Norb=1, Nbath=13, bath="random", seed=20251015)
    ds = DistKronSector(cfg, 7, 7, device=dev, real=True)
    w0, nw = ds.local_rows
    i = torch.arange(w0 * ds.du + 1, (w0 + nw) * ds.du + 1, dtype=torch.float64, device="cuda")
    x = torch.sin(i)
    for _ in range(2):
        ds.hxv(x)
    dt, _ = _timed(dist, lambda: [ds.hxv(x) for _ in range(iters)])
    ds.close()
    return {"ms_per_hxv": round(dt / iters * 1e3, 4), "n_gpus": world, "scaling": "strong",
            "dim": ds.du * ds.dd, "local_rows": nw,
            "workload": "Nlevels=28 Norb=1 Nbath=13 (7,7) sector split by down rows; Kronecker rows/cols "
                        "kernels + 2 all_to_all exchanges per H·v (RCCL; strip layout, no transposes)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--niter", type=int, default=512)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-farm", action="store_true", help="skip the configs[3]/[4] sections")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # rehearsal switches (not used by the driver): ED_BENCH_BACKEND=gloo and
        # ED_BENCH_ONE_DEVICE=1 run N ranks on one GPU to exercise the N>1 flow
        if os.environ.get("ED_BENCH_ONE_DEVICE"):
            local = 0
        torch.cuda.set_device(local)
        backend = os.environ.get("ED_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    from edgpu.hamiltonian import Sector
    from edgpu.params import make_config

    cfg = make_config(Norb=1, Nbath=7, bath="random", seed=20251015 + rank)
    S = Sector(cfg, 4, 4, stored=True, direct=False, real=True, device=dev)
    v0 = torch.sin(torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda"))

    def step():
        return S.lanc_run(args.niter, v0_dev=v0)

    for _ in range(args.warmup):
        step()

    def barrier():
        if dist:
            tdist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    dev_ms = 0.0
    for _ in range(args.steps):
        _, _, ms = step()
        dev_ms += ms
    barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = float(t.item())
    iters_total = args.steps * args.niter * world
    value = iters_total / dt

    # configs[2]: the same sector through the matrix-free kernel (rank-local, untimed by the
    # barrier bracket above; device time of the same 512-iteration runs)
    Sd = Sector(cfg, 4, 4, stored=False, direct=True, real=True, device=dev)
    for _ in range(2):
        Sd.lanc_run(args.niter, v0_dev=v0)
    dms = [Sd.lanc_run(args.niter, v0_dev=v0)[2] for _ in range(5)]
    direct_ips = args.niter / (min(dms) * 1e-3)
    Sd.close()

    split = None if args.no_farm else bench_split(dist, world, dev)
    farm = None if args.no_farm else bench_farm(dist, world, dev)
    nonsu2 = None if args.no_farm else bench_nonsu2(dist, world, dev)

    out = None
    if rank == 0:
        # SpMV GB/s on the headline sector (L2-resident; launch-latency bound)
        dim2, nnz2, ms2 = measure_spmv(Sector, cfg, (4, 4), 2000)
        gbs2 = spmv_bytes_real(nnz2, dim2) / (ms2 * 1e-3) / 1e9
        roof = None
        if not args.no_roofline:
            cfg28 = make_config(Norb=1, Nbath=13, bath="random", seed=20251015)
            inf28 = {}
            dim28, nnz28, ms28 = measure_spmv(Sector, cfg28, (7, 7), 50, info=inf28)
            # achieved: SURVEY §8(d)'s algorithmic bytes for this unit (real(8) CSR
            # stored SpMV).  The packed form moves fewer bytes, so this may exceed
            # the physical rate; `traffic` is the PMC-measured HBM
            # side and own_format_bytes the packed kernel's own algorithmic bytes.
            B = spmv_bytes_real(nnz28, dim28)
            Bown = spmv_bytes_packed(inf28["padded"], dim28) if inf28["packed"] else B
            ach = B / (ms28 * 1e-3) / 1e9
            traffic, tsrc = None, None
            tfile = os.path.join(ROOT, "profiles", "r1", "spmv_n28_traffic.json")
            if os.path.exists(tfile):   # PMC bytes cannot be read in-process: rocprofv3 passes
                with open(tfile) as fh:
                    tj = json.load(fh)
                if bool(tj.get("packed", False)) == bool(inf28["packed"]):   # same kernel only
                    traffic = tj["traffic_bytes_per_launch"]
                    tsrc = ("profiles/r1/spmv_n28_traffic.json (rocprofv3 FETCH_SIZE/WRITE_SIZE "
                            "passes, same kernel+sector)")
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "traffic_source": tsrc,
                    "achieved_basis": "SURVEY §8(d) real(8) stored SpMV bytes 12*nnz+8*(dim+1)+16*dim",
                    "kernel": ("k_spmv_pk<real> (stored SELL-64, 32-bit {col|value index} words, "
                               f"{inf28['npdict']}-value dictionary)") if inf28["packed"]
                              else "k_spmv<real,real> (stored SELL-64 H·v)",
                    "workload": f"Nlevels=28 Norb=1 Nbath=13 (7,7) sector, dim {dim28}, nnz {nnz28}, "
                                f"real(8), {B} algorithmic bytes/launch",
                    "ms_per_launch": round(ms28, 4),
                    "own_format_bytes": Bown,
                    "own_format_gbs": round(Bown / (ms28 * 1e-3) / 1e9, 1),
                    "physical_gbs": round(traffic / (ms28 * 1e-3) / 1e9, 1) if traffic else None}
        cpu = None if args.no_cpu else cpu_baseline()
        out = {
            "metric": "Lanczos SpMV GB/s + ground-state iters/s, Ns=16 half-filled sector, 1/2/4/8 GPU",
            "value": round(value, 1),
            "unit": "Lanczos iters/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded random bath per rank)",
            "config": {"workload": "c2: Norb=1 Nbath=7 (Nlevels=16) half-filled (4,4) sector, dim 4900, "
                                   f"stored real(8) H, plain Lanczos {args.niter} iters/step",
                       "parallelism": f"sector replicas x{world}"},
            "device_ms_per_step": round(dev_ms / args.steps, 4),
            "direct_iters_per_s": round(direct_ips, 1),
            "direct_note": "configs[2]: same sector, matrix-free H·v (Kronecker form, tables in LDS), one GPU",
            "spmv_gbs_c2": round(gbs2, 1),
            "spmv_ms_c2": round(ms2, 5),
            "farm_c4": farm,
            "split_n28": split,
            "nonsu2_c5": nonsu2,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    S.close()
    if dist:
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
