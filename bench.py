"""Benchmark of the Lanczos H·v hot path (BASELINE.json metric:
"Lanczos SpMV GB/s + ground-state iters/s, Ns=16 half-filled sector, 1/2/4/8 GPU").

Workload (configs[1]): Norb=1, Nbath=7 (reference Nlevels=16), half-filled
sector (nup,ndw)=(4,4), dim 4,900, stored H in real(8), synthetic random bath
(seeded per rank).  One step = one device-resident plain-Lanczos run of
`--niter` iterations (lanc_niter=512 by default) from a fixed start vector.
value = Lanczos iterations/s summed over all ranks (weak scaling: every rank
runs its own sector replica; sectors are independent, no collective in the
data path).  The timed runs take persistent MODE 4: one workgroup holds the
stored matrix's entries in the Kronecker register layout (the stored SELL
matrix has the form D + Hup(x)1 + 1(x)Hdw; its values, read back from the
device matrix, sit in registers — DESIGN.md §1).  Beside it:
  * stored_mode2_iters_per_s: the same sector with the stored matrix as ELL
    words in registers (MODE 2, no Kronecker structure used);
  * direct_iters_per_s: configs[2], matrix-free tables (MODE 4 from the hop
    tables);
  * complex_iters_per_s: complex(8) vectors (the reference's arithmetic) on the
    real(8) stored values of the same H (persistent MODE 4, 512-thread complex
    register layout by default); complex_h_iters_per_s: complex(8) H values and
    vectors (MODE 2);
  * validation: the lowest Ritz value of the last timed run's tridiagonal
    against the committed oracle E0 (tests/golden/c2_e0.json) at 1e-10.
Sections (rank 0 prints, all ranks take part):
  * farm_c4 (configs[3]), nonsu2_c5 (configs[4]) — asserted against the
    committed oracle fixtures tests/golden/c4_diag_random.json /
    c5_gf_random.npz;
  * roofline: stored SpMV on the Nlevels=28 (7,7) sector (dim 11,778,624), the
    only size where HBM is the bound, HIP events on the launch
    stream; frac on the bytes the timed kernel moves;
  * kron_n28: the matrix-free two-pass Kronecker H·v on the same sector;
  * cpu_baseline: the oracle's row-gather CSR + plain recurrence (restated
    reference loops, complex(8)) on 1 host core and on P processes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "dmft-ed_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
GOLD = os.path.join(ROOT, "tests", "golden")
PROFILES = [os.path.join(ROOT, "profiles", r) for r in ("r6", "r5", "r4", "r3")]  # newest summary first


def spmv_bytes_real(nnz, dim):
    """SURVEY §8(d) real(8) stored SpMV bytes in the reference's CSR form:
    12 nnz + 8 (dim+1) + 16 dim."""
    return 12 * nnz + 8 * (dim + 1) + 16 * dim


def spmv_bytes_packed(padded, dim):
    """Bytes the packed SELL-64 kernel (k_spmv_pk) moves: 4-B words per slot,
    slice pointers, real(8) diagonal, read v, write Hv."""
    nslice = (dim + 63) // 64
    return 4 * padded + 8 * (nslice + 1) + 8 * dim + 16 * dim


def time_kernel(fn, iters, stream, batch=False):
    """Average device time (ms) of one fn() launch: each of `iters` launches
    bracketed by its own pair of HIP events on `stream` — the per-dispatch
    duration a rocprofv3 kernel trace reports (back-to-back launches timed
    as one batch overlap each other's ramp and tail: ~3 % lower on the N28
    stored kernel), so the line's ms can be checked against profiles/."""
    if batch:  # (microsecond kernels: one event pair around the whole batch)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(iters):
            fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / iters
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for b, e in ev:
        b.record(stream)
        fn()
        e.record(stream)
    ev[-1][1].synchronize()
    return sum(b.elapsed_time(e) for b, e in ev) / iters


def spmv_bytes_packed_complex(padded, dim):
    """Bytes of k_spmv_pk on complex(8) H and vectors: 4-B words per slot,
    slice pointers, complex(8) diagonal, read v, write Hv (16 B each)."""
    nslice = (dim + 63) // 64
    return 4 * padded + 8 * (nslice + 1) + 16 * dim + 32 * dim


def spmv_bytes_fused(inf, dim, cplx):
    """Bytes the fused one-pass re-laid stored H·v (k_spmv_fu) moves: the
    re-laid matrix (4-B A and L words, 8-B U entries, 40-B unit descriptors),
    the diagonal (8 B real H, 16 B complex), read v and write Hv (8 or 16 B)."""
    hd = 8 if inf["real_h"] else 16
    vb = 16 if cplx else 8
    return inf["fused_bytes"] + hd * dim + 2 * vb * dim


def spmv_bytes_split(inf, dim):
    """Bytes the two-segment stored H·v (k_spmv_sa + k_spmv_sb) moves: the
    re-laid matrix (4-B A words, 8-B U entries, 4-B L words, A slice pointers),
    segment B's work list and slice table, and 48·dim of vectors — A reads the
    diagonal and v, writes y; B reads y and v, writes Hv (v is read by both
    passes: every byte of both passes counted)."""
    return inf["split_bytes"] + inf["split_list_bytes"] + 48 * dim


def measure_hxv(Sector, cfg, q, iters, path=0, warm=5, info=None, cplx=False, batch=False, options=(),
                real_h=None):
    """Average ms per H·v launch.  cplx: complex(8) vectors, and complex(8) H
    values unless real_h=True (complex vectors on the real H)."""
    stored = path == 0
    real = (not cplx) if real_h is None else real_h
    with Sector(cfg, q[0], q[1], stored=stored, direct=not stored, real=real, options=options) as S:
        dim, nnz = S.dim, S.nnz
        if info is not None:
            exact = "stored_exact" in options
            fused = int(S.info.fused) if (stored and not exact and "no_fused" not in options) else 0
            info.update(packed=int(S.info.packed), padded=int(S.info.padded), npdict=int(S.info.npdict),
                        split=int(S.info.split) if (stored and not cplx and not exact) else 0,
                        split_bytes=int(S.info.split_bytes), split_list_bytes=int(S.info.split_list_bytes),
                        split_far=int(S.info.split_far), split_far_uniform=int(S.info.split_far_uniform),
                        fused=fused if (cplx or not S.info.split) else 0, fused_bytes=int(S.info.fused_bytes),
                        fused_far=int(S.info.fused_far), fused_far_uniform=int(S.info.fused_far_uniform),
                        real_h=int(real))
        i = torch.arange(1, dim + 1, dtype=torch.float64, device="cuda")
        x = (torch.complex(torch.sin(i), torch.cos(3 * i)) if cplx else torch.sin(i)).contiguous()
        y = torch.empty_like(x)
        st = torch.cuda.current_stream()
        for _ in range(warm):
            S.hxv_dev(x, y, path=path, stream=st)
        ms = time_kernel(lambda: S.hxv_dev(x, y, path=path, stream=st), iters, st, batch=batch)
        return dim, nnz, ms


def _cpu_worker(args):
    seed, n, budget = args
    from golden.golden_configs import c2_config
    from oracle.oracle import Oracle, lanc_tridiag, start_vector

    orc = Oracle(c2_config("random", seed))
    hmap = orc.build_sector(4, 4)
    csr = orc.build_csr(hmap)
    v0 = start_vector(len(hmap))
    t0 = time.perf_counter()
    runs = 0
    while time.perf_counter() - t0 < budget:
        lanc_tridiag(csr, v0, n, threshold=0.0)
        runs += 1
    return runs * n, time.perf_counter() - t0


def cpu_baseline(budget_s=8.0):
    """The oracle (restated reference loops: complex(8) row-gather CSR
    spMatVec_cc + the .repo/PLAIN_LANCZOS.f90 recurrence) on the host cores:
    1 process, then P independent processes each on its own c2 replica (the
    CPU analogue of the GPU's sector replicas).  P = the host CPUs this job
    may use, capped at 16 (one GPU's share of the box)."""
    from multiprocessing import get_context

    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    P = max(1, min(16, ncpu))
    it1, dt1 = _cpu_worker((20251015, 200, budget_s))
    with get_context("spawn").Pool(P) as pool:
        res = pool.map(_cpu_worker, [(20251015 + r, 200, budget_s) for r in range(P)])
    itp = sum(r[0] / r[1] for r in res)
    return {"value": round(itp, 1), "unit": "Lanczos iters/s", "cores": P, "kind": "port",
            "single_core": {"value": round(it1 / dt1, 1), "cores": 1},
            "sample": f"c2 (4,4) sector, random bath, 200-step plain-Lanczos runs, complex(8) H and vectors "
                      f"(the reference's arithmetic); 1 process for {dt1:.1f}s, then {P} processes x {budget_s:.0f}s "
                      f"(one replica each, iters/s summed)",
            "note": "the port is a C restatement of the reference loops; the reference's own Fortran "
                    "(amdflang -O3, 1 core of the CPU container) ran 5,409 it/s on this sector "
                    "(SURVEY §6, BASELINE.md), ~3.9x below the port's single-core rate"}


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
    """configs[3]: all 169 (Nup,Ndw) sectors of Norb=2 Nbath=5 through ed_diag's
    default path (dense <= 256, device thick-restart Lanczos for the 6
    lowest otherwise), sectors farmed over the ranks (LPT), one all_gather of
    eigenvalues.  Strong scaling: the same job on 1/2/4/8 GPUs.  The result is
    checked against the committed oracle fixture."""
    from edgpu.diag import DiagOptions
    from edgpu.farm import farm_diag
    from golden.golden_configs import c4_config

    cfg = c4_config("random")
    opt = DiagOptions()
    farm_diag(cfg, opt, device=dev)        # warm-up (code objects, allocator)
    dt, res = _timed(dist, lambda: farm_diag(cfg, opt, device=dev))
    with open(os.path.join(GOLD, "c4_diag_random.json")) as fh:
        gold = json.load(fh)
    worst = max(float(np.max(np.abs(np.asarray(res.eigenvalues[int(k)])[: len(g["eigenvalues"])]
                                    - np.asarray(g["eigenvalues"])))) for k, g in gold["sectors"].items())
    worst /= abs(gold["E0"])
    e0_dev = abs(res.states.emin - gold["E0"]) / abs(gold["E0"])
    assert e0_dev < 1e-10 and worst < 1e-10 and res.states.sectors == gold["states"]["sectors"], \
        f"farm_c4 differs from the oracle fixture: E0 {e0_dev:.2e}, eigenvalues {worst:.2e}"
    # north_star's ">= 6x near-linear 1->8-GPU scaling on sector-parallel
    # ed_diag" is THIS field (strong scaling of one fixed job), not `value`
    # (weak scaling of independent c2 replicas): the wall time against the
    # committed single-GPU time of the same job and build
    ref_path = os.path.join(ROOT, "profiles", "farm_c4_1gpu.json")
    ref = None
    if os.path.exists(ref_path):
        with open(ref_path) as fh:
            ref = json.load(fh)
    speed = None
    if world == 1:
        speed = 1.0
    elif ref:
        speed = round(float(ref["wall_s"]) / dt, 3)
    from edgpu.farm import QUEUE_FALLBACK
    return {"wall_s": round(dt, 4), "sectors": len(res.eigenvalues), "n_gpus": world,
            "reference_1gpu_wall_s": ref["wall_s"] if ref else None,
            "reference_1gpu_source": ref.get("source") if ref else None,
            "speedup_vs_1gpu": speed,
            "north_star_scaling_field": True,
            "queue_fallback": QUEUE_FALLBACK[0] if QUEUE_FALLBACK else None,
            "E0": round(float(res.states.emin), 10), "gs_states": res.states.size,
            "rank0_sectors": len(res.local), "scaling": "strong",
            "schedule": (f"{opt.farm_schedule} over {world} ranks" if world > 1 else "one rank") +
                        f", {opt.workers} worker threads per GPU",
            "parity": {"fixture": "tests/golden/c4_diag_random.json", "E0_rel_dev": e0_dev,
                       "worst_eigenvalue_dev_rel_E0": worst, "bar": 1e-10},
            "workload": "configs[3]: Norb=2 Nbath=5 Uloc=(2,2,0) Ust=1 Jh=0.5 random bath, all 169 sectors, "
                        "lanc_method=arpack (Neigen=6, ncv=23) on device"}


def bench_nonsu2(dist, world, dev):
    """configs[4]: nonSU2 Norb=1 Nbath=6 (Nlevels=14): complex ground state over
    all sectors + the Green's function (diagonal + spin-mixed seeds, 200-step
    Lanczos each, Lmats=Lreal=5000), seeds farmed over the ranks; G(iw) checked
    against the committed oracle fixture."""
    from edgpu.diag import DiagOptions
    from edgpu.farm import farm_diag
    from edgpu.gf import GFOptions, _job_list, build_gf
    from golden.golden_configs import c5_config

    cfg = c5_config("random")
    opt = DiagOptions()
    gopt = GFOptions()
    res = farm_diag(cfg, opt, device=dev)
    build_gf(cfg, res.states, gopt, device=dev, owners=res.owners)   # warm-up
    t_diag, res = _timed(dist, lambda: farm_diag(cfg, opt, device=dev))
    t_gf, (Gm, _) = _timed(dist, lambda: build_gf(cfg, res.states, gopt, device=dev, owners=res.owners))
    gold = np.load(os.path.join(GOLD, "c5_gf_random.npz"))
    rel = float(np.max(np.abs(Gm[..., gold["iw_index"]] - gold["Gm"])) / np.max(np.abs(gold["Gm"])))
    e0_dev = abs(res.states.emin - float(gold["E0"])) / abs(float(gold["E0"]))
    assert rel < 1e-10 and e0_dev < 1e-10, f"nonsu2_c5 differs from the oracle fixture: G {rel:.2e}, E0 {e0_dev:.2e}"
    return {"diag_s": round(t_diag, 4), "gf_s": round(t_gf, 4), "n_gpus": world,
            "gf_seeds": len(_job_list(cfg, res.states)[0]), "E0": round(float(res.states.emin), 10),
            "G_iw0_00": [round(float(Gm[0, 0, 0, 0, 0].real), 10), round(float(Gm[0, 0, 0, 0, 0].imag), 10)],
            "parity": {"fixture": "tests/golden/c5_gf_random.npz", "G_iw_max_rel_dev": rel, "E0_rel_dev": e0_dev,
                       "bar": 1e-10},
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
    if dist:
        import torch.distributed as tdist
        backend = tdist.get_backend()
        how = "RCCL" if backend == "nccl" else backend
    else:
        how = "one rank: no exchange"
    return {"ms_per_hxv": round(dt / iters * 1e3, 4), "n_gpus": world, "scaling": "strong", "backend": how,
            "dim": ds.du * ds.dd, "local_rows": nw,
            "workload": "Nlevels=28 Norb=1 Nbath=13 (7,7) sector split by down rows; Kronecker rows/cols "
                        f"kernels + 2 all_to_all exchanges per H·v ({how}; strip layout, no transposes)"}


def _lanc_rate(S, niter, v0, reps=5, options=()):
    """Best-of device time of `reps` niter-step runs -> iters/s (and the last α, β),
    with the sector's kernel options `options` (ED_OPT_* names) during the runs."""
    S.set_options(*options)
    try:
        for _ in range(2):
            S.lanc_run(niter, v0_dev=v0)
        runs = [S.lanc_run(niter, v0_dev=v0) for _ in range(reps)]
    finally:
        S.set_options()
    return niter / (min(r[2] for r in runs) * 1e-3), runs[-1]


def bench_batched(S, v0, niter, last_alpha, ks=(256, 1024), cplx=False):
    """The whole chip on configs[1]: K independent Lanczos recurrences on the
    same sector in ONE persistent launch (ed_sector_lanc_tridiag_batch, one
    workgroup per start vector — how the Green's-function seeds of a target
    sector run).  Wall time of the call (workspace, start-vector
    copy, launch, alpha/beta download), best of 3.  Start vector 0 is the
    timed single run's v0: its alpha must equal that run's."""
    from edgpu.gf import _tridiag_batch

    g = torch.Generator(device=v0.device).manual_seed(7)
    out = {}
    for k in ks:
        seeds = v0.unsqueeze(0).repeat(k, 1)
        seeds[1:] *= 1.0 + 0.05 * torch.rand(k - 1, v0.numel(), dtype=torch.float64, device=v0.device, generator=g)
        seeds = seeds.contiguous()
        torch.cuda.synchronize()
        _tridiag_batch(S, seeds, niter, not cplx, 1e-300)
        best = None
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a, b, n = _tridiag_batch(S, seeds, niter, not cplx, 1e-300)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        dev = float(np.max(np.abs(a[0] - last_alpha[:niter])) / np.max(np.abs(last_alpha[:niter])))
        assert dev < 1e-12 and int(n.min()) == niter, f"batched run {k}: alpha of seed 0 off by {dev}"
        out[str(k)] = {"iters_per_s": round(k * niter / best, 1), "wall_s": round(best, 5),
                       "alpha_seed0_rel_dev": dev}
    out["note"] = ("K start vectors on the configs[1] sector, one workgroup each, one launch "
                   "(the headline value is ONE recurrence on one CU)" +
                   ("; complex(8) vectors on the real(8) stored H (MODE 4, 512-thread register layout per run)" if cplx else ""))
    return out


def _traffic(name):
    """Per-launch HBM-side bytes from a committed rocprofv3 summary
    (profiles/r4/<name>.json, else round 3's: 2 x FETCH_SIZE + WRITE_SIZE, the
    gfx950 x2 calibrated for 4/8/16-B lane loads in profiles/r2/fetch_calib.json)."""
    for d in PROFILES:
        f = os.path.join(d, name)
        if os.path.exists(f):
            with open(f) as fh:
                tj = json.load(fh)
            return tj.get("traffic_bytes_per_launch"), os.path.relpath(f, ROOT)
    return None, None


def _profile_ms(name):
    """Steady-state per-launch duration of the same kernel on the same sector
    from a committed rocprofv3 kernel trace (profiles/r4/<name>_trace.json,
    tools/trace_summary.py: the probe's warm-up launches dropped), for
    comparison with this run's HIP-event average."""
    for d in PROFILES:
        f = os.path.join(d, f"{name}_trace.json")
        if os.path.exists(f):
            with open(f) as fh:
                tj = json.load(fh)
            return {"rocprof_steady_mean_ms": round(tj["steady_mean_ns"] * 1e-6, 4),
                    "rocprof_steady_median_ms": round(tj["steady_median_ns"] * 1e-6, 4),
                    "source": os.path.relpath(f, ROOT)}
    return None


def roofline_sweep(Sector, make_config):
    """The rest of SURVEY §8(d)'s roofline sweep beside the headline N28 line:
    the Norb=2 Nbath=6 (7,7) sector (Nlevels=28, Norb=2 hopping structure)
    and the configs[3] half-filled (6,6) sector (dim 853,776; matrix + vectors
    ~ the 256 MB Infinity Cache), stored packed real(8) H·v and the two-pass
    matrix-free H·v; average of 50 launches after 5 warm-ups, HIP events on the
    launch stream.  `frac` on the bytes each kernel moves; traffic from the
    committed PMC summaries where present."""
    from golden.golden_configs import SEED

    out = {}
    for name, kw, q, tname in (("n28b", dict(Norb=2, Nbath=6), (7, 7), "n28b"),
                               ("c4_66", None, (6, 6), "c4")):
        if kw is None:
            from golden.golden_configs import c4_config
            cfg = c4_config("random")
        else:
            cfg = make_config(bath="random", seed=SEED, **kw)
        inf = {}
        dim, nnz, ms = measure_hxv(Sector, cfg, q, 50, path=0, info=inf)
        if inf["split"]:
            Bown = spmv_bytes_split(inf, dim)
            tr, tsrc = _traffic(f"split_{tname}_traffic.json")
            kern = "k_spmv_sa + k_spmv_sb<real> (two-segment stored)"
        else:
            Bown = spmv_bytes_packed(inf["padded"], dim) if inf["packed"] else spmv_bytes_real(nnz, dim)
            tr, tsrc = _traffic(f"spmv_{tname}_traffic.json")
            kern = "k_spmv_pk<real>" if inf["packed"] else "k_spmv<real,real>"
        row = {"dim": dim, "nnz": nnz, "ms_per_launch": round(ms, 4), "bytes_per_launch": Bown,
               "achieved": round(Bown / (ms * 1e-3) / 1e9, 1),
               "frac": round(Bown / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
               "csr_equivalent_gbs": round(spmv_bytes_real(nnz, dim) / (ms * 1e-3) / 1e9, 1),
               "traffic": tr, "traffic_source": tsrc,
               "physical_gbs": round(tr / (ms * 1e-3) / 1e9, 1) if tr else None,
               "kernel": kern}
        _, _, msk = measure_hxv(Sector, cfg, q, 50, path=2)
        tk, tksrc = _traffic(f"kron_{tname}_traffic.json")
        two = dim >= (1 << 19)   # the library's two-pass threshold
        row["matrix_free"] = {"ms_per_hxv": round(msk, 4),
                              "frac_16dim": round(16 * dim / (msk * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                              "kernel": "k_kron_up + k_kron_dw (two-pass)" if two else "k_kron (one pass)",
                              "traffic": tk, "traffic_source": tksrc}
        if two:
            row["matrix_free"]["two_pass_gbs"] = round(40 * dim / (msk * 1e-3) / 1e9, 1)
        out[name] = row
    # HBM-sized sectors WITHOUT the Kronecker form: the stored kernel (real and
    # complex H) and the generic matrix-free k_direct are the only paths
    for name, kw, q in (("n28j", dict(Norb=2, Nbath=6, Uloc=(2.0, 2.0, 0.0), Ust=1.0, Jh=0.5, Jx=0.5, Jp=0.5),
                         (7, 7)),
                        ("n26s", dict(Norb=1, Nbath=12, Nspin=2, ed_mode="nonsu2"), (13, 0))):
        cfg = make_config(bath="random", seed=SEED, **kw)
        row = {}
        for cplx in (False, True):
            inf = {}
            dim, nnz, ms = measure_hxv(Sector, cfg, q, 30, path=0, info=inf, cplx=cplx)
            if inf["fused"]:
                Bown = spmv_bytes_fused(inf, dim, cplx)
            elif inf["packed"]:
                Bown = (spmv_bytes_packed_complex if cplx else spmv_bytes_packed)(inf["padded"], dim)
            else:
                Bown = (20 * nnz + 8 * (dim + 1) + 32 * dim) if cplx else spmv_bytes_real(nnz, dim)
            tr, tsrc = _traffic(f"{'fused' if inf['fused'] else 'spmv'}_{name}{'_cplx' if cplx else ''}_traffic.json")
            row["stored_complex" if cplx else "stored"] = {
                "dim": dim, "nnz": nnz, "ms_per_launch": round(ms, 4), "bytes_per_launch": Bown,
                "achieved": round(Bown / (ms * 1e-3) / 1e9, 1),
                "frac": round(Bown / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic": tr, "traffic_source": tsrc,
                "physical_gbs": round(tr / (ms * 1e-3) / 1e9, 1) if tr else None,
                "kernel": ("k_spmv_fu" if inf["fused"] else "k_spmv_pk" if inf["packed"] else "k_spmv") +
                          ("<complex>" if cplx else "<real>")}
        _, _, msd = measure_hxv(Sector, cfg, q, 20, path=1)
        td, tdsrc = _traffic(f"direct_{name}_traffic.json")
        row["direct_generic"] = {"ms_per_hxv": round(msd, 4),
                                 "frac_16dim": round(16 * dim / (msd * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                 "own_bytes": 24 * dim,  # v read, Hv written, diagonal vector read
                                 "frac_own": round(24 * dim / (msd * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                 "traffic": td, "traffic_source": tdsrc,
                                 "kernel": "k_direct (wave per 64-row chunk, op lists, LDS rank tables, diagonal vector from k_gen_diag)"}
        out[name] = row
    out["workloads"] = {"n28b": "Norb=2 Nbath=6 (Nlevels=28) (7,7) sector, random bath, real(8)",
                        "c4_66": "configs[3] Norb=2 Nbath=5 half-filled (6,6) sector, random bath, real(8)",
                        "n28j": "Norb=2 Nbath=6 (Nlevels=28) (7,7) with Jx=Jp=0.5 (no Kronecker form), random bath",
                        "n26s": "nonSU2 Norb=1 Nbath=12 (Nlevels=26) N=13 sector (spin flips: no Kronecker form), "
                                "random bath"}
    return out


def bench_roofline(Sector, make_config):
    """The roofline entries (rank 0, run before the farm sections so the
    timed kernels see the same clean device a lone probe run sees): stored
    real(8) H·v on the Nlevels=28 (7,7) sector (`roofline`), complex(8)
    stored, two-pass matrix-free, generic matrix-free and SURVEY §8(d)'s
    sweep (`kron_n28`, `roofline.sweep`)."""
    from golden.golden_configs import SEED

    cfg28 = make_config(Norb=1, Nbath=13, bath="random", seed=SEED)
    inf28 = {}
    dim28, nnz28, ms28 = measure_hxv(Sector, cfg28, (7, 7), 50, path=0, info=inf28)
    # frac on the bytes the timed kernels move (their own format: the
    # two-segment form's A words / U entries, or the one-pass kernel's 4-B
    # {col|value index} words); SURVEY §8(d)'s CSR-equivalent rate is
    # reported beside it and can exceed the physical rate
    Bcsr = spmv_bytes_real(nnz28, dim28)
    split = bool(inf28.get("split"))
    if split:
        Bown = spmv_bytes_split(inf28, dim28)
        tname = "split_n28"
        kern = ("k_spmv_sa + k_spmv_sb<real> (two-segment stored H·v: diagonal + in-block elements in row "
                "order -> y, then the cross-block elements — "
                f"{inf28['split_far_uniform']} of {inf28['split_far']} stored once per 128-row slice — "
                f"in column-chunk order, added to y; {inf28['npdict']}-value dictionary)")
        basis = ("bytes the two timed kernels move: split_bytes (4-B A words, 8-B U entries, A slice pointers) + "
                 "split_list_bytes (segment B's work list, slice table) + 48*dim (A: diagonal, v, y; B: y, v, Hv)")
    else:
        Bown = spmv_bytes_packed(inf28["padded"], dim28) if inf28["packed"] else Bcsr
        tname = "spmv_n28"
        kern = (("k_spmv_pk<real> (stored SELL-64, 32-bit {col|value index} words, "
                 f"{inf28['npdict']}-value dictionary)") if inf28["packed"]
                else "k_spmv<real,real> (stored SELL-64 H·v)")
        basis = ("bytes the timed kernel moves: 4*padded slots + 8*(nslice+1) + 8*dim "
                 "(diagonal) + 16*dim (read v, write Hv)") if inf28["packed"] else "12*nnz + 8*(dim+1) + 16*dim"
    ach = Bown / (ms28 * 1e-3) / 1e9
    traffic, tsrc = _traffic(f"{tname}_traffic.json")
    roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
            "achieved_basis": basis, "kernel": kern,
            "workload": f"Nlevels=28 Norb=1 Nbath=13 (7,7) sector, dim {dim28}, nnz {nnz28}, real(8)",
            "ms_per_launch": round(ms28, 4), "bytes_per_launch": Bown,
            "csr_equivalent_bytes": Bcsr,
            "csr_equivalent_gbs": round(Bcsr / (ms28 * 1e-3) / 1e9, 1),
            "physical_gbs": round(traffic / (ms28 * 1e-3) / 1e9, 1) if traffic else None,
            "traffic_over_own": round(traffic / Bown, 3) if traffic else None,
            "profile": _profile_ms(tname)}
    if split:
        # the one-pass kernel in spMatVec_cc's per-row order (ED_OPT_STORED_EXACT,
        # bit-identical to the oracle) on the same sector, for comparison
        inf1 = {}
        _, _, ms1 = measure_hxv(Sector, cfg28, (7, 7), 30, path=0, info=inf1, options=("stored_exact",))
        B1 = spmv_bytes_packed(inf1["padded"], dim28)
        t1, t1src = _traffic("spmv_n28_traffic.json")
        roof["one_pass_exact"] = {"ms_per_launch": round(ms1, 4), "bytes_per_launch": B1,
                                  "frac": round(B1 / (ms1 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                  "traffic": t1, "traffic_source": t1src,
                                  "kernel": "k_spmv_pk<real> (one pass, bit-identical to spMatVec_cc)",
                                  "profile": _profile_ms("spmv_n28")}
    dimk, _, msk = measure_hxv(Sector, cfg28, (7, 7), 50, path=2)
    Bk = 16 * dimk
    tk, tksrc = _traffic("kron_n28_traffic.json")
    kron = {"ms_per_hxv": round(msk, 4), "algorithmic_bytes": Bk,
            "achieved_gbs": round(Bk / (msk * 1e-3) / 1e9, 1),
            "frac": round(Bk / (msk * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": tk, "traffic_source": tksrc,
            "physical_gbs": round(tk / (msk * 1e-3) / 1e9, 1) if tk else None,
            "profile": _profile_ms("kron_n28"),
            "two_pass_bytes": 40 * dimk,
            "two_pass_gbs": round(40 * dimk / (msk * 1e-3) / 1e9, 1),
            "basis": "SURVEY §8(d) direct: 16*dim real (read v, write Hv); two_pass_bytes = 40*dim, "
                     "the least a two-pass form moves (pass U reads V, writes y; pass D reads V and "
                     "y, writes Hv)",
            "kernel": "k_kron_up + k_kron_dw (two-pass matrix-free Kronecker H·v)"}
    # generic matrix-free (any ed_mode) and complex(8) stored H·v on the same sector
    _, _, msd = measure_hxv(Sector, cfg28, (7, 7), 20, path=1)
    td, tdsrc = _traffic("direct_n28_traffic.json")
    kron["direct_generic"] = {"ms_per_hxv": round(msd, 4),
                              "kernel": "k_direct (wave per 64-row chunk, op lists, LDS rank tables, diagonal vector from k_gen_diag)",
                              "frac_16dim": round(Bk / (msd * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                              "own_bytes": 24 * dimk,  # v read, Hv written, diagonal vector read
                              "frac_own": round(24 * dimk / (msd * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                              "traffic": td, "traffic_source": tdsrc, "profile": _profile_ms("direct_n28")}
    # complex(8): H values and vectors (the reference's arithmetic), and
    # complex vectors on the real H (the cpu_baseline's arithmetic)
    for key, real_h, tn in (("complex", False, "cplx_n28"), ("complex_vectors_real_h", True, "cvec_n28")):
        infc = {}
        _, _, msc = measure_hxv(Sector, cfg28, (7, 7), 20, path=0, info=infc, cplx=True, real_h=real_h)
        inf1 = {}
        _, _, ms1 = measure_hxv(Sector, cfg28, (7, 7), 20, path=0, info=inf1, cplx=True, real_h=real_h,
                                options=("stored_exact",))
        B1 = spmv_bytes_packed_complex(inf1["padded"], dim28) - (8 * dim28 if real_h else 0)
        if infc["fused"]:
            Bc = spmv_bytes_fused(infc, dim28, True)
            tc, tcsrc = _traffic(f"fused_{tn}_traffic.json")
            kern = (f"k_spmv_fu<{'real' if real_h else 'complex'} H, complex v> (fused one-pass re-laid stored "
                    f"H·v: 64-row units, in-block words, {infc['fused_far_uniform']} of {infc['fused_far']} "
                    f"cross-block elements once per unit; {infc['npdict']}-value dictionary)")
            basis = ("fused_bytes (4-B A and L words, 8-B U entries, unit descriptors) + diagonal "
                     f"({8 if real_h else 16}*dim) + 32*dim (v, Hv)")
            prof = _profile_ms(f"fused_{tn}")
        else:
            Bc, tc, tcsrc, prof = B1, *_traffic(f"spmv_{tn}_traffic.json"), _profile_ms(f"spmv_{tn}")
            kern = f"k_spmv_pk<{'real' if real_h else 'complex'} H, complex v>"
            basis = "4*padded + 8*(nslice+1) + diagonal + 32*dim (v, Hv)"
        t1, t1src = _traffic(f"spmv_{tn}_traffic.json")
        roof[key] = {"ms_per_launch": round(msc, 4), "bytes_per_launch": Bc,
                     "achieved": round(Bc / (msc * 1e-3) / 1e9, 1),
                     "frac": round(Bc / (msc * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "one_pass_bytes_gbs": round(B1 / (msc * 1e-3) / 1e9, 1),
                     "frac_on_one_pass_bytes": round(B1 / (msc * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "csr_equivalent_gbs": round((20 * nnz28 + 8 * (dim28 + 1) + 32 * dim28)
                                                 / (msc * 1e-3) / 1e9, 1),
                     "traffic": tc, "traffic_source": tcsrc,
                     "traffic_over_own": round(tc / Bc, 3) if tc else None, "profile": prof,
                     "kernel": kern, "achieved_basis": basis,
                     "one_pass_exact": {"ms_per_launch": round(ms1, 4), "bytes_per_launch": B1,
                                        "frac": round(B1 / (ms1 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                        "traffic": t1, "traffic_source": t1src,
                                        "kernel": "k_spmv_pk (one pass, bit-identical to spMatVec_cc)"}}
    roof["sweep"] = roofline_sweep(Sector, make_config)
    return roof, kron


def spawn_ranks(n, argv):
    """`--gpus N` without an external launcher: start N ranks (one process per
    GPU) with torch.distributed.run as a CHILD process and return its exit
    code.  Called before anything touches the GPU (importing torch and
    counting devices do not), and never by exec: the parent only waits."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC (the box's driver)
    return subprocess.run(cmd, env=env).returncode


def rank_env(args):
    """(world, rank, local) of this process; checks that the launch matches
    --gpus (a driver run of `--gpus 8` must measure 8 ranks, not one)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if not (0 <= rank < world):
        raise SystemExit(f"bench.py: RANK={rank} outside WORLD_SIZE={world}")
    return world, rank, local


def launch_check(args):
    """`--launch-check`: the N-rank flow without a GPU (CPU test): every rank
    joins a gloo group, the barrier-bracketed max-over-ranks timing runs on a
    CPU stand-in step, rank 0 prints the line with n_gpus = world."""
    import torch.distributed as tdist

    world, rank, local = rank_env(args)
    if world > 1:
        tdist.init_process_group("gloo")
    seen = torch.tensor([float(rank), float(local)], dtype=torch.float64)
    allv = [torch.zeros(2, dtype=torch.float64) for _ in range(world)]
    if world > 1:
        tdist.all_gather(allv, seen)
    else:
        allv = [seen]
    t0 = time.perf_counter()
    if world > 1:
        tdist.barrier()
    dt = torch.tensor([time.perf_counter() - t0 + 1e-3 * (rank + 1)], dtype=torch.float64)
    if world > 1:
        tdist.all_reduce(dt, op=tdist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks": [int(v[0]) for v in allv],
                          "local_ranks": [int(v[1]) for v in allv], "max_dt": float(dt.item())}))
    if world > 1:
        tdist.destroy_process_group()


def north_star_scalars(out, mode2_ips, direct_ips, cplx_ips, cplxh_ips):
    """The north_star numbers as top-level scalars, last in the JSON line: the
    ">= 6x" farm scaling field (farm_c4 wall time and its speedup over the
    committed 1-GPU time), the rates of the other arithmetic on the headline
    sector, and the roofline fractions of the stored H·v."""
    farm = out.get("farm_c4") or {}
    c5 = out.get("nonsu2_c5") or {}
    roof = out.get("roofline") or {}
    cplx = roof.get("complex") or {}
    return {
        "stored_mode2_iters_per_s": round(mode2_ips, 1),
        "direct_iters_per_s": round(direct_ips, 1),
        "complex_iters_per_s": round(cplx_ips, 1),
        "complex_h_iters_per_s": round(cplxh_ips, 1),
        "nonsu2_c5_diag_s": c5.get("diag_s"),
        "nonsu2_c5_gf_s": c5.get("gf_s"),
        "roofline_frac": roof.get("frac"),
        "roofline_complex_ms": cplx.get("ms_per_launch"),
        "roofline_complex_frac": cplx.get("frac"),
        "roofline_complex_frac_on_one_pass_bytes": cplx.get("frac_on_one_pass_bytes"),
        "farm_c4_wall_s": farm.get("wall_s"),
        "farm_c4_speedup_vs_1gpu": farm.get("speedup_vs_1gpu"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--niter", type=int, default=512)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-farm", action="store_true", help="skip the configs[3]/[4] sections")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if args.launch_check:
        return launch_check(args)

    world, rank, local = rank_env(args)
    dist = world > 1
    # rehearsal switches (not used by the driver): ED_BENCH_BACKEND=gloo and
    # ED_BENCH_ONE_DEVICE=1 run N ranks on one GPU to exercise the N>1 flow
    one_device = bool(os.environ.get("ED_BENCH_ONE_DEVICE"))
    backend = os.environ.get("ED_BENCH_BACKEND", "nccl") if dist else None
    if one_device:
        local = 0
    ndev = torch.cuda.device_count()
    if local >= ndev:
        raise SystemExit(f"bench.py: rank {rank} wants GPU {local} but {ndev} are visible")
    torch.cuda.set_device(local)
    if dist:
        import torch.distributed as tdist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)
        assert tdist.get_world_size() == args.gpus
    dev = torch.cuda.current_device()

    from edgpu.hamiltonian import Sector
    from edgpu.params import make_config
    from golden.golden_configs import SEED, c2_config

    seed = SEED + rank
    cfg = c2_config("random", seed)
    S = Sector(cfg, 4, 4, stored=True, direct=False, real=True, device=dev)
    v0 = torch.sin(torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda"))
    mode = S.lanc_mode(real=True, path=0)

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
    last = None
    for _ in range(args.steps):
        last = step()
        dev_ms += last[2]
    barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = float(t.item())
    iters_total = args.steps * args.niter * world
    value = iters_total / dt

    # validation of the timed work: lowest Ritz value of the last run's
    # tridiagonal vs the oracle's E0 for this rank's bath (committed fixture)
    from scipy.linalg import eigh_tridiagonal

    a, b, _ = last
    ritz = float(eigh_tridiagonal(a, b[1:], eigvals_only=True, select="i", select_range=(0, 0))[0])
    with open(os.path.join(GOLD, "c2_e0.json")) as fh:
        e0_ref = json.load(fh)["by_seed"].get(str(seed), {}).get("E0")
    valid = None
    if e0_ref is not None:
        valid = {"ritz_min": ritz, "E0_oracle": e0_ref, "rel_dev": abs(ritz - e0_ref) / abs(e0_ref),
                 "fixture": "tests/golden/c2_e0.json", "bar": 1e-10}
        assert valid["rel_dev"] < 1e-10, f"timed Lanczos run: lowest Ritz value {ritz} vs oracle E0 {e0_ref}"

    # configs[1] with the stored matrix as ELL words in registers (MODE 2, no
    # Kronecker structure), complex(8) arithmetic, and configs[2] matrix-free
    mode2_ips, _ = _lanc_rate(S, args.niter, v0, options=("no_pkron",))
    vc = torch.complex(v0, torch.cos(3 * torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda")))
    cplx_ips, (ac, bc_, _) = _lanc_rate(S, args.niter, vc)
    cplx_mode = S.lanc_mode(real=False, path=0)
    with Sector(cfg, 4, 4, stored=True, direct=False, real=False, device=dev) as Sc:
        cplxh_ips, _ = _lanc_rate(Sc, args.niter, vc)
        cplxh_mode = Sc.lanc_mode(real=False, path=0)
    with Sector(cfg, 4, 4, stored=False, direct=True, real=True, device=dev) as Sd:
        direct_ips, _ = _lanc_rate(Sd, args.niter, v0)
        direct_mode = Sd.lanc_mode(real=True, path=2)

    roof_kron = (None, None) if (args.no_roofline or rank != 0) else bench_roofline(Sector, make_config)
    split = None if args.no_farm else bench_split(dist, world, dev)
    farm = None if args.no_farm else bench_farm(dist, world, dev)
    nonsu2 = None if args.no_farm else bench_nonsu2(dist, world, dev)

    out = None
    if rank == 0:
        # SpMV GB/s on the headline sector (L2-resident; launch-latency bound)
        dim2, nnz2, ms2 = measure_hxv(Sector, cfg, (4, 4), 2000, batch=True)
        gbs2 = spmv_bytes_real(nnz2, dim2) / (ms2 * 1e-3) / 1e9
        batched = bench_batched(S, v0, args.niter, np.asarray(last[0]))
        batched_c = bench_batched(S, vc, args.niter, np.asarray(ac), cplx=True)
        roof, kron = roof_kron
        # the CPU baseline is a rank-0, N=1 measurement (task contract)
        cpu = None if (args.no_cpu or world > 1) else cpu_baseline()
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
                                   f"stored real(8) H, plain Lanczos {args.niter} iters/step, persistent MODE "
                                   f"{mode} (4 = stored matrix in the Kronecker register layout)",
                       "parallelism": f"sector replicas x{world}"},
            "device_ms_per_step": round(dev_ms / args.steps, 4),
            "validation": valid,
            "stored_mode2_note": "configs[1]: stored SELL matrix as ELL words {col|value} in registers (MODE 2)",
            "direct_note": f"configs[2]: same sector, matrix-free hop tables (persistent MODE {direct_mode})",
            "complex_note": f"complex(8) vectors on the real(8) stored H (persistent MODE {cplx_mode}); the "
                            "arithmetic of cpu_baseline (its H has zero imaginary parts)",
            "complex_h_note": f"complex(8) H values and vectors, stored (persistent MODE {cplxh_mode})",
            "batched_c2": batched,
            "batched_c2_complex": batched_c,
            "spmv_gbs_c2": round(gbs2, 1),
            "spmv_ms_c2": round(ms2, 5),
            # the long nested blocks first: the driver records the tail of
            # stdout, so the north-star scalars below end the line
            "roofline": roof,
            "kron_n28": kron,
            "cpu_baseline": cpu,
            "split_n28": split,
            "nonsu2_c5": nonsu2,
            "farm_c4": farm,
        }
        out.update(north_star_scalars(out, mode2_ips, direct_ips, cplx_ips, cplxh_ips))
        print(json.dumps(out))
    S.close()
    if dist:
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
