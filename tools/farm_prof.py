"""configs[3] sector farm on one GPU for profiling: wall time, and per Lanczos
sector the solve time, H·v products and restarts' worth of work.

    python tools/farm_prof.py [--workers N] [--reps R] [--serial-stats out.json]

--serial-stats: additionally solve every Lanczos sector alone on one thread
(create / eigh / close timed separately, nhv from ed_sector_eigh) and write a
JSON table (the fixed-cost fit of edgpu.farm.sector_cost comes from it).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmft-ed_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
from edgpu.diag import DiagOptions, _start_vector, lanczos_params  # noqa: E402
from edgpu.farm import farm_diag  # noqa: E402
from edgpu.hamiltonian import Sector  # noqa: E402
from edgpu.sectors import setup_pointers  # noqa: E402
from golden.golden_configs import c4_config  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workers", type=int, default=8)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--serial-stats", default="")
ap.add_argument("--options", default="", help="comma-separated ED_OPT_* names for every sector")
ap.add_argument("--bath", default="random", help="configs[3] bath: random | flat")
ap.add_argument("--private-streams", action="store_true",
                help="DiagOptions.worker_streams=False: a private stream per sector (A/B)")
ap.add_argument("--budget", type=float, default=None, help="DiagOptions.cache_budget_mb (default: the library default)")
ap.add_argument("--timeline", default="", help="write per-sector (start, end, thread, dim) of the last rep")
ap.add_argument("--maps", default="", help="write the process's shared-object mappings (for symbolising a crash)")
ap.add_argument("--dim-range", default="", help="lo:hi — farm only the sectors with lo <= dim < hi (where the wall goes)")
ap.add_argument("--small-workers", type=int, default=None, help="DiagOptions.small_workers (default: the library's)")
ap.add_argument("--batch-max-dim", type=int, default=None,
                help="DiagOptions.batch_max_dim (default: the library's; > 0 farms without the per-sector timeline)")
ap.add_argument("--lib", default="", help="load this libedgpu.so build instead (A/B of kernel variants)")
a = ap.parse_args()
if a.lib:
    import edgpu._lib as _edl  # noqa: E402
    _edl.LIB_PATH = os.path.abspath(a.lib)
cfg = c4_config(a.bath)
opts = tuple(x for x in a.options.split(",") if x)

if a.serial_stats:
    opt = DiagOptions()
    rows = []
    for sec in setup_pointers(cfg):
        neigen, nitermax, nblock = lanczos_params(sec.dim, opt)
        if neigen == sec.dim or sec.dim <= opt.lanc_dim_threshold:
            continue
        t0 = time.perf_counter()
        S = Sector(cfg, sec.q1, sec.q2, stored=True, real=True, options=opts)
        t1 = time.perf_counter()
        w, X, nconv, nhv = S.eigh(neigen=neigen, ncv=min(nblock, 64), maxit=nitermax,
                                  v0=_start_vector(sec.dim, False), on_device=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        S.close()
        t3 = time.perf_counter()
        rows.append(dict(sector=[sec.q1, sec.q2], dim=sec.dim, create_s=round(t1 - t0, 5),
                         eigh_s=round(t2 - t1, 5), close_s=round(t3 - t2, 5), nhv=nhv, nconv=nconv))
        print(rows[-1], flush=True)
    tot = {k: round(sum(r[k] for r in rows), 4) for k in ("create_s", "eigh_s", "close_s")}
    tot["nhv"] = sum(r["nhv"] for r in rows)
    print("serial totals", tot, flush=True)
    with open(a.serial_stats, "w") as f:
        json.dump(dict(config="configs[3] random bath, Lanczos sectors, one thread", options=list(opts),
                       totals=tot, sectors=rows), f, indent=1)

opt = DiagOptions(workers=a.workers, kernel_options=opts, worker_streams=not a.private_streams)
if a.small_workers is not None:
    opt.small_workers = a.small_workers
if a.budget is not None:
    opt.cache_budget_mb = a.budget
if a.batch_max_dim is not None:
    opt.batch_max_dim = a.batch_max_dim
if a.maps:
    # every mapped shared object with its load base (the lowest start of its
    # mappings) and the executable segment (start, file offset): native crash
    # PCs map to (object, offset) for addr2line / llvm-symbolizer in the
    # builder container (same image)
    from edgpu import _lib as _edlib  # noqa: E402
    _edlib.load()
    objs = {}
    with open("/proc/self/maps") as fh:
        for ln in fh:
            f = ln.split()
            if len(f) < 6 or not f[5].startswith("/"):
                continue
            lo, hi = (int(x, 16) for x in f[0].split("-"))
            o = objs.setdefault(f[5], {"base": lo, "exec": []})
            o["base"] = min(o["base"], lo - int(f[2], 16))
            if "x" in f[1]:
                o["exec"].append([hex(lo), hex(hi), hex(int(f[2], 16))])
    with open(a.maps, "w") as fh:
        json.dump({k: {"base": hex(v["base"]), "exec": v["exec"]} for k, v in objs.items()}, fh, indent=1)
import threading  # noqa: E402

from edgpu.diag import solve_sector  # noqa: E402

events = []


def timed_solver(cfg_, sec, opt_, device):
    t0 = time.perf_counter()
    r = solve_sector(cfg_, sec, opt_, device)
    events.append(dict(sector=[sec.q1, sec.q2], dim=sec.dim, t0=t0, t1=time.perf_counter(),
                       thread=threading.get_ident(), method=r.method))
    return r


subset = None
if a.dim_range:
    lo, hi = (float(x) if x else None for x in a.dim_range.split(":"))
    subset = [s.isector for s in setup_pointers(cfg)
              if (lo is None or s.dim >= lo) and (hi is None or s.dim < hi)]
    print(f"dim range {a.dim_range}: {len(subset)} sectors", flush=True)
for rep in range(a.reps):
    events.clear()
    torch.cuda.synchronize()
    t = time.perf_counter()
    # (the small-sector batch runs only with the library's own solver)
    res = farm_diag(cfg, opt, solver=None if opt.batch_max_dim > 0 else timed_solver, sectors=subset)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t
    print(f"farm workers={a.workers} batch_max_dim={opt.batch_max_dim} wall {wall:.4f} s "
          f"states={res.states.size}", flush=True)
    if not events:
        continue
    busy = sum(e["t1"] - e["t0"] for e in events)
    first = min(e["t0"] for e in events) - t
    last = max(e["t1"] for e in events) - t
    print(f"  sector solves: sum {busy:.3f} s over {len(events)} (mean concurrency {busy / max(last - first, 1e-9):.2f}),"
          f" first start {first * 1e3:.1f} ms, last end {last * 1e3:.1f} ms", flush=True)
if a.timeline and events:
    t0 = min(e["t0"] for e in events)
    for e in events:
        e["t0"] = round(e["t0"] - t0, 6)
        e["t1"] = round(e["t1"] - t0, 6)
    with open(a.timeline, "w") as f:
        json.dump(events, f)
