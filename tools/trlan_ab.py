"""A/B of the thick-restart eigensolver's kernel options on single configs[3]
sectors (device time of ed_sector_eigh, best of N): default against the
listed ED_OPT_* alternatives.

    python tools/trlan_ab.py [--reps 5] [--opts trlan_fullupd,eigh_no_verify]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmft-ed_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from edgpu.diag import DiagOptions, _start_vector, lanczos_params  # noqa: E402
from edgpu.hamiltonian import Sector  # noqa: E402
from golden.golden_configs import c4_config  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--opts", default="trlan_fullupd,eigh_no_verify")
ap.add_argument("--sectors", default="6,6;5,6;4,5;3,4;2,3")
ap.add_argument("--ncv", default="", help="comma list of ncv values (restart length) instead of the options")
ap.add_argument("--keep", default="", help="comma list of ED_TRLAN_KEEP values (Ritz vectors kept beyond nev)")
ap.add_argument("--grid", default="", help="comma list of ED_TRLAN_GRID values (Krylov sweep block cap)")
a = ap.parse_args()
cfg = c4_config("random")
opt = DiagOptions()
variants = [("default", (), None, None)]
if a.grid:
    variants += [(f"grid={g}", (), None, ("GRID", g)) for g in a.grid.split(",")]
elif a.ncv or a.keep:
    for n in (a.ncv.split(",") if a.ncv else [None]):
        for k in (a.keep.split(",") if a.keep else [None]):
            variants.append((f"ncv={n} keep={k}", (), int(n) if n else None, k))
else:
    variants += [(o, (o,), None, None) for o in a.opts.split(",") if o]
for q in a.sectors.split(";"):
    q1, q2 = (int(x) for x in q.split(","))
    with Sector(cfg, q1, q2, stored=True, real=True) as S:
        neigen, nitermax, nblock = lanczos_params(S.dim, opt)
        v0 = _start_vector(S.dim, False)
        ref = None
        for name, o, ncv, keep in variants:
            S.set_options(*o)
            os.environ.pop("ED_TRLAN_KEEP", None)
            os.environ.pop("ED_TRLAN_GRID", None)
            if isinstance(keep, tuple):
                os.environ["ED_TRLAN_" + keep[0]] = keep[1]
            elif keep is not None:
                os.environ["ED_TRLAN_KEEP"] = keep
            best, nhv = 1e9, 0
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t = time.perf_counter()
                w, _, _, nhv = S.eigh(neigen=neigen, ncv=min(ncv or nblock, 64), maxit=nitermax, v0=v0, vectors=False)
                best = min(best, time.perf_counter() - t)
            ref = w if ref is None else ref
            print(f"({q1},{q2}) dim {S.dim:7d} {name:15s} {best * 1e3:8.2f} ms  nhv {nhv:4d}  "
                  f"dE {np.max(np.abs(np.asarray(w) - ref)):.1e}", flush=True)
        S.set_options()
        os.environ.pop("ED_TRLAN_KEEP", None)
        os.environ.pop("ED_TRLAN_GRID", None)
