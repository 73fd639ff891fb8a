"""A/B of the thick-restart eigensolver's kernel options on single configs[3]
sectors (device time of ed_sector_eigh, best of N): default against the
listed ED_OPT_* alternatives.

    python tools/trlan_ab.py [--reps 5] [--opts trlan_fullupd,eigh_no_verify] [--ncv 16,23,32]
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
ap.add_argument("--forms", default="", help="comma list of stored forms built at any size instead of the "
                "options: fused (ED_FUSED_ON), split (ED_SPLIT_ON), both")
# (round 4 also swept the kept Ritz vectors and the Krylov block cap through
# temporary library switches, since removed: DESIGN.md §2 has the results)
a = ap.parse_args()
cfg = c4_config("random")
opt = DiagOptions()
variants = [("default", (), None, None)]
if a.ncv:
    variants += [(f"ncv={n}", (), int(n), None) for n in a.ncv.split(",")]
else:
    variants += [(o, (o,), None, None) for o in a.opts.split(",") if o]
forms = [("", {})]
if a.forms:
    fl = {"fused": dict(fused=True, split=False), "split": dict(split=True, fused=False),
          "both": dict(split=True, fused=True)}
    forms += [(f, fl[f]) for f in a.forms.split(",")]
    variants = [("default", (), None, None)]
for q in a.sectors.split(";"):
  q1, q2 = (int(x) for x in q.split(","))
  for fname, fkw in forms:
    with Sector(cfg, q1, q2, stored=True, real=True, **fkw) as S:
        neigen, nitermax, nblock = lanczos_params(S.dim, opt)
        v0 = _start_vector(S.dim, False)
        ref = None
        for name, o, ncv, _ in variants:
            S.set_options(*o)
            best, nhv = 1e9, 0
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t = time.perf_counter()
                w, _, _, nhv = S.eigh(neigen=neigen, ncv=min(ncv or nblock, 64), maxit=nitermax, v0=v0, vectors=False)
                best = min(best, time.perf_counter() - t)
            ref = w if ref is None else ref
            name = fname or name
            print(f"({q1},{q2}) dim {S.dim:7d} {name:15s} {best * 1e3:8.2f} ms  nhv {nhv:4d}  "
                  f"dE {np.max(np.abs(np.asarray(w) - ref)):.1e}", flush=True)
        S.set_options()
