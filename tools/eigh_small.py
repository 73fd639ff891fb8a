"""Repeated device eigh (thick-restart Lanczos, Neigen=6, ncv=23) of one small
configs[3] sector, for kernel traces of the per-step / per-restart cost.

    python tools/eigh_small.py [--sector 0 4] [--reps 10] [--options a,b]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmft-ed_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

torch.cuda.init()
from edgpu.diag import _start_vector  # noqa: E402
from edgpu.hamiltonian import Sector  # noqa: E402
from golden.golden_configs import c4_config  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--sector", type=int, nargs=2, default=[0, 4])
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--options", default="")
a = ap.parse_args()
cfg = c4_config("random")
with Sector(cfg, *a.sector, stored=True, real=True, options=tuple(x for x in a.options.split(",") if x)) as S:
    v0 = _start_vector(S.dim, False)
    S.eigh(neigen=6, ncv=23, maxit=512, v0=v0, on_device=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.reps):
        w, X, nconv, nhv = S.eigh(neigen=6, ncv=23, maxit=512, v0=v0, on_device=True)
    torch.cuda.synchronize()
    print(f"sector {a.sector} dim {S.dim}: {(time.perf_counter() - t) / a.reps * 1e3:.3f} ms per eigh, "
          f"{nhv} H.v, nconv {nconv}", flush=True)
    print("evals", " ".join(f"{float(x):.14f}" for x in w), flush=True)
