"""Time device Lanczos runs (µs/iteration) for the small-sector paths.

usage: python tools/lanc_probe.py [--niter 512]
Runs c2 (4,4) and c5 N=7 through stored / matrix-free, persistent / multi-kernel.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dmft-ed_amd"))
import torch  # noqa: E402

from edgpu.hamiltonian import Sector  # noqa: E402
from edgpu.params import make_config  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--niter", type=int, default=512)
a = ap.parse_args()
cases = [
    ("c2 real", make_config(Norb=1, Nbath=7, bath="random"), (4, 4), True),
    ("c2 complex", make_config(Norb=1, Nbath=7, bath="random"), (4, 4), False),
    ("c5 nonsu2", make_config(Norb=1, Nbath=6, Nspin=2, ed_mode="nonsu2", bath="random"), (7, 0), True),
    ("c4 real", make_config(Norb=2, Nbath=5, bath="random"), (6, 6), True),
]
MODES = {"stored": [("reg", ()), ("l2", ("persist_stored",)), ("multi", ("no_persist",))],
         "direct": [("reg", ()), ("lds", ("no_preg",)), ("multi", ("no_persist",))]}
for name, cfg, q, real in cases:
    for kind in ("stored", "direct"):
        for label, opts in MODES[kind]:
            with Sector(cfg, q[0], q[1], stored=kind == "stored", direct=kind == "direct", real=real,
                        options=opts) as S:
                dt = torch.float64 if real else torch.complex128
                v0 = torch.sin(torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda")).to(dt)
                mode = S.lanc_mode(real=real)
                S.lanc_run(a.niter, v0_dev=v0)
                ms = min(S.lanc_run(a.niter, v0_dev=v0)[2] for _ in range(3))
                print(f"{name:11s} dim={S.dim:7d} {kind:6s} {label:7s} mode={mode:2d} "
                      f"{1e3 * ms / a.niter:8.3f} us/iter  {a.niter / (ms * 1e-3):10.0f} it/s", flush=True)
