"""Complex(8) vectors on the real configs[1] stored H (the reference's vector
type): persistent MODE 4, 512-thread register layout.  Prints us per Lanczos
step (best of 5 512-step runs, device time) for two back-to-back runs and the
largest alpha deviation between them (the run-to-run spread of the A/B).

    python tools/cvec_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dmft-ed_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import _lanc_rate  # noqa: E402
from edgpu.hamiltonian import Sector  # noqa: E402
from edgpu.params import make_config  # noqa: E402

cfg = make_config(Norb=1, Nbath=7, bath="random", seed=20251015)
with Sector(cfg, 4, 4, stored=True, real=True) as S:
    i = torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda")
    v0 = torch.complex(torch.sin(i), torch.cos(3 * i)).contiguous()
    out = {}
    for name in ("run1", "run2"):
        ips, run = _lanc_rate(S, 512, v0)
        out[name] = run
        print(f"{name}: {1e6 / ips:.3f} us/step ({ips:.0f} it/s)", flush=True)
    a0, a1 = np.asarray(out["run1"][0]), np.asarray(out["run2"][0])
    n = min(len(a0), len(a1), 64)
    print(f"alpha max rel dev run1 vs run2 {np.max(np.abs(a0[:n] - a1[:n])) / np.max(np.abs(a1[:n])):.2e}")
