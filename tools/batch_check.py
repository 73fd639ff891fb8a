"""Batched vs single Lanczos alpha on the configs[1] sector, for a grid of
batch sizes K and iteration counts (real and complex vectors) — a debugging
probe for ed_sector_lanc_tridiag_batch.

    python tools/batch_check.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmft-ed_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from edgpu.gf import _tridiag_batch  # noqa: E402
from edgpu.hamiltonian import Sector  # noqa: E402
from golden.golden_configs import c2_config  # noqa: E402

cfg = c2_config("random")
with Sector(cfg, 4, 4, stored=True, real=True) as S:
    i = torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda")
    for cplx in (False, True):
        v0 = torch.sin(i)
        if cplx:
            v0 = torch.complex(v0, torch.cos(3 * i))
        v0 = v0.contiguous()
        print("mode", S.lanc_mode(real=not cplx), "cplx", cplx, flush=True)
        for niter in (50, 512):
            a1, _, _ = S.lanc_run(niter, v0_dev=v0)
            a1 = np.asarray(a1)
            for k in (3, 64, 256):
                seeds = v0.unsqueeze(0).repeat(k, 1).contiguous()
                a, b, n = _tridiag_batch(S, seeds, niter, not cplx, 1e-300)
                dev = [float(np.max(np.abs(a[j] - a1[:niter])) / np.max(np.abs(a1[:niter]))) for j in (0, k - 1)]
                first_bad = int(np.argmax(np.abs(a[0] - a1[:niter]) > 1e-12 * np.max(np.abs(a1))))
                print(f"  niter {niter} K {k}: rel dev run0 {dev[0]:.3e} run{k-1} {dev[1]:.3e} "
                      f"n.min {int(n.min())} first index off {first_bad}", flush=True)
