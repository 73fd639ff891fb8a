"""Complex(8) vectors on the real configs[1] stored H (the reference's vector
type): persistent MODE 4 in the 512-thread register layout (default) against
the 1024-thread LDS layout (ED_OPT_PKRON_C1024).  Prints µs per Lanczos step
(best of 5 512-step runs, device time) and the largest alpha/beta deviation
between the two layouts.

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
    for name, opts in (("c512", ()), ("c1024", ("pkron_c1024",)), ("c512slot", ("pkron_cslot",)),
                       ("c512_2", ())):
        ips, run = _lanc_rate(S, 512, v0, options=opts)
        out[name] = run
        print(f"{name}: {1e6 / ips:.3f} us/step ({ips:.0f} it/s)", flush=True)
    a2 = np.asarray(out["c512slot"][0])
    print(f"slot layout alpha max rel dev vs c512 {np.max(np.abs(a2[:64] - np.asarray(out['c512'][0])[:64])) / np.max(np.abs(a2[:64])):.2e}")
    a0, b0 = np.asarray(out["c512"][0]), np.asarray(out["c512"][1])
    a1, b1 = np.asarray(out["c1024"][0]), np.asarray(out["c1024"][1])
    n = min(len(a0), len(a1), 64)
    print(f"alpha max rel dev {np.max(np.abs(a0[:n] - a1[:n])) / np.max(np.abs(a1[:n])):.2e}, "
          f"beta {np.max(np.abs(b0[:n] - b1[:n])) / np.max(np.abs(b1[:n])):.2e}")
