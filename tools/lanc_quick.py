"""µs per Lanczos step of the configs[1] sector (stored real, persistent path);
ED_GPU_LIB_VARIANT selects an experimental build (timing probes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dmft-ed_amd"))
import torch  # noqa: E402

from edgpu.hamiltonian import Sector  # noqa: E402
from edgpu.params import make_config  # noqa: E402

cfg = make_config(Norb=1, Nbath=7, bath="random")
with Sector(cfg, 4, 4, stored=True, direct=False, real=True) as S:
    v0 = torch.sin(torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda"))
    S.lanc_run(512, v0_dev=v0)
    ms = min(S.lanc_run(512, v0_dev=v0)[2] for _ in range(5))
    print(f"variant={os.environ.get('ED_GPU_LIB_VARIANT', '-')} mode={S.lanc_mode(real=True)} "
          f"{1e3 * ms / 512:.3f} us/step", flush=True)
