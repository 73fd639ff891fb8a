"""Run the c2 persistent Lanczos kernels (stored-in-registers MODE 2 and
Kronecker MODE 1) once each for PMC collection under rocprofv3."""
import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "dmft-ed_amd")]
import torch
torch.cuda.init()
from edgpu.hamiltonian import Sector
from edgpu.params import make_config

cfg = make_config(Norb=1, Nbath=7, bath="random")
for kw in (dict(stored=True), dict(stored=False, direct=True)):
    with Sector(cfg, 4, 4, real=True, **kw) as S:
        v0 = torch.sin(torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda"))
        print(kw, S.lanc_mode(real=True), S.lanc_run(512, v0_dev=v0)[2], flush=True)
