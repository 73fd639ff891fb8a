import os, sys, numpy as np
sys.path.insert(0, "dmft-ed_amd")
from edgpu.hamiltonian import Sector
from edgpu.params import make_config
cfg = make_config(Norb=2, Nbath=5)
for kw in (dict(stored=True), dict(stored=False, direct=True)):
    with Sector(cfg, 6, 6, real=True, **kw) as S:
        e0, vec, nl = S.lanc_eigh(nitermax=512, threshold=1e-12)
        print(kw, "fresh eigh vec", e0, nl, np.linalg.norm(vec), flush=True)
    with Sector(cfg, 6, 6, real=True, **kw) as S:
        a, b, n = S.lanc_tridiag(None, 40)
        e0, vec, nl = S.lanc_eigh(nitermax=512, threshold=1e-12, vector=False)
        print(kw, "eigh after tridiag", e0, nl, flush=True)
