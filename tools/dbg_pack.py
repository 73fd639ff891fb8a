import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "dmft-ed_amd"), os.path.join(os.getcwd(), "tests")]
import numpy as np
import torch
torch.cuda.init()
from edgpu.hamiltonian import Sector
from cases import CASES
for name, make, secs in CASES:
    cfg = make()
    if not cfg.is_real():
        continue
    for q in secs:
        with Sector(cfg, q[0], q[1], stored=True, real=True) as S:
            rp, c, v = S.dump_csr()
            offd = np.concatenate([v[rp[i] + 1:rp[i + 1]] for i in range(S.dim)]).real
            print(name, q, S.dim, "packed", S.info.packed, "npdict", S.info.npdict, "distinct", len(np.unique(offd.view(np.uint64))), flush=True)
