"""Per-phase timing of the configs[3] farm on one GPU (sector build vs solve)."""
import os, sys, time
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "dmft-ed_amd")]
import numpy as np
import torch
torch.cuda.init()
from edgpu.params import make_config
from edgpu.diag import DiagOptions, lanczos_params, _start_vector
from edgpu.sectors import setup_pointers
from edgpu.hamiltonian import Sector

sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from golden.golden_configs import c4_config
cfg = c4_config("random")
opt = DiagOptions()
tot = {"build": 0.0, "eigh": 0.0, "dense_build": 0.0, "dense_dump": 0.0, "dense_eigh": 0.0, "close": 0.0}
rows = []
for rep in range(2):
    for k in tot: tot[k] = 0.0
    for sec in setup_pointers(cfg):
        neigen, nitermax, nblock = lanczos_params(sec.dim, opt)
        dense = neigen == sec.dim or sec.dim <= opt.lanc_dim_threshold
        t0 = time.perf_counter()
        S = Sector(cfg, sec.q1, sec.q2, stored=True, real=True)
        t1 = time.perf_counter()
        if dense:
            rp, c, v = S.dump_csr(); t2 = time.perf_counter()
            H = np.zeros((sec.dim, sec.dim)); np.add.at(H, (np.repeat(np.arange(sec.dim), np.diff(rp)), c), v.real)
            np.linalg.eigh(H); t3 = time.perf_counter()
            tot["dense_build"] += t1 - t0; tot["dense_dump"] += t2 - t1; tot["dense_eigh"] += t3 - t2
        else:
            w, X, nconv, nhv = S.eigh(neigen=neigen, ncv=min(nblock, 64), maxit=nitermax, v0=_start_vector(sec.dim, False))
            t3 = time.perf_counter()
            tot["build"] += t1 - t0; tot["eigh"] += t3 - t1
            if rep: rows.append((t3 - t0, t1 - t0, sec.dim, nhv))
        t4 = time.perf_counter(); S.close(); tot["close"] += time.perf_counter() - t4
    print({k: round(v, 3) for k, v in tot.items()}, flush=True)
rows.sort(reverse=True)
for r in rows[:8]: print("total %.4f build %.4f dim %d nhv %d" % r)
small = [r for r in rows if r[2] < 5000]
print("small sectors", len(small), "mean total ms", 1e3 * np.mean([r[0] for r in small]), "mean nhv", np.mean([r[3] for r in small]))
