"""Time the configs[3] sector farm (Norb=2 Nbath=5, 169 sectors) on one GPU:
device thick-restart eigh vs the earlier host-ARPACK (scipy) + device H·v path."""
import os, sys, time
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "dmft-ed_amd")]
import numpy as np
import torch
torch.cuda.init()
from edgpu.params import make_config
from edgpu.diag import DiagOptions, ed_diag, solve_sector
from edgpu.sectors import setup_pointers
from edgpu.hamiltonian import Sector

cfg = make_config(Norb=2, Nbath=5, bath="random", seed=20251015)
secs = {(s.q1, s.q2): s for s in setup_pointers(cfg)}
opt = DiagOptions()
big = secs[(6, 6)]
for rep in range(2):
    t = time.perf_counter()
    r = solve_sector(cfg, big, opt)
    print(f"(6,6) dim {big.dim} device eigh: {time.perf_counter()-t:.3f}s  E={r.eigenvalues[:3]}", flush=True)
with Sector(cfg, 6, 6, stored=True, real=True) as S:
    t = time.perf_counter(); S.eigh(); print(f"  eigh only {time.perf_counter()-t:.3f}s", flush=True)
    ev, _, nconv, nhv = S.eigh(vectors=False)
    t = time.perf_counter(); S.eigh(vectors=False); dt = time.perf_counter()-t
    print(f"  eigh no-vec {dt:.3f}s nhv {nhv} -> {dt/nhv*1e3:.3f} ms per H·v step", flush=True)
    import scipy.sparse.linalg as sla
    xd = torch.empty(big.dim, dtype=torch.float64, device="cuda"); yd = torch.empty_like(xd)
    def mv(x):
        xd.copy_(torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64).ravel())); S.hxv_dev(xd, yd)
        return yd.cpu().numpy()
    op = sla.LinearOperator((big.dim, big.dim), matvec=mv, dtype=np.float64)
    i = np.arange(1, big.dim + 1.0)
    t = time.perf_counter()
    w, v = sla.eigsh(op, k=6, which="SA", ncv=23, tol=1e-12, v0=np.sin(i))
    print(f"  host ARPACK + device H·v: {time.perf_counter()-t:.3f}s  maxdiff {np.max(np.abs(np.sort(w)-ev)):.2e}", flush=True)
for rep in range(2):
    t = time.perf_counter()
    res, sl = ed_diag(cfg, opt)
    print(f"farm serial 169 sectors: {time.perf_counter()-t:.3f}s  E0 {sl.emin:.10f} nstates {sl.size}", flush=True)
from collections import Counter
print(Counter(r.method for r in res))
