"""Oracle-backed sector solver with the edgpu.diag.solve_sector signature.

Test infrastructure: lets the farm / sector-loop logic run on CPU (gloo) and
serves as the reference the GPU ed_diag is compared with.
"""
import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as sla

from edgpu.diag import SectorResult, lanczos_params
from oracle.oracle import Oracle


def solve_sector_oracle(cfg, sec, opt, device=0):
    orc = Oracle(cfg)
    hmap = orc.build_sector(sec.q1, sec.q2)
    rp, cols, vals = orc.build_csr(hmap)
    dim = len(hmap)
    neigen, nitermax, nblock = lanczos_params(dim, opt)
    A = sp.csr_matrix((vals, cols, rp), shape=(dim, dim))
    dense = neigen == dim or dim <= max(opt.lanc_dim_threshold, opt.mpi_size)
    if dense or opt.lanc_method == "dense":
        w, v = np.linalg.eigh(A.toarray())
        return SectorResult(sec.isector, (sec.q1, sec.q2), dim, w, neigen, v[:, :neigen], "dense")
    k = 1 if opt.lanc_method == "lanczos" else neigen
    # fixed start vector: ARPACK's internal random start advances across calls
    i = np.arange(1, dim + 1, dtype=np.float64)
    v0 = np.sin(i) + 1j * np.cos(3.0 * i) if np.iscomplexobj(A.data) else np.sin(i)
    w, v = sla.eigsh(A, k=k, which="SA", tol=1e-13, v0=v0)
    o = np.argsort(w)
    return SectorResult(sec.isector, (sec.q1, sec.q2), dim, w[o], k, v[:, o], "eigsh")
