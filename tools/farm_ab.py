"""configs[3] farm wall time with and without the eigensolver's deflated
verification (ED_GPU_EIGH_NO_VERIFY), and the H·v count per sector class."""
import os
import sys
import time

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "dmft-ed_amd"), os.path.join(os.getcwd(), "tests")]
import numpy as np
import torch

torch.cuda.init()
from edgpu.diag import DiagOptions, _start_vector, lanczos_params
from edgpu.farm import farm_diag
from edgpu.hamiltonian import Sector
from edgpu.sectors import setup_pointers
from golden.golden_configs import c4_config

cfg = c4_config(sys.argv[1] if len(sys.argv) > 1 else "random")
opt = DiagOptions()
for nv in (False, True, False, True):
    if nv:
        os.environ["ED_GPU_EIGH_NO_VERIFY"] = "1"
    else:
        os.environ.pop("ED_GPU_EIGH_NO_VERIFY", None)
    torch.cuda.synchronize()
    t = time.perf_counter()
    res = farm_diag(cfg, opt)
    torch.cuda.synchronize()
    print(f"no_verify={nv} farm wall {time.perf_counter() - t:.3f} s E0 {res.states.emin:.10f}", flush=True)
# H·v counts and times of the largest sectors, serial
rows = []
for verify in (True, False):
    if verify:
        os.environ.pop("ED_GPU_EIGH_NO_VERIFY", None)
    else:
        os.environ["ED_GPU_EIGH_NO_VERIFY"] = "1"
    tot_hv = 0
    tot_t = 0.0
    for sec in setup_pointers(cfg):
        neigen, nitermax, nblock = lanczos_params(sec.dim, opt)
        if neigen == sec.dim or sec.dim <= opt.lanc_dim_threshold:
            continue
        with Sector(cfg, sec.q1, sec.q2, stored=True, real=True) as S:
            t = time.perf_counter()
            w, X, nconv, nhv = S.eigh(neigen=neigen, ncv=min(nblock, 64), maxit=nitermax,
                                      v0=_start_vector(sec.dim, False), on_device=True)
            dt = time.perf_counter() - t
        tot_hv += nhv
        tot_t += dt
        if verify:
            rows.append((sec.dim, nhv, dt))
    print(f"verify={verify}: serial eigh {tot_t:.3f} s, {tot_hv} H.v products", flush=True)
rows.sort(reverse=True)
for r in rows[:6]:
    print("dim %8d nhv %4d %.4f s" % r)
