"""Phase breakdown of the configs[3] farm on one GPU (profiles/r2/farm_c4_phases.json).

Serial pass over the 169 sectors (one host thread, so the phases add up):
  build  - Sector create: host tables + device H assembly (k_count/k_fill/pack)
  solve  - device thick-restart Lanczos (ed_sector_eigh), eigenvectors kept in HBM
  d2h    - what copying those eigenvectors to the host would cost (torch .cpu())
  dense  - the small sectors: CSR dump + host LAPACK eigh
  close  - Sector destroy
then the farm itself (8 worker threads) with device-resident vectors (default)
and with host copies of every sector's vectors (round-1 behaviour).
"""
import json
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

cfg = c4_config("random")
opt = DiagOptions()
phases = {}
for rep in range(2):
    tot = {"build": 0.0, "solve": 0.0, "d2h": 0.0, "dense": 0.0, "close": 0.0}
    d2h_bytes = 0
    for sec in setup_pointers(cfg):
        neigen, nitermax, nblock = lanczos_params(sec.dim, opt)
        dense = neigen == sec.dim or sec.dim <= opt.lanc_dim_threshold
        t0 = time.perf_counter()
        S = Sector(cfg, sec.q1, sec.q2, stored=True, real=True)
        t1 = time.perf_counter()
        if dense:
            rp, c, v = S.dump_csr()
            H = np.zeros((sec.dim, sec.dim))
            np.add.at(H, (np.repeat(np.arange(sec.dim), np.diff(rp)), c), v.real)
            np.linalg.eigh(H)
            tot["build"] += t1 - t0
            tot["dense"] += time.perf_counter() - t1
        else:
            w, X, nconv, nhv = S.eigh(neigen=neigen, ncv=min(nblock, 64), maxit=nitermax,
                                      v0=_start_vector(sec.dim, False), on_device=True)
            t2 = time.perf_counter()
            X.T.cpu()
            t3 = time.perf_counter()
            tot["build"] += t1 - t0
            tot["solve"] += t2 - t1
            tot["d2h"] += t3 - t2
            d2h_bytes += X.numel() * 8
        t4 = time.perf_counter()
        S.close()
        tot["close"] += time.perf_counter() - t4
    phases = {k: round(v, 4) for k, v in tot.items()}
    phases["d2h_bytes"] = d2h_bytes
    print(phases, flush=True)


def farm_wall(device_vectors):
    o = DiagOptions(device_vectors=device_vectors)
    farm_diag(cfg, o)
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        res = farm_diag(cfg, o)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best, res


wd, rd = farm_wall(True)
wh, rh = farm_wall(False)
assert rd.states.sectors == rh.states.sectors
out = {"config": "configs[3] Norb=2 Nbath=5 random bath (seed 20251015), 169 sectors, arpack path",
       "serial_phases_s": phases,
       "farm_wall_s_device_vectors": round(wd, 4),
       "farm_wall_s_host_vectors": round(wh, 4),
       "kept_states": len(rd.states.sectors),
       "note": "serial phases on one host thread; farm walls are best of 3 with 8 worker threads"}
print(json.dumps(out))
os.makedirs("gpurun_out", exist_ok=True)
with open(os.path.join("gpurun_out", "farm_c4_phases.json"), "w") as f:
    json.dump(out, f, indent=1)
