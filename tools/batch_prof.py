"""Time the batched small-sector eigh (ed_sectors_eigh_batch) on configs[3]:
sector builds, the batch solve and the closes separately, against the same
sectors solved one after the other with ed_sector_eigh.

    python tools/batch_prof.py [--bath random] [--max-dim N] [--reps 3] [--single]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmft-ed_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

torch.cuda.init()
from edgpu.diag import DiagOptions, _start_vector, batchable, lanczos_params  # noqa: E402
from edgpu.hamiltonian import Sector, eigh_batch  # noqa: E402
from edgpu.sectors import diag_sectors  # noqa: E402
from golden.golden_configs import c4_config  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--bath", default="random")
ap.add_argument("--max-dim", type=int, default=None, help="DiagOptions.batch_max_dim (default: the library's)")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--single", action="store_true", help="also the per-sector solves")
a = ap.parse_args()
cfg = c4_config(a.bath)
opt = DiagOptions() if a.max_dim is None else DiagOptions(batch_max_dim=a.max_dim)
secs = [s for s in diag_sectors(cfg) if batchable(cfg, s, opt)]
st = torch.cuda.Stream()
print(f"{len(secs)} batchable sectors, dims {min(s.dim for s in secs)}-{max(s.dim for s in secs)}", flush=True)
for rep in range(a.reps):
    t0 = time.perf_counter()
    hs = [Sector(cfg, s.q1, s.q2, stored=True, real=True, stream=st) for s in secs]
    t1 = time.perf_counter()
    groups = {}
    for h, s in zip(hs, secs):
        ne, nit, nb = lanczos_params(s.dim, opt)
        groups.setdefault((ne, min(nb, 64, s.dim)), []).append(h)
    nhv = nbat = 0
    for (ne, ncv), g in groups.items():
        mx = [max(lanczos_params(h.dim, opt)[1], 10) for h in g]
        res, nb = eigh_batch(g, ne, ncv, mx, opt.lanc_tolerance, [_start_vector(h.dim, False) for h in g],
                             vectors=True, on_device=True, stream=st)
        nhv += sum(r[3] for r in res)
        nbat += nb
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    if a.single and rep == 0:
        for h, s in zip(hs, secs):
            ne, nit, nb = lanczos_params(s.dim, opt)
            h.eigh(neigen=ne, ncv=min(nb, 64, s.dim), maxit=max(nit, 10), v0=_start_vector(h.dim, False),
                   on_device=True)
        torch.cuda.synchronize()
        print(f"  single: {time.perf_counter() - t2:.4f} s", flush=True)
        t2 = time.perf_counter()
    for h in hs:
        h.close()
    t3 = time.perf_counter()
    print(f"rep {rep}: create {t1 - t0:.4f} s, batch eigh {t2 - t1:.4f} s ({nbat} in batch, {nhv} H·v), "
          f"close {t3 - t2:.4f} s", flush=True)
