"""configs[4] (nonSU2 Norb=1 Nbath=6, random bath): ground state over all
sectors + the 12-seed Green's function, on one GPU with ONE farm worker thread
(the form that runs under rocprofv3 --kernel-trace: tools/farm_rocprof.sh).

    python tools/c5_run.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dmft-ed_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

torch.cuda.init()
from edgpu.diag import DiagOptions  # noqa: E402
from edgpu.farm import farm_diag  # noqa: E402
from edgpu.gf import GFOptions, build_gf  # noqa: E402
from golden.golden_configs import c5_config  # noqa: E402

cfg = c5_config("random")
t = time.perf_counter()
res = farm_diag(cfg, DiagOptions(workers=1), device=0)
torch.cuda.synchronize()
t1 = time.perf_counter()
Gm, _ = build_gf(cfg, res.states, GFOptions(), device=0)
torch.cuda.synchronize()
print(f"c5 diag {t1 - t:.4f} s gf {time.perf_counter() - t1:.4f} s E0 {res.states.emin:.10f}", flush=True)
