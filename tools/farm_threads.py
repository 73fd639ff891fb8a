"""configs[3] farm wall time on one GPU vs host worker threads."""
import os, sys, time
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "dmft-ed_amd")]
import torch
torch.cuda.init()
from edgpu.params import make_config
from edgpu.diag import DiagOptions, ed_diag

cfg = make_config(Norb=2, Nbath=5, bath="random", seed=20251015)
ed_diag(cfg, DiagOptions(workers=1))
for w in (1, 2, 4, 8):
    t = time.perf_counter()
    res, sl = ed_diag(cfg, DiagOptions(workers=w))
    print(f"workers={w} wall={time.perf_counter() - t:.3f}s E0={sl.emin:.10f} n={sl.size}", flush=True)
