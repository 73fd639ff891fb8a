"""configs[3] farm on one host thread (for rocprofv3 kernel statistics)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmft-ed_amd"), os.path.join(ROOT, "tests")]
import torch

torch.cuda.init()
from edgpu.diag import DiagOptions
from edgpu.farm import farm_diag
from golden.golden_configs import c4_config

cfg = c4_config("random")
opt = DiagOptions(workers=int(sys.argv[1]) if len(sys.argv) > 1 else 1)
t = time.perf_counter()
res = farm_diag(cfg, opt)
torch.cuda.synchronize()
print(f"farm workers={opt.workers} wall {time.perf_counter() - t:.3f} s E0 {res.states.emin:.10f}")
