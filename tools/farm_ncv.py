"""configs[3] farm wall time and H·v count vs the thick-restart basis size
(ncv = lanc_ncv_factor*6 + lanc_ncv_add; the reference's Nblock is 23)."""
import os
import sys
import time

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "dmft-ed_amd"), os.path.join(os.getcwd(), "tests")]
import numpy as np
import torch

torch.cuda.init()
from edgpu.diag import DiagOptions
from edgpu.farm import farm_diag
from golden.golden_configs import c4_config
import json

cfg = c4_config("random")
gold = json.load(open(os.path.join("tests", "golden", "c4_diag_random.json")))
for add in (5, -5, 0, 11, 17):
    opt = DiagOptions(lanc_ncv_add=add)
    farm_diag(cfg, opt)
    best = 1e9
    for _ in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        res = farm_diag(cfg, opt)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    worst = max(float(np.max(np.abs(np.asarray(res.eigenvalues[int(k)])[: len(g["eigenvalues"])]
                                     - np.asarray(g["eigenvalues"])))) for k, g in gold["sectors"].items())
    print(f"ncv={3 * 6 + add} farm wall {best:.3f} s worst eigenvalue dev {worst:.1e}", flush=True)
