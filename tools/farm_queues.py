"""configs[3] farm wall time on one GPU vs host worker threads, for the
hardware-queue count given in GPU_MAX_HW_QUEUES (set by the caller before HIP
starts; HIP's default is 4, so 8 worker streams share 4 hardware queues).

    GPU_MAX_HW_QUEUES=8 python tools/farm_queues.py
"""
import os
import sys
import time

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "dmft-ed_amd"), os.path.join(os.getcwd(), "tests")]
import torch

torch.cuda.init()
from edgpu.diag import DiagOptions, ed_diag
from golden.golden_configs import c4_config

cfg = c4_config("random")
ed_diag(cfg, DiagOptions(workers=8))
q = os.environ.get("GPU_MAX_HW_QUEUES", "default")
for w in (4, 8, 12, 16):
    best = None
    for _ in range(2):
        t = time.perf_counter()
        res, sl = ed_diag(cfg, DiagOptions(workers=w))
        dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
        del res, sl
    print(f"queues={q} workers={w} wall={best:.3f}s", flush=True)
