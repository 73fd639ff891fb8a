"""Where the two-pass matrix-free Kronecker H·v (k_kron_up + k_kron_dw) starts
to beat the one-pass k_kron: H·v time of configs[3] sectors of growing dim
with Sector(kron2=False) (one pass) and kron2=True (two pass), HIP events, 50 launches.

    python tools/kron2_threshold.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dmft-ed_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from edgpu.hamiltonian import Sector  # noqa: E402
from golden.golden_configs import c4_config  # noqa: E402

cfg = c4_config("random")
out = []
for q in [(3, 3), (3, 4), (4, 4), (4, 5), (5, 5), (5, 6), (6, 6)]:
    row = {"sector": q}
    for k in ("0", "1"):
        with Sector(cfg, q[0], q[1], stored=False, direct=True, real=True, kron2=(k == "1")) as S:
            i = torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda")
            x = torch.sin(i)
            y = torch.empty_like(x)
            st = torch.cuda.current_stream()
            for _ in range(5):
                S.hxv_dev(x, y, path=2, stream=st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(50):
                S.hxv_dev(x, y, path=2, stream=st)
            e1.record(st)
            e1.synchronize()
            row["dim"] = S.dim
            row["two_pass" if k == "1" else "one_pass"] = round(e0.elapsed_time(e1) / 50, 5)
    print(row, flush=True)
    out.append(row)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "kron2_threshold.json"), "w") as f:
    json.dump(out, f, indent=1)
