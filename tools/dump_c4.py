"""Dump the device ed_diag eigenvalues of configs[3] (flat and random bath) for
comparison with the committed fixtures (diagnostic)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "dmft-ed_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
from edgpu.diag import DiagOptions  # noqa: E402
from edgpu.farm import farm_diag  # noqa: E402
from golden.golden_configs import c4_config  # noqa: E402

out = {}
for bath in ("flat", "random"):
    res = farm_diag(c4_config(bath), DiagOptions())
    out[bath] = {str(k): [float(x) for x in v] for k, v in res.eigenvalues.items()}
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "c4_dump.json"), "w") as fh:
    json.dump(out, fh)
print("dumped")
