"""A/B of the stored H·v forms on the HBM-sized sectors, one process: the
fused one-pass re-laid kernel (default where built), the two-segment form /
one-pass packed kernel (ED_OPT_NO_FUSED) and the bit-exact one-pass kernel
(ED_OPT_STORED_EXACT), real and complex vectors, real and complex(8) H.

    python tools/fused_ab.py [--iters N] [--sectors n28,n26s,...] [--json out.json]

Prints HIP-event milliseconds per launch on the launch stream (median of
five 10-launch windows) and writes them to --json.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dmft-ed_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from edgpu.hamiltonian import Sector  # noqa: E402
from edgpu.params import make_config  # noqa: E402

SECTORS = {
    "n28": (dict(Norb=1, Nbath=13), (7, 7)),
    "n28b": (dict(Norb=2, Nbath=6), (7, 7)),
    "n28j": (dict(Norb=2, Nbath=6, Uloc=(2.0, 2.0, 0.0), Ust=1.0, Jh=0.5, Jx=0.5, Jp=0.5), (7, 7)),
    "n26s": (dict(Norb=1, Nbath=12, Nspin=2, ed_mode="nonsu2"), (13, 0)),
}

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--sectors", default="n28,n26s,n28b,n28j")
ap.add_argument("--json", default="")
ap.add_argument("--lib", default="", help="load this libedgpu.so build instead (A/B of kernel variants)")
a = ap.parse_args()
if a.lib:
    import edgpu._lib as _edl
    _edl.LIB_PATH = os.path.abspath(a.lib)


def timed(S, x, y, st, n):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    out = []
    for _ in range(5):
        ev[0].record(st)
        for _ in range(n):
            S.hxv_dev(x, y, path=0, stream=st)
        ev[1].record(st)
        ev[1].synchronize()
        out.append(ev[0].elapsed_time(ev[1]) / n)
    return float(np.median(out))


res = {}
st = torch.cuda.Stream()
for name in a.sectors.split(","):
    kw, q = SECTORS[name]
    cfg = make_config(bath="random", seed=20251015, **kw)
    for real_h in (True, False):
        with torch.cuda.stream(st), Sector(cfg, q[0], q[1], stored=True, real=real_h, stream=st) as S:
            inf = S.info
            for cvec in ((False, True) if real_h else (True,)):
                dt = torch.complex128 if cvec else torch.float64
                i = torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda")
                x = (torch.complex(torch.sin(i), torch.cos(3 * i)) if cvec else torch.sin(i)).to(dt)
                y = torch.empty_like(x)
                row = {}
                ref = None
                for label, opts in (("default", ()), ("no_fused", ("no_fused",)), ("exact", ("stored_exact",))):
                    S.set_options(*opts)
                    for _ in range(3):
                        S.hxv_dev(x, y, path=0, stream=st)
                    st.synchronize()
                    if ref is None:
                        ref = y.clone()
                    dev = float((y - ref).abs().max() / ref.abs().max())
                    row[label] = round(timed(S, x, y, st, a.iters), 4)
                    row[label + "_dev"] = dev
                S.set_options()
                key = f"{name}/{'cH' if not real_h else 'rH'}/{'cv' if cvec else 'rv'}"
                row.update(dim=S.dim, nnz=S.nnz, fused=inf.fused, split=inf.split,
                           fused_far=inf.fused_far, fused_far_uniform=inf.fused_far_uniform,
                           fused_bytes=inf.fused_bytes, split_bytes=inf.split_bytes)
                res[key] = row
                print(key, row, flush=True)
if a.json:
    with open(a.json, "w") as fh:
        json.dump(res, fh, indent=1)
