"""Launch one H·v kernel repeatedly on a chosen sector (for rocprofv3 runs).

usage: python tools/spmv_probe.py [--sector n28|n28b|n28j|n26s|c4|c4r|c2] [--path 0|1|2] [--complex] [--iters N]
Prints the HIP-event average per launch on the launch stream.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dmft-ed_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from edgpu.hamiltonian import Sector  # noqa: E402
from edgpu.params import make_config  # noqa: E402

SECTORS = {
    "n28": (dict(Norb=1, Nbath=13), (7, 7)),
    "n28b": (dict(Norb=2, Nbath=6), (7, 7)),
    "c4": (dict(Norb=2, Nbath=5), (6, 6)),
    "c2": (dict(Norb=1, Nbath=7), (4, 4)),
    # HBM-sized sectors without the Kronecker form (stored or generic matrix-free only)
    "n28j": (dict(Norb=2, Nbath=6, Uloc=(2.0, 2.0, 0.0), Ust=1.0, Jh=0.5, Jx=0.5, Jp=0.5), (7, 7)),
    "n26s": (dict(Norb=1, Nbath=12, Nspin=2, ed_mode="nonsu2"), (13, 0)),
}

ap = argparse.ArgumentParser()
ap.add_argument("--sector", default="n28")
ap.add_argument("--path", type=int, default=0)
ap.add_argument("--complex", action="store_true", help="complex(8) H values (and vectors)")
ap.add_argument("--cvec", action="store_true", help="real H, complex vectors")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--options", default="", help="comma-separated ED_OPT_* names")
ap.add_argument("--split", default="default", choices=["default", "on", "off"],
                help="two-segment stored form: library default, forced on, or not built")
ap.add_argument("--fused", default="default", choices=["default", "on", "off"],
                help="fused one-pass re-laid stored form: library default, forced on, or not built")
ap.add_argument("--lib", default="", help="load this libedgpu.so build instead (A/B of kernel variants)")
a = ap.parse_args()
if a.lib:
    import edgpu._lib as _edl
    _edl.LIB_PATH = os.path.abspath(a.lib)
if a.sector == "c4r":   # bench.py's configs[3] parameters (Uloc=(2,2,0), Ust=1, Jh=0.5), (6,6)
    from golden.golden_configs import c4_config
    cfg, q = c4_config("random"), (6, 6)
else:
    kw, q = SECTORS[a.sector]
    cfg = make_config(bath="random", seed=20251015, **kw)
real = not a.complex
opts = tuple(o for o in a.options.split(",") if o)
split = {"default": None, "on": True, "off": False}[a.split]
fused = {"default": None, "on": True, "off": False}[a.fused]
with Sector(cfg, q[0], q[1], stored=(a.path == 0), direct=(a.path != 0), real=real, split=split,
            fused=fused, options=opts) as S:
    dt = torch.float64 if (real and not a.cvec) else torch.complex128
    i = torch.arange(1, S.dim + 1, dtype=torch.float64, device="cuda")
    x = torch.sin(i) if dt == torch.float64 else torch.complex(torch.sin(i), torch.cos(3 * i))
    x = x.to(dt).contiguous()
    y = torch.empty_like(x)
    st = torch.cuda.current_stream()
    for _ in range(3):
        S.hxv_dev(x, y, path=a.path, stream=st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(a.iters):
        S.hxv_dev(x, y, path=a.path, stream=st)
    e1.record(st)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    # the same launches bracketed one by one (what a per-dispatch trace sees)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
    for b, e in ev:
        b.record(st)
        S.hxv_dev(x, y, path=a.path, stream=st)
        e.record(st)
    ev[-1][1].synchronize()
    each = sorted(b.elapsed_time(e) for b, e in ev)
    print(f"per-launch events: mean {sum(each) / len(each):.5f} min {each[0]:.5f} median {each[len(each) // 2]:.5f} ms")
    print(f"sector={a.sector} dim={S.dim} nnz={S.nnz} padded={S.info.padded} path={a.path} "
          f"real={real} cvec={a.cvec} packed={S.info.packed} ndict={S.info.npdict} ms/launch={ms:.5f}")
    if S.info.split:
        print(f"split: far={S.info.split_far} uniform={S.info.split_far_uniform} bytes={S.info.split_bytes}")
