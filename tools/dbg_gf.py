import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "dmft-ed_amd"), os.path.join(os.getcwd(), "tests")]
import numpy as np
import torch
torch.cuda.init()
import edgpu.gf as gf
from edgpu.diag import DiagOptions, ed_diag
from edgpu.params import make_config
cfg = make_config(Norb=1, Nbath=4, Nspin=2, ed_mode="nonsu2")
_, sl = ed_diag(cfg, DiagOptions(lanc_method="lanczos"))
orig = gf.tridiag_poles
def tp(a, b, n):
    if not (np.all(np.isfinite(a[:n])) and np.all(np.isfinite(b[:n]))):
        print("NONFINITE", n, a[:8], b[:8])
    try:
        return orig(a, b, n)
    except Exception as e:
        print("FAIL", n, "a", a[:n], "b", b[:n])
        raise
gf.tridiag_poles = tp
orig_tri = gf._tridiag_dev
def td(S, seed, nlanc, real, thr):
    a, b, n = orig_tri(S, seed, nlanc, real, thr)
    print("dim", S.dim, "real", real, "mode", S.lanc_mode(real=real), "nlanc", nlanc, "n", n, "finite", np.all(np.isfinite(a)), flush=True)
    return a, b, n
gf._tridiag_dev = td
gf.build_gf(cfg, sl, gf.GFOptions(Lmats=30, Lreal=30))
