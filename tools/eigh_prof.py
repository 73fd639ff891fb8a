"""Kernel-level profile of the device thick-restart eigh on the configs[3]
half-filled (6,6) sector (dim 853,776; or the sector given as `q1 q2` on the
command line): run under rocprofv3 --kernel-trace --stats."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dmft-ed_amd"))
import torch  # noqa: E402
torch.cuda.init()
if os.environ.get("ED_LIB"):  # A/B of library builds
    import edgpu._lib as _edl  # noqa: E402
    _edl.LIB_PATH = os.path.abspath(os.environ["ED_LIB"])
from edgpu.params import make_config  # noqa: E402
from edgpu.hamiltonian import Sector  # noqa: E402

cfg = make_config(Norb=2, Nbath=5, bath="random", seed=20251015)
q1, q2 = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (6, 6)
mf = os.environ.get("ED_FORM") == "direct"   # matrix-free H·v (the Kronecker two-pass form when the sector has it)
with Sector(cfg, q1, q2, stored=not mf, direct=mf, real=True) as S:
    opts = [o for o in os.environ.get("ED_OPTS", "").split(",") if o]   # ED_OPT_* names (A/B)
    if opts:
        S.set_options(*opts)
    print(f"form {'matrix-free' if mf else 'stored'} kron={S.info.kron} options {opts}", flush=True)
    S.eigh(vectors=False)
    for _ in range(3):
        torch.cuda.synchronize(); t = time.perf_counter()
        ev, _, nconv, nhv = S.eigh(vectors=False)
        torch.cuda.synchronize(); dt = time.perf_counter() - t
        print(f"eigh ({q1},{q2}) dim {S.dim}: {dt*1e3:.2f} ms, nhv {nhv}, {dt/nhv*1e6:.1f} us per H·v step, E0 {ev[0]:.10f}", flush=True)
