"""cProfile of the configs[4] nonSU2 Green's function (12 seeds, L=5000) on one GPU."""
import cProfile, os, pstats, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dmft-ed_amd"))
import torch  # noqa: E402
torch.cuda.init()
from edgpu.diag import DiagOptions  # noqa: E402
from edgpu.farm import farm_diag  # noqa: E402
from edgpu.gf import GFOptions, build_gf  # noqa: E402
from edgpu.params import make_config  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tests"))
from golden.golden_configs import c5_config
cfg = c5_config("random")
res = farm_diag(cfg, DiagOptions(), device=0)
g = GFOptions()
build_gf(cfg, res.states, g, device=0)
for _ in range(2):
    torch.cuda.synchronize(); t = time.perf_counter()
    Gm, _ = build_gf(cfg, res.states, g, device=0)
    print(f"build_gf {1e3 * (time.perf_counter() - t):.1f} ms G00(iw0) {Gm[0,0,0,0,0]:.10f}", flush=True)
pr = cProfile.Profile()
pr.enable(); build_gf(cfg, res.states, g, device=0); pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
