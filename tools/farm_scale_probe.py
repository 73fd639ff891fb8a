"""Projected N-GPU wall time of the configs[3] sector farm, measured on one GPU.

farm_diag gives rank r of N the LPT part `lpt_partition(costs, N)[r]` and has no
collective until the eigenvalue all_gather (KB), so an N-GPU farm takes
max over r of (rank r's part solved alone on its GPU) + the gather.  Every
part is timed here on the one GPU, alone, exactly as farm_diag's rank would run
it (solve_many, `DiagOptions.workers` host threads); the maximum over parts is
the projected wall time.  Also records every sector's solo time, to check the
LPT cost model (sector_cost) against the measured cost.

    python tools/farm_scale_probe.py [--out gpurun_out/farm_scale.json]
"""
import argparse
import json
import os
import sys
import time

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "dmft-ed_amd"), os.path.join(os.getcwd(), "tests")]
import torch

torch.cuda.init()
from edgpu.diag import DiagOptions, solve_many, solve_sector
from edgpu.farm import lpt_partition, sector_cost
from edgpu.sectors import diag_sectors
from golden.golden_configs import c4_config

ap = argparse.ArgumentParser()
ap.add_argument("--out", default="gpurun_out/farm_scale.json")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--ranks", default="1,2,4,8")
ap.add_argument("--batch-max-dim", type=int, default=None, help="DiagOptions.batch_max_dim (default: the library's)")
ap.add_argument("--no-solo", action="store_true", help="skip the per-sector solo times")
args = ap.parse_args()

cfg = c4_config("random")
opt = DiagOptions() if args.batch_max_dim is None else DiagOptions(batch_max_dim=args.batch_max_dim)
secs = diag_sectors(cfg)
costs = [sector_cost(cfg, s, opt) for s in secs]


def run(part):
    mine = [secs[i] for i in part]
    best = None
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = list(solve_many(cfg, mine, opt, 0, solver=solve_sector, cost=lambda s: sector_cost(cfg, s, opt)))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        del out
        best = dt if best is None else min(best, dt)
    return best


run(list(range(len(secs))))  # warm-up: code objects, allocator pools
# every sector alone (one thread), to compare with the cost model
solo = []
for i, s in enumerate([] if args.no_solo else secs):
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = solve_sector(cfg, s, opt)
    torch.cuda.synchronize()
    solo.append(time.perf_counter() - t)
    del r
if solo:
    print(f"solo sum {sum(solo):.3f}s, largest {max(solo):.4f}s", flush=True)
else:
    solo = [0.0] * len(secs)

res = {"workload": "configs[3] Norb=2 Nbath=5 random bath, 169 sectors, Neigen=6 ncv=23 tol 1e-12",
       "method": "each LPT part of N ranks timed alone on one MI355X with the farm's worker threads; "
                 "projected N-GPU wall = max over parts (the eigenvalue all_gather is KB and not included)",
       "workers": opt.workers, "batch_max_dim": opt.batch_max_dim, "solo_sum_s": round(sum(solo), 4),
       "ranks": {}}
base = None
for n in [int(x) for x in args.ranks.split(",")]:
    parts = lpt_partition(costs, n)
    times = [run(p) for p in parts]
    wall = max(times)
    base = wall if n == 1 else base
    model = [sum(costs[i] for i in p) for p in parts]
    measured = [sum(solo[i] for i in p) for p in parts]
    res["ranks"][n] = {"wall_s": round(wall, 4), "part_s": [round(t, 4) for t in times],
                       "speedup": round(base / wall, 3) if base else None,
                       "model_load_rel": [round(m / max(model), 3) for m in model],
                       "solo_load_s": [round(m, 4) for m in measured]}
    print(f"N={n}: wall {wall:.4f}s parts {[round(t, 3) for t in times]} speedup {base / wall:.2f}", flush=True)

# largest sectors: cost model vs measured (skipped with --no-solo)
if args.no_solo:
    res.pop("solo_sum_s")
    for v in res["ranks"].values():
        v.pop("solo_load_s")
res["solo"] = [{"sector": [s.q1, s.q2], "dim": s.dim, "solo_s": round(solo[i], 5), "cost_model": costs[i]}
               for i, s in enumerate(secs)]
top = sorted(range(len(secs)), key=lambda i: -solo[i])[:12]
res["largest"] = [{"sector": [secs[i].q1, secs[i].q2], "dim": secs[i].dim, "solo_s": round(solo[i], 4),
                   "cost_model": costs[i]} for i in top]
if args.no_solo:
    del res["solo"], res["largest"]
os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
with open(args.out, "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res["ranks"]))
