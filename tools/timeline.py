"""GPU occupancy of a rocprofv3 kernel trace (kernel_trace.csv): wall from the
first kernel start to the last end, the union of kernel-busy intervals (the
fraction of the wall with at least one kernel running), the mean number of
kernels in flight while busy, and per kernel name its summed duration and
its busy-union share.

    python tools/timeline.py kernel_trace.csv [out.json]
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"^void ", "", n)
    return n[:80]


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


rows = list(csv.DictReader(open(sys.argv[1])))
iv = []
by = defaultdict(list)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    iv.append((s, e))
    by[short(r["Kernel_Name"])].append((s, e))
t0 = min(s for s, _ in iv)
t1 = max(e for _, e in iv)
busy = union(iv)
summed = sum(e - s for s, e in iv)
out = {"kernels": len(iv), "wall_ms": (t1 - t0) / 1e6, "busy_ms": busy / 1e6, "busy_frac": busy / (t1 - t0),
       "summed_kernel_ms": summed / 1e6, "mean_in_flight_when_busy": summed / busy,
       "by_kernel": sorted(({"name": k, "calls": len(v), "summed_ms": sum(e - s for s, e in v) / 1e6,
                             "union_ms": union(v) / 1e6} for k, v in by.items()),
                           key=lambda d: -d["summed_ms"])[:20]}
print(json.dumps({k: v for k, v in out.items() if k != "by_kernel"}))
for d in out["by_kernel"][:12]:
    print(f"  {d['name'][:60]:60s} calls {d['calls']:7d} summed {d['summed_ms']:8.1f} ms union {d['union_ms']:8.1f} ms")
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
