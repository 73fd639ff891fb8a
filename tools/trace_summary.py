"""Per-launch kernel durations from a rocprofv3 --kernel-trace CSV, split
into the warm-up launches and the steady-state ones — the same launches
bench.py times with HIP events (after its warm-ups), so the line's
`ms_per_launch` can be recomputed from profiles/.

usage: python tools/trace_summary.py TRACE.csv KERNEL_REGEX SKIP OUT.json [--grid X] [--note TEXT]

SKIP = dispatches of the matching kernel(s) dropped at the start (the
probe's warm-up launches); --grid keeps only dispatches of that grid size
(Grid_Size_X: one sector's launches inside a whole bench.py trace).
Durations are End - Start of each dispatch (ns).  Several kernels matching the regex in one H·v (the two-pass Kronecker form)
are summed per launch in dispatch order.
"""
import argparse
import csv
import json
import re
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("pat")
    ap.add_argument("skip", type=int)
    ap.add_argument("out")
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    path, skip, out, note = a.trace, a.skip, a.out, a.note
    rx = re.compile(a.pat)
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if rx.search(r["Kernel_Name"]) and (a.grid is None or int(r["Grid_Size_X"]) == a.grid):
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"],
                             int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), int(r["Grid_Size_X"])))
    rows.sort()
    names = sorted({n for _, n, _, _ in rows})
    per = len(names)  # kernels per H·v (1, or 2 for the two-pass form)
    launches = [sum(d for _, _, d, _ in rows[i:i + per]) for i in range(0, len(rows) - per + 1, per)]
    # per (kernel, grid): one sector's launches when a trace holds several
    # sectors' (a whole bench.py run); each group's first SKIP dropped
    groups = {}
    for _, n, d, g in rows:
        groups.setdefault(f"{n[:60]} | grid {g}", []).append(d)
    by_grid = {k: {"launches": len(v), "steady_mean_ns": round(statistics.fmean(v[skip:]), 1) if v[skip:] else None}
               for k, v in groups.items()}
    # runs: maximal stretches of consecutive dispatch ids of one (kernel,
    # grid) — one measurement loop of one sector (sectors of equal dimension
    # share a grid; the kernels that build the next sector break the run)
    runs = []
    for did, n, d, g in rows:
        r = runs[-1] if runs else None
        if r and r["kernel"] == n[:80] and r["grid_size_x"] == g and did == r["_last"] + 1:
            r["_d"].append(d)
            r["_last"] = did
        else:
            runs.append({"kernel": n[:80], "grid_size_x": g, "first_dispatch": did, "_last": did, "_d": [d]})
    for r in runs:
        dd = r.pop("_d")
        r.pop("_last")
        r["launches"] = len(dd)
        r["steady_mean_ns"] = round(statistics.fmean(dd[skip:]), 1) if dd[skip:] else None
    runs = [r for r in runs if r["launches"] > skip]
    steady = launches[skip:]
    if not steady:
        raise SystemExit("no steady-state launches")
    res = {
        "trace": path.split("gpurun_out/")[-1],
        "kernels": [n[:160] for n in names],
        "grid_size_x": a.grid,
        "launches": len(launches),
        "warmup_dropped": skip,
        "warmup_ns": launches[:skip],
        "steady_mean_ns": round(statistics.fmean(steady), 1),
        "steady_median_ns": float(statistics.median(steady)),
        "steady_min_ns": min(steady),
        "steady_max_ns": max(steady),
        "all_mean_ns": round(statistics.fmean(launches), 1),
        "by_kernel_grid": by_grid,
        "runs": runs,
        "note": note,
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: res[k] for k in ("launches", "steady_mean_ns", "steady_median_ns", "all_mean_ns")}))


if __name__ == "__main__":
    main()
