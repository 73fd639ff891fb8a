"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel, the number
of dispatches and the median counter value (kB as rocprofv3 reports FETCH_SIZE
/ WRITE_SIZE) -> JSON on stdout.

usage: python tools/pmc_summary.py <dir-or-csv> [...]
"""
import csv
import glob
import json
import os
import statistics
import sys


def summarise(path):
    files = [path] if path.endswith(".csv") else glob.glob(os.path.join(path, "**", "*counter_collection.csv"),
                                                          recursive=True)
    out = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = (row["Kernel_Name"][:90], row["Counter_Name"])
                out.setdefault(k, []).append(float(row["Counter_Value"]))
    res = []
    for (kern, ctr), vals in sorted(out.items()):
        res.append({"kernel": kern, "counter": ctr, "dispatches": len(vals),
                    "median": statistics.median(vals), "min": min(vals), "max": max(vals)})
    return res


if __name__ == "__main__":
    allr = {}
    for p in sys.argv[1:]:
        allr[os.path.basename(p.rstrip("/"))] = summarise(p)
    json.dump(allr, sys.stdout, indent=1)
    print()
