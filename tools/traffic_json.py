"""Per-launch HBM traffic summaries for bench.py's roofline lines.

usage: python tools/traffic_json.py OUT.json KERNEL_REGEX FETCH_DIR WRITE_DIR [note]
       python tools/traffic_json.py --calib OUT.json FETCH_DIR WRITE_DIR

FETCH_DIR / WRITE_DIR are rocprofv3 `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
output directories (one counter per pass).  rocprofv3 reports both in KiB;
the gfx950 correction is x2 on FETCH_SIZE and x1 on WRITE_SIZE, measured in
this repository by tools/fetch_calib.hip (1 GiB streamed with 4-, 8- and
16-byte lane loads: FETCH_SIZE = 0.5 GiB for each width, WRITE_SIZE = 1 GiB)
— see the --calib summary.  Kernels matching KERNEL_REGEX are summed per
launch (median over the dispatches of each kernel).
"""
import json
import os
import re
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarise  # noqa: E402

FETCH_X = 2.0
WRITE_X = 1.0


def per_kernel(d, counter):
    out = {}
    for r in summarise(d):
        if r["counter"] == counter:
            out[r["kernel"]] = r["median"] * 1024.0
    return out


def main():
    if sys.argv[1] == "--calib":
        out, fd, wd = sys.argv[2:5]
        f, w = per_kernel(fd, "FETCH_SIZE"), per_kernel(wd, "WRITE_SIZE")
        gib = float(1 << 30)
        rows = {}
        for k, v in f.items():
            m = re.search(r"k_(read|write)<([^>]*>?)", k)
            if m and m.group(1) == "read":
                rows["read " + m.group(2)] = {"FETCH_SIZE_bytes": v, "true_bytes": gib, "factor": gib / v}
        for k, v in w.items():
            m = re.search(r"k_(read|write)<([^>]*>?)", k)
            if m and m.group(1) == "write":
                rows["write " + m.group(2)] = {"WRITE_SIZE_bytes": v, "true_bytes": gib, "factor": gib / v}
        res = {"probe": "tools/fetch_calib.hip: 1 GiB buffer (4x the Infinity Cache) streamed once per launch",
               "widths": rows, "fetch_factor": FETCH_X, "write_factor": WRITE_X}
    else:
        out, pat, fd, wd = sys.argv[1:5]
        note = sys.argv[5] if len(sys.argv) > 5 else ""
        rx = re.compile(pat)
        f = {k: v for k, v in per_kernel(fd, "FETCH_SIZE").items() if rx.search(k)}
        w = {k: v for k, v in per_kernel(wd, "WRITE_SIZE").items() if rx.search(k)}
        fetch = FETCH_X * sum(f.values())
        write = WRITE_X * sum(w.values())
        res = {"kernels": sorted(f), "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
               "traffic_bytes_per_launch": fetch + write,
               "correction": "FETCH_SIZE x2, WRITE_SIZE x1 (profiles/r2/fetch_calib.json)",
               "source": [os.path.basename(fd.rstrip("/")), os.path.basename(wd.rstrip("/"))],
               "note": note}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
