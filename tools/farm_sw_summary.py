"""Summarise tools/farm_sw.sh logs: per configuration the best rep of every
run and the median / mean of all reps after each run's first (warm-up)."""
import re
import statistics as st
import sys

cur, d = None, {}
for line in open(sys.argv[1]):
    m = re.match(r"== (.*)", line)
    if m:
        cur = m.group(1).strip()
        d.setdefault(cur, []).append([])
        continue
    m = re.search(r"wall ([\d.]+) s", line)
    if m and cur:
        d[cur][-1].append(float(m.group(1)))
for k, v in d.items():
    later = [x for run in v for x in run[1:]]
    print(f"{k:36s} best/run {[round(min(r[1:]), 3) for r in v if len(r) > 1]} "
          f"median {st.median(later):.4f} mean {st.mean(later):.4f}")
