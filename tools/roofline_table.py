"""Print the roofline table of a bench line together with the committed
rocprofv3 evidence it rests on: per entry the bench time, the bytes the
kernel's own format moves, the fraction of 8 TB/s, the counter traffic
(2 x FETCH_SIZE + WRITE_SIZE per launch, profiles/<round>/*_traffic.json) and
traffic / own bytes, and the rocprofv3 average of the entry's kernels
(profiles/<round>/*_kernel_stats.csv).

    python tools/roofline_table.py [profiles/r3/bench_line.json]
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
line = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r3", "bench_line.json")
d = json.load(open(line))
prof = os.path.dirname(line)
PEAK = 8000.0  # GB/s


def stats_us(name, pattern):
    """rocprofv3 average (us) of the kernels whose name contains `pattern`."""
    f = os.path.join(prof, f"{name}_kernel_stats.csv")
    if not os.path.exists(f):
        return None
    rows = [r for r in csv.DictReader(open(f)) if pattern in r["Name"]]
    return round(sum(float(r["AverageNs"]) for r in rows) / 1e3, 1) if rows else None


def row(label, ms, own, traffic, stats):
    frac = own / (ms * 1e-3) / 1e9 / PEAK if own else None
    tr = f"{traffic / 1e9:.3f} GB ({traffic / own:.2f}x)" if traffic and own else "-"
    print(f"{label:44s} {ms:8.4f} ms  own {own / 1e9:6.3f} GB  frac {frac:5.3f}  traffic {tr:22s}  "
          f"rocprof {stats if stats is not None else '-'} us")


r = d["roofline"]
print(f"headline: {d['value']:.0f} {d['unit']}  ({d['config']['workload'][:60]}...)")
row("N28 stored real k_spmv_pk (roofline)", r["ms_per_launch"], r["bytes_per_launch"], r["traffic"],
    stats_us("spmv_n28", "k_spmv_pk<false"))
c = r["complex"]
row("N28 stored complex k_spmv_pk", c["ms_per_launch"], c["bytes_per_launch"], c.get("traffic"),
    stats_us("spmv_cplx_n28", "k_spmv_pk<true"))
k = d["kron_n28"]
row("N28 two-pass Kronecker (40*dim floor)", k["ms_per_hxv"], k["two_pass_bytes"], k.get("traffic"),
    stats_us("kron_n28", "k_kron"))
g = k["direct_generic"]
row("N28 generic matrix-free k_direct (24*dim)", g["ms_per_hxv"], g["own_bytes"], g.get("traffic"),
    stats_us("direct_n28", "k_direct"))
for name in ("n28j", "n26s"):
    s = r["sweep"][name]
    row(f"{name} stored real", s["stored"]["ms_per_launch"], s["stored"]["bytes_per_launch"],
        s["stored"].get("traffic"), stats_us(f"spmv_{name}", "k_spmv_pk<false"))
    gd = s["direct_generic"]
    row(f"{name} k_direct (24*dim)", gd["ms_per_hxv"], gd.get("own_bytes", 24 * s["stored"]["dim"]),
        gd.get("traffic"), stats_us(f"direct_{name}", "k_direct"))
print(f"farm_c4 {d['farm_c4']['wall_s']} s, nonsu2_c5 diag {d['nonsu2_c5']['diag_s']} s + gf "
      f"{d['nonsu2_c5']['gf_s']} s, complex(8) vectors {d['complex_iters_per_s']:.0f} it/s, "
      f"cpu_baseline {d['cpu_baseline']['value']:.0f} it/s")
