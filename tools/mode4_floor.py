"""Per-step cycle breakdown of the complex(8) MODE 4 Lanczos step from the
counter passes of tools/mode4_pmc.sh (medians per 512-step dispatch of
k_lanc_persist, one 512-thread workgroup = 8 waves on one CU, 2 per SIMD).

    python tools/mode4_floor.py gpurun_out/r6m4 [out.json]
    python tools/mode4_floor.py profiles/r6        (the committed mode4_cplx_pmc_p*.json)

Units: SQ_BUSY_CYCLES and the SQ_LDS_* counters are CU cycles; SQ_WAVE_CYCLES,
SQ_WAIT_* and SQ_ACTIVE_INST_* are summed over waves in quad-cycles (x4).  A
wave64 VALU instruction (f64 or not) issues in 4 cycles on its SIMD.
"""
import json
import os
import sys

d = sys.argv[1]
ctr = {}
for p in ("p1", "p2", "p3"):
    f = os.path.join(d, p + ".json")
    doc = json.load(open(f if os.path.exists(f) else os.path.join(d, f"mode4_cplx_pmc_{p}.json")))
    rows = doc if isinstance(doc, list) else [r for v in doc.values() for r in v]
    for r in rows:
        if "k_lanc_persist" in r["kernel"]:
            ctr[r["counter"]] = r["median"]
            kern = r["kernel"]
steps, waves, simd_waves = 512, int(ctr["SQ_WAVES"]), int(ctr["SQ_WAVES"]) // 4
per_step = lambda c: ctr[c] / steps  # noqa: E731
per_wave_q = lambda c: ctr[c] * 4 / (steps * waves)  # noqa: E731  quad-cycles -> cycles, per wave
busy = per_step("SQ_BUSY_CYCLES")
lds = per_step("SQ_LDS_IDX_ACTIVE")
conf = per_step("SQ_LDS_BANK_CONFLICT")
valu_i = ctr["SQ_INSTS_VALU"] / (steps * waves)
f64_i = (ctr["SQ_INSTS_VALU_FMA_F64"] + ctr["SQ_INSTS_VALU_MUL_F64"] + ctr["SQ_INSTS_VALU_ADD_F64"]) / (steps * waves)
lds_i = ctr["SQ_INSTS_LDS"] / (steps * waves)
valu_simd = valu_i * 4 * simd_waves
clk = 2.4e9
floor = max(lds, valu_simd)
out = {
    "kernel": kern[:90], "steps_per_dispatch": steps, "waves": waves,
    "cu_cycles_per_step": round(busy), "us_per_step_at_2.4GHz": round(busy / clk * 1e6, 3),
    "lds_array_cycles_per_step": round(lds), "lds_bank_conflict_cycles_per_step": round(conf),
    "lds_array_busy_frac": round(lds / busy, 3),
    "lds_insts_per_wave_step": round(lds_i, 1), "valu_insts_per_wave_step": round(valu_i, 1),
    "f64_valu_insts_per_wave_step": round(f64_i, 1),
    "valu_issue_cycles_per_simd_step": round(valu_simd), "valu_busy_frac": round(valu_simd / busy, 3),
    "wave_wait_cycles_per_step": round(per_wave_q("SQ_WAIT_ANY")),
    "wave_wait_lds_issue_cycles_per_step": round(per_wave_q("SQ_WAIT_INST_LDS")),
    "floor_cycles": round(floor), "floor_us": round(floor / clk * 1e6, 3),
    "floor_iters_per_s": round(clk / floor),
    "floor_without_conflicts_cycles": round(max(lds - conf, valu_simd)),
    "floor_without_conflicts_iters_per_s": round(clk / max(lds - conf, valu_simd)),
    "measured_over_floor": round(busy / floor, 3),
    "target_300k_cycles": round(clk / 300e3),
}
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
