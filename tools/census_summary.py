#!/usr/bin/env python3
"""Per-phase VALU of the Cornell kernel from tools/census.sh: build k runs
phase k twice (RT_CENSUS, rt_kernel.hip), so its SQ_INSTS_VALU minus the
plain build's is phase k's dynamic VALU (wave instructions).  Reported per
launch and as lane-slot VALU per sample (x 64 / samples).

    tools/census_summary.py <census_dir>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

PHASES = {"cz1": "camera ray (Halton dims 0-1 + generateCameraRay)",
          "cz2": "closest-hit queries (box clusters + candidate pair tests)",
          "cz3": "shadow any-hit queries",
          "cz4": "Halton dims 2-5 of the bounces",
          "cz5": "shading arithmetic (light sample, NEE term, cosine direction)",
          "cz6": "in-order pixel sums (DPP row shifts)"}
SAMPLES = 1920 * 1080 * 256


def counters(d):
    acc = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                if "path_trace" in r.get("Kernel_Name", ""):
                    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    d = sys.argv[1]
    base = counters(os.path.join(d, "base"))
    out = {"samples_per_launch": SAMPLES, "base": base,
           "base_lane_valu_per_sample": 64 * base["SQ_INSTS_VALU"] / SAMPLES, "phases": {}}
    total = 0.0
    for k, name in PHASES.items():
        c = counters(os.path.join(d, k))
        if not c:
            continue
        dv = {n: c[n] - base[n] for n in base}
        per = 64 * dv["SQ_INSTS_VALU"] / SAMPLES
        total += per
        other = dv["SQ_INSTS_VALU"] - sum(dv.get(n, 0.0) for n in (
            "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_ADD_F32",
            "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_CVT"))
        out["phases"][k] = {"phase": name, "valu_wave_insts_per_launch": dv["SQ_INSTS_VALU"],
                            "lane_valu_per_sample": per,
                            "share_of_base": dv["SQ_INSTS_VALU"] / base["SQ_INSTS_VALU"],
                            "cmp_sel_minmax_mov_share": other / dv["SQ_INSTS_VALU"] if dv["SQ_INSTS_VALU"] else None,
                            "salu_per_launch": dv["SQ_INSTS_SALU"], "mix": dv}
    out["phases_total_lane_valu_per_sample"] = total
    out["rest_lane_valu_per_sample"] = out["base_lane_valu_per_sample"] - total
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
