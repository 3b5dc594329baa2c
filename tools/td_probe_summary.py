#!/usr/bin/env python3
"""Summary of tools/td_probe.sh: per case the probe's timing and, from its PMC
pass (launches 2-4, the timed ones), TA / TD busy per CU and TD cycles per load
instruction.   tools/td_probe_summary.py <outdir>"""
import csv
import glob
import json
import os
import sys

CUS = 256


def main(d):
    res = {}
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        name = os.path.basename(f)[:-5]
        if name == "summary":
            continue
        case = json.loads(open(f).read().strip().splitlines()[-1])
        per = {}
        for c in glob.glob(os.path.join(d, "pmc_" + name, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(c)):
                per.setdefault(int(row["Dispatch_Id"]), {})[row["Counter_Name"]] = float(row["Counter_Value"])
        disp = [per[k] for k in sorted(per)][1:]  # the first launch is the untimed warm-up
        if disp:
            avg = {k: sum(x.get(k, 0.0) for x in disp) / len(disp) for k in disp[0]}
            xcd_cycles = avg.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
            loads = avg.get("TA_FLAT_READ_WAVEFRONTS_sum", 0.0)
            case["ta_busy"] = round(avg.get("TA_TA_BUSY_sum", 0.0) / CUS / xcd_cycles, 3) if xcd_cycles else None
            case["td_busy"] = round(avg.get("TD_TD_BUSY_sum", 0.0) / CUS / xcd_cycles, 3) if xcd_cycles else None
            case["td_cycles_per_load"] = round(avg.get("TD_TD_BUSY_sum", 0.0) / loads, 2) if loads else None
            case["ta_cycles_per_load"] = round(avg.get("TA_TA_BUSY_sum", 0.0) / loads, 2) if loads else None
        res[name] = case
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
