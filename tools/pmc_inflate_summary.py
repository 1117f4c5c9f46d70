#!/usr/bin/env python3
"""Per-launch SQ counters of gz_inflate_kernel from tools/inflate_pmc.sh's
passes: every counter summed over the kernel's dispatches and divided by the
dispatch count, plus the ratios that say what bounds the waves (the SQ
cycle counters are in quad-cycles; WAIT_ANY + WAIT_INST_ANY +
ACTIVE_INST_ANY ~ WAVE_CYCLES).
  python3 tools/pmc_inflate_summary.py gpurun_out/TAG/inflate_pmc"""
import csv
import glob
import json
import os
import sys


def main():
    root = sys.argv[1]
    per = {}
    disp = {}
    for f in sorted(glob.glob(os.path.join(root, "pass*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if "gz_inflate" not in r["Kernel_Name"]:
                continue
            per[r["Counter_Name"]] = per.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            disp.setdefault(r["Counter_Name"], set()).add((f, r["Dispatch_Id"]))
    out = {"per_launch": {k: per[k] / max(1, len(disp[k])) for k in sorted(per)},
           "dispatches": {k: len(v) for k, v in sorted(disp.items())}}
    p = out["per_launch"]
    wc = p.get("SQ_WAVE_CYCLES")
    if wc:
        out["share_of_wave_cycles"] = {k: round(p[k] / wc, 4) for k in
                                       ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                        "SQ_ACTIVE_INST_SALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS") if k in p}
    if p.get("SQ_INSTS_VALU") and p.get("SQ_WAVES"):
        out["insts_per_wave"] = {k: round(p[k] / p["SQ_WAVES"], 1) for k in p if k.startswith("SQ_INSTS_")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
