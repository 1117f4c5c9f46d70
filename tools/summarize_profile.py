#!/usr/bin/env python3
"""Summarise tools/profile_round.sh output into profiles/<round>/ and
profiles/pmc_traffic.json (per-launch HBM bytes for bench.py's roofline).
Usage: python tools/summarize_profile.py r01"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path):
    agg = defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "msw::" in r["Kernel_Name"]:
                agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{rnd}")
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    for f in glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(dst, "kernel_stats_bench.csv"))
    c = {}
    for part in ("fetch", "write", "occ", "inst"):
        c.update(counters(os.path.join(src, part)))
    kernels = sorted({k for k, _ in c})
    summary = {}
    traffic = {}
    for k in kernels:
        d = {cn: v for (kn, cn), v in c.items() if kn == k}
        summary[k] = d
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            fetch_b = d["FETCH_SIZE"] * 1024
            write_b = d["WRITE_SIZE"] * 1024
            traffic_entry = {
                "fetch_bytes_raw": fetch_b, "write_bytes": write_b,
                "hbm_bytes_per_launch": fetch_b * 2 + write_b,
                "note": "FETCH_SIZE x 2 (gfx950 reports half of wide 16 B/lane reads, "
                        "MI355X_MICROARCH.md HBM section) + WRITE_SIZE; per launch; batch is "
                        "re-read every step and may be served from the 256 MiB Infinity Cache",
            }
            kind = "sw_kernel" if "sw_kernel" in k else ("sw_mixed_kernel" if "mixed" in k else k)
            traffic[k] = traffic_entry
            # tools/profile_round.sh profiles the default bench workload
            traffic.setdefault("config2:linear", traffic_entry)
        if "GRBM_GUI_ACTIVE" in d:
            summary[k]["note_clock"] = "effective clock = GRBM_GUI_ACTIVE / 8 / kernel time"
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
