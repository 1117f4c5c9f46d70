#!/usr/bin/env python3
"""Summarise tools/profile_round.sh output into profiles/<round>/ and
profiles/pmc_traffic.json (per-launch HBM bytes for bench.py's roofline,
keyed "config<k>:<kind>" as bench.py looks them up).
Usage: python tools/summarize_profile.py r01 [--only 3]
(--only: refresh those configs' entries and keep the others, e.g. config 2's
hand-split non-sequence fetch)"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KIND = {2: "linear", 3: "affine_coords", 5: "linear"}  # bench.py scoring per config


def counters(path):
    agg = defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "msw::" in r["Kernel_Name"]:
                agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    only = {int(x) for x in sys.argv[sys.argv.index("--only") + 1].split(",")} if "--only" in sys.argv else None
    src = os.path.join(ROOT, "gpurun_out", f"prof_{rnd}")
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    summary, traffic = {}, {}
    # the commit whose build was profiled: gpurun_out/prof_<round>/COMMIT (written by
    # tools/profile_round.sh from the tree it ran), else this checkout's HEAD
    try:
        commit = open(os.path.join(src, "COMMIT")).read().strip()
    except OSError:
        import subprocess
        commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                text=True).stdout.strip()
    for cfg in (2, 3, 5):
        if only and cfg not in only:
            continue
        d = os.path.join(src, f"c{cfg}")
        if not os.path.isdir(d):
            continue
        for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
            shutil.copy(f, os.path.join(dst, f"kernel_stats_config{cfg}.csv"))
        c = {}
        for part in ("fetch", "write", "occ", "inst"):
            c.update(counters(os.path.join(d, part)))
        per_kernel = {}
        for k in sorted({k for k, _ in c}):
            per_kernel[k] = {cn: v for (kn, cn), v in c.items() if kn == k}
        summary[f"config{cfg}"] = per_kernel
        # the dominant (scoring) kernel of the config: the one fetching most
        main_k = sorted((k for k in per_kernel if "FETCH_SIZE" in per_kernel[k] and "WRITE_SIZE" in per_kernel[k]),
                        key=lambda k: -per_kernel[k]["FETCH_SIZE"])[:1]
        for k in main_k:
            m = per_kernel[k]
            if True:
                fetch_b, write_b = m["FETCH_SIZE"] * 1024, m["WRITE_SIZE"] * 1024
                traffic[f"config{cfg}:{KIND[cfg]}"] = {
                    "kernel": k, "fetch_bytes_raw": fetch_b, "write_bytes": write_b,
                    "hbm_bytes_per_launch": fetch_b * 2 + write_b, "round": rnd, "commit": commit,
                    "note": "FETCH_SIZE x 2 (gfx950 reports half of wide 16 B/lane reads, "
                            "MI355X_MICROARCH.md HBM section) + WRITE_SIZE; per launch; the batch is "
                            "re-read every step and may be served from the 256 MiB Infinity Cache"}
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if only:  # merge: the other configs' entries stay as they are
        old = json.load(open(tpath)) if os.path.exists(tpath) else {}
        old.update(traffic)
        traffic = old
    with open(os.path.join(dst, "pmc_summary.json" if not only else "pmc_summary_only.json"), "w") as f:
        json.dump(summary, f, indent=1)
    with open(tpath, "w") as f:
        json.dump(traffic, f, indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
