#!/usr/bin/env python3
"""Summarise tools/traffic_split.sh: per-launch HBM reads of the config-2 and
config-5 scoring kernels split by buffer (windows, reads, the rest = lengths /
slot order / results), from the FETCH_SIZE of the in-tree build and of the
probe builds whose window (nowin) or read (noread) loads are constants.
  python3 tools/traffic_split.py gpurun_out/TAG/traffic OUT.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# algorithmic bytes per launch by buffer (bench.py workloads)
ALG = {"c2": {"kernel": "sw_kernel", "pairs": 10000, "reads": 10000 * 150.0, "windows": 10000 * 300.0,
              "padded_reads": 10000 * 160, "padded_windows": 10000 * 304},
       "c5": {"kernel": "sw_multi_kernel", "pairs": 100000}}


def counters(d, part):
    agg = defaultdict(list)
    for f in glob.glob(os.path.join(d, part, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    src, out = sys.argv[1], sys.argv[2]
    res = {}
    for cfg, meta in ALG.items():
        row = {}
        for v in ("base", "nowin", "noread"):
            c = counters(os.path.join(src, f"{cfg}_{v}"), "fetch")
            k = [(kn, cn) for (kn, cn) in c if meta["kernel"] in kn and cn == "FETCH_SIZE"]
            row[v] = c[k[0]] * 1024 if k else None
        w = counters(os.path.join(src, f"{cfg}_base"), "write")
        wk = [key for key in w if meta["kernel"] in key[0]]
        q = counters(os.path.join(src, f"{cfg}_base"), "req")
        qk = {cn: val for (kn, cn), val in q.items() if meta["kernel"] in kn}
        base, nowin, noread = row["base"], row["nowin"], row["noread"]
        win_raw, read_raw = base - nowin, base - noread
        rest_raw = base - win_raw - read_raw
        res[cfg] = {
            "fetch_raw_bytes": {"base": base, "nowin": nowin, "noread": noread},
            "write_bytes": w[wk[0]] * 1024 if wk else None,
            "rdreq_64b": qk.get("TCC_EA0_RDREQ_sum"), "rdreq_32b": qk.get("TCC_EA0_RDREQ_32B_sum"),
            "split_bytes_x2": {"windows": 2 * win_raw, "reads": 2 * read_raw, "rest": 2 * rest_raw,
                               "total": 2 * base},
            "note": "FETCH_SIZE x 2 (MI355X_MICROARCH.md: gfx950 counts half of 16 B/lane reads; the byte "
                    "pattern of the read loads counts 1.04x of that, profiles/r02/traffic/fetch_calib.json); "
                    "windows = base - nowin, reads = base - noread, rest = base - windows - reads",
        }
        for k in ("reads", "windows", "padded_reads", "padded_windows"):
            if k in meta:
                res[cfg].setdefault("reference_bytes", {})[k] = meta[k]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
