#!/usr/bin/env python3
"""GPU time of a rocprofv3 kernel trace (CSV) split by kernel family: each
family's summed kernel time, its own busy union, and the union of all
kernels against the trace's span (and the run record's wall, if given).
Kernels of different families co-run on the CUs, so summed times exceed the
union; the union's idle share is what no family fills.
  python3 tools/trace_split.py gpurun_out/X/t_kernel_trace.csv [--record rec.json]"""
import argparse
import csv
import json

FAMILIES = [("inflate", ("gz_inflate",)), ("crc", ("gz_crc",)), ("score", ("sw_kernel", "sw_multi", "sw_long")),
            ("parse", ("k_count", "k_scan", "k_line", "k_lens", "k_fin", "k_emit", "parse")),
            ("cut_windows", ("cut_windows",)), ("copy", ("copy", "Copy", "pull_copy", "d2h")),
            ("fill", ("fill", "Fill"))]


def family(name):
    for fam, keys in FAMILIES:
        if any(k in name for k in keys):
            return fam
    return "other"


def union(iv):
    iv = sorted(iv)
    if not iv:
        return 0
    tot, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + ce - cs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--record", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    by = {}
    allv = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        f = family(r["Kernel_Name"])
        d = by.setdefault(f, {"n": 0, "sum_ns": 0, "iv": []})
        d["n"] += 1
        d["sum_ns"] += e - s
        d["iv"].append((s, e))
        allv.append((s, e))
    span = max(e for _, e in allv) - min(s for s, _ in allv)
    busy = union(allv)
    out = {"kernels": len(rows), "span_ms": round(span / 1e6, 2), "busy_union_ms": round(busy / 1e6, 2),
           "idle_ms": round((span - busy) / 1e6, 2),
           "families": {f: {"launches": d["n"], "sum_ms": round(d["sum_ns"] / 1e6, 2),
                            "union_ms": round(union(d["iv"]) / 1e6, 2)}
                        for f, d in sorted(by.items(), key=lambda kv: -kv[1]["sum_ns"])}}
    if a.record:
        rec = json.load(open(a.record))
        out["record"] = {k: rec.get(k) for k in ("wall_ms", "setup_ms", "kernel_ms", "reads_per_second",
                                                 "total_reads", "inflate_bytes_out")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
