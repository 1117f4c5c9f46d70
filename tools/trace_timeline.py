#!/usr/bin/env python3
"""Timeline summary of a rocprofv3 kernel trace (CSV): GPU-busy union, the
largest idle gaps, and the main kernels in start order.
  python tools/trace_timeline.py gpurun_out/X/prof/t_kernel_trace.csv [--from MS] [--to MS]"""
import argparse
import csv

KEYS = ["gz_inflate", "gz_crc", "sw_kernel", "k_emit", "k_line", "k_count", "k_scan", "k_lens", "k_fin",
        "cut_windows", "copyBuffer", "fillBuffer"]


def short(n):
    for k in KEYS:
        if k in n:
            return k
    return n[:24]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--from", dest="t_from", type=float, default=0.0)
    ap.add_argument("--to", type=float, default=1e12)
    ap.add_argument("--min-ms", type=float, default=0.5, help="list kernels at least this long")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    t0 = iv[0][0]
    iv = [(s, e, n) for s, e, n in iv if args.t_from <= (s - t0) / 1e6 <= args.to]
    busy, gaps = 0, []
    cs, ce = iv[0][0], iv[0][1]
    for s, e, _ in iv[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append((s - ce, ce - t0))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    span = max(e for _, e, _ in iv) - iv[0][0]
    print(f"span {span / 1e6:.1f} ms, GPU busy (union) {busy / 1e6:.1f} ms")
    print("largest gaps (ms @ ms):", [(round(g / 1e6, 2), round(a / 1e6, 1)) for g, a in sorted(gaps)[::-1][:10]])
    for s, e, n in iv:
        if (e - s) / 1e6 >= args.min_ms:
            print(f"{(s - t0) / 1e6:8.1f} {(e - s) / 1e6:7.2f} {n}")


if __name__ == "__main__":
    main()
