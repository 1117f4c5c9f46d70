"""Idle gaps of a rocprofv3 kernel trace (--kernel-trace CSV): GPU busy time
inside the region from the first inflate to the last scoring kernel, and the
gaps longer than --min-ms with the kernels on either side."""
import argparse
import csv


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").replace("msw::", "")
    return n.split("(")[0][:24]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--min-ms", type=float, default=1.0)
    a = ap.parse_args()
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Stream_Id"])
                for r in csv.DictReader(open(a.trace)))
    first = min(s for s, e, n, _ in ev if "inflate" in n)
    last = max(e for s, e, n, _ in ev if "sw_kernel" in n)
    ce, prev, busy, cs, gaps = None, None, 0, None, 0.0
    for s, e, n, st in ev:
        if s < first or s > last:
            continue
        if ce is not None and s > ce:
            busy += ce - cs
            gaps += (s - ce) / 1e6
            if s - ce > a.min_ms * 1e6:
                print(f"gap {(s - ce) / 1e6:5.2f} ms at t={(ce - first) / 1e6:7.2f}  after {prev[2]:24s}(st{prev[3]}) "
                      f"before {n:24s}(st{st})")
            cs = s
        if cs is None:
            cs = s
        if ce is None or e > ce:
            ce, prev = e, (s, e, n, st)
    busy += ce - cs
    print(f"region {(last - first) / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, idle {gaps:.2f} ms")


if __name__ == "__main__":
    main()
