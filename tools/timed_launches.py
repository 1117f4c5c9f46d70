#!/usr/bin/env python3
"""The headline's timed launches in a rocprofv3 kernel trace of
`bench.py` (default command): sw_kernel<13,f,f,f> dispatches in time order
on the bench's first stream are warm-up + preheat + the K timed steps; the
pipelined figure's launches follow on two streams.  Prints per-launch
durations of the K timed launches and their mean, to compare with the
line's roofline.avg_launch_ms (HIP events in bench.py).

  python3 tools/timed_launches.py TRACE_DIR BENCH_JSON
"""
import csv
import glob
import json
import sys

import numpy as np

KERNEL = "void msw::sw_kernel<13, false, false, false>(msw::SwParams)"


def main():
    tdir, bj = sys.argv[1], sys.argv[2]
    d = json.loads([ln for ln in open(bj) if ln.startswith("{")][0])
    K = d["steps"]
    rows = []
    for f in glob.glob(f"{tdir}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"] == KERNEL:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Stream_Id"]))
    rows.sort()
    first_stream = rows[0][3]
    serial = []
    for r in rows:
        if r[3] != first_stream:
            break
        serial.append(r)
    # runs of back-to-back launches (gaps under 50 us); the preheat syncs
    # every 20 launches, the fence precedes the timed run and the pipelined
    # figure's first launch follows it: the timed steps are the last run of
    # exactly K launches
    runs, cur = [], [serial[0]]
    for a, b in zip(serial, serial[1:]):
        if b[0] - a[1] > 50_000:
            runs.append(cur)
            cur = []
        cur.append(b)
    runs.append(cur)
    timed = [r for r in runs if len(r) == K][-1]
    dur = np.array([(e - s) / 1e3 for s, e, _, _ in timed])
    span = (timed[-1][1] - timed[0][0]) / 1e3
    out = {"kernel": KERNEL, "serial_launches_on_first_stream": len(serial), "timed_K": K,
           "timed_mean_us": round(float(dur.mean()), 2), "timed_min_us": round(float(dur.min()), 2),
           "timed_max_us": round(float(dur.max()), 2), "timed_span_us_per_step": round(span / K, 2),
           "bench_avg_launch_ms": d["roofline"]["avg_launch_ms"], "bench_ms_per_step": d["ms_per_step"],
           "all_calls_mean_us": round(float(np.mean([(e - s) / 1e3 for s, e, _, _ in rows])), 2),
           "all_calls": len(rows)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
