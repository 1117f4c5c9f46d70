#!/usr/bin/env python3
"""The headline's timed launches in a rocprofv3 kernel trace of
`bench.py` (default command): sw_kernel<13,f,f,f> dispatches in time order
on the bench's first stream are warm-up + preheat + the K timed steps; the
pipelined figure's launches follow on two streams.  Prints per-launch
durations of the K timed launches and their mean, to compare with the
line's roofline.avg_launch_ms (HIP events in bench.py).

  python3 tools/timed_launches.py TRACE_DIR BENCH_JSON
(TRACE_DIR holds the csv output, `--output-format csv`, or rocprofv3's
default rocpd sqlite database, `*_results.db`.)
"""
import csv
import glob
import json
import sqlite3
import sys

import numpy as np

KERNEL = "void msw::sw_kernel<13, false, false, false, false>(msw::SwParams)"


def dispatches(tdir):
    """(start ns, end ns, queue, stream) of every KERNEL dispatch."""
    rows = []
    for f in glob.glob(f"{tdir}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"] == KERNEL:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Stream_Id"]))
    for f in glob.glob(f"{tdir}/**/*_results.db", recursive=True):
        c = sqlite3.connect(f)
        rows += [(int(a), int(b), str(q), str(s)) for a, b, q, s in
                 c.execute("select start, end, queue_id, stream_id from kernels where name = ?", (KERNEL,))]
    return rows


def kernel_stats(tdir):
    """Per-kernel calls / total / average ns from a rocpd database (the
    --stats table rocprofv3 writes only with csv output)."""
    out = []
    for f in glob.glob(f"{tdir}/**/*_results.db", recursive=True):
        c = sqlite3.connect(f)
        out += list(c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                              "from kernels group by name order by sum(duration) desc"))
    return out


def main():
    tdir, bj = sys.argv[1], sys.argv[2]
    d = json.loads([ln for ln in open(bj) if ln.startswith("{")][0])
    if len(sys.argv) > 3:  # write the per-kernel summary as csv
        with open(sys.argv[3], "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"])
            for r in kernel_stats(tdir):
                w.writerow([r[0], r[1], r[2], round(r[3], 1), r[4], r[5]])
    K = d["steps"]
    rows = sorted(dispatches(tdir))
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
           "bench_avg_launch_ms": d["roofline"]["avg_launch_ms"] if "roofline" in d else d["summary"]["c2"].get(
               "avg_launch_ms"), "bench_ms_per_step": d["ms_per_step"],
           "all_calls_mean_us": round(float(np.mean([(e - s) / 1e3 for s, e, _, _ in rows])), 2),
           "all_calls": len(rows)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
