#!/usr/bin/env python3
"""Where the host-to-host streaming rate of config 2 goes (bench.py's
pcie_inclusive.genome_pinned_stream): 10k-pair batches (150 x 300) submitted
asynchronously from pinned arrays against an HBM-resident genome, DEPTH in
flight.  Prints one JSON line per setting: ms per batch, host time inside the
submission call (Python + C), inside the wait, and, with --trace, the C
side's split (MSW_HOST_TRACE: scan / stage / submit / wait per call).

  python3 tools/stream_probe.py [--trace] [--batches 400] [--pairs 10000]
"""
import argparse
import json
import os
import re
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", action="store_true")
    ap.add_argument("--batches", type=int, default=400)
    ap.add_argument("--pairs", type=int, default=10_000)
    ap.add_argument("--depths", default="1,2,3,3", help="batches in flight, one pass per entry")
    a = ap.parse_args()
    err_fd = None
    if a.trace:
        os.environ["MSW_HOST_TRACE"] = "1"
        tmp = tempfile.TemporaryFile(mode="w+")
        err_fd = os.dup(2)
        os.dup2(tmp.fileno(), 2)
    from mini_parallel_amd import Context, Scoring
    from mini_parallel_amd.aligner import pinned_empty
    from mini_parallel_amd.synthetic import config_shard
    b = config_shard(2, 0, a.pairs)
    ctx = Context(0)
    ws = b.wins.shape[1]
    genome = ctx.load_genome(np.ascontiguousarray(b.wins).reshape(-1))

    def pinned(x):
        p = pinned_empty(x.shape, x.dtype)
        p[...] = x
        return p
    arrs = tuple(pinned(x) for x in (b.reads, b.read_len, np.arange(b.n_pairs, dtype=np.int64) * ws, b.win_len))
    sc = Scoring()
    want = ctx.align_reads(genome, *arrs, scoring=sc)[0]
    rows = []
    for depth in [int(x) for x in a.depths.split(",")]:
        for timed in (False, True):
            n = a.batches if timed else max(50, a.batches // 4)
            pend, sub, wt = [], 0.0, 0.0
            t0 = time.perf_counter()
            for _ in range(n):
                t1 = time.perf_counter()
                pend.append(ctx.align_reads(genome, *arrs, scoring=sc, asynchronous=True))
                t2 = time.perf_counter()
                sub += t2 - t1
                if len(pend) == depth:
                    last = pend.pop(0).wait()[0]
                    wt += time.perf_counter() - t2
            while pend:
                last = pend.pop(0).wait()[0]
            dt = (time.perf_counter() - t0) / n
        assert np.array_equal(last, want)
        rows.append({"depth": depth, "batches": n, "ms_per_batch": round(dt * 1e3, 4),
                     "gcups": round(b.cells / dt / 1e9, 1), "submit_us": round(sub / n * 1e6, 1),
                     "wait_us": round(wt / n * 1e6, 1)})
    # the C call alone, no Python wrapper around it: a bound ctypes call
    genome.close()
    ctx.close()
    if a.trace:
        sys.stderr.flush()
        os.dup2(err_fd, 2)
        tmp.seek(0)
        tr = [tuple(float(x) for x in m) for m in
              re.findall(r"scan=([\d.]+)us stage=([\d.]+)us submit=([\d.]+)us wait=([\d.]+)us", tmp.read())]
        if tr:
            t = np.array(tr[-a.batches:])
            rows.append({"c_side_us_per_call_last_pass": dict(zip(("scan", "stage", "submit", "wait"),
                                                                  np.round(t.mean(0), 2).tolist())),
                         "calls": len(tr)})
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
