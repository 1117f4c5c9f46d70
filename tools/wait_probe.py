#!/usr/bin/env python3
"""Host cost of waiting on an already finished 10k-pair host-to-host call
(the host-to-host stream's wait half): submit one msw_align_reads_async
batch, let the GPU finish (msw_synchronize-free: a sleep), then time
Pending.wait() and, separately, the bare msw_wait ctypes call.  Median of
--reps; one JSON line.   python3 tools/wait_probe.py [--reps 200]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--pairs", type=int, default=10_000)
    a = ap.parse_args()
    from mini_parallel_amd import Context, Scoring
    from mini_parallel_amd._lib import lib
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
    ctx.align_reads(genome, *arrs, scoring=sc)
    py, raw, sub = [], [], []
    L = lib()
    for k in range(a.reps):
        t0 = time.perf_counter()
        p = ctx.align_reads(genome, *arrs, scoring=sc, asynchronous=True)
        sub.append(time.perf_counter() - t0)
        time.sleep(0.002)  # the batch has finished
        if k % 2:
            t0 = time.perf_counter()
            p.wait()
            py.append(time.perf_counter() - t0)
        else:
            t0 = time.perf_counter()
            L.msw_wait(ctx.handle, p.ticket)
            raw.append(time.perf_counter() - t0)
            p.wait()
    med = lambda v: round(float(np.median(v)) * 1e6, 1)
    print(json.dumps({"pairs": a.pairs, "submit_us": med(sub), "wait_python_us": med(py), "msw_wait_us": med(raw)}),
          flush=True)
    genome.close()
    ctx.close()


if __name__ == "__main__":
    main()
