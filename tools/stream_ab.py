#!/usr/bin/env python3
"""The host-to-host stream of 10k-pair calls (bench.py's
pcie_inclusive.genome_pinned_stream: pinned reads + positions against an
HBM-resident genome, three in flight) under environment settings read per
call by the library, alternated --reps times after a preheat; every run's
last scores checked.  One JSON line per run.
  python3 tools/stream_ab.py --setting base= --setting other=VAR=VALUE"""
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
    ap.add_argument("--setting", action="append", required=True)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--batches", type=int, default=400)
    a = ap.parse_args()
    from mini_parallel_amd import Context, Scoring
    from mini_parallel_amd.aligner import pinned_empty
    from mini_parallel_amd.synthetic import config_shard
    b = config_shard(2, 0, 10_000)
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
    settings = []
    for s in a.setting:
        name, _, rest = s.partition("=")
        settings.append((name, dict(kv.split("=", 1) for kv in rest.split(",") if kv)))

    def run(n):
        pend, sub = [], 0.0
        t0 = time.perf_counter()
        for _ in range(n):
            t1 = time.perf_counter()
            pend.append(ctx.align_reads(genome, *arrs, scoring=sc, asynchronous=True))
            sub += time.perf_counter() - t1
            if len(pend) == 3:
                pend.pop(0).wait()
        last = None
        while pend:
            last = pend.pop(0).wait()[0]
        return (time.perf_counter() - t0) / n, sub / n, last
    for rep in range(a.reps):
        for name, env in settings:
            for k in list(os.environ):
                if k in ("MSW_COPY_STREAM", "MSW_ASYNC_ONE_STREAM"):
                    del os.environ[k]
            os.environ.update(env)
            run(a.batches // 2)  # preheat
            dt, sub, last = run(a.batches)
            print(json.dumps({"setting": name, "rep": rep, "us_per_batch": round(dt * 1e6, 1),
                              "gcups": round(b.cells / dt / 1e9, 1), "submit_us": round(sub * 1e6, 1),
                              "bit_exact": bool(np.array_equal(last, want))}), flush=True)
    genome.close()
    ctx.close()


if __name__ == "__main__":
    main()
