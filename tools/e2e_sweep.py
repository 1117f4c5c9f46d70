#!/usr/bin/env python3
"""Host-to-host chunk-size sweep: the same batch through msw_align_reads
(genome-resident windows, pinned reads/positions) and msw_align_batch (pinned
pairs) with several chunk sizes; one JSON line per point.
  python tools/e2e_sweep.py --config 3 --chunks 65536,131072,262144"""
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
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=0)
    ap.add_argument("--chunks", default="32768,65536,131072,262144,524288")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch  # noqa: F401
    from mini_parallel_amd import Context, Scoring
    from mini_parallel_amd.aligner import pinned_empty
    from mini_parallel_amd.synthetic import config_batch
    sc = {2: Scoring(), 3: Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True), 5: Scoring()}[args.config]
    b = config_batch(args.config, n_pairs=args.pairs or {2: 10_000, 3: 1_000_000, 5: 100_000}[args.config])
    cells = b.cells
    ctx = Context(0)
    ws = b.wins.shape[1]
    g = ctx.load_genome(np.ascontiguousarray(b.wins).reshape(-1))

    def pin(a):
        p = pinned_empty(a.shape, a.dtype)
        p[...] = a
        return p
    pos = np.arange(b.n_pairs, dtype=np.int64) * ws
    rd = [pin(a) for a in (b.reads, b.read_len, pos, b.win_len)]
    pr = [pin(a) for a in (b.reads, b.read_len, b.wins, b.win_len)]
    ref = None
    for chunk in [int(c) for c in args.chunks.split(",")]:
        for name, fn in (("genome_pinned", lambda: ctx.align_reads(g, *rd, scoring=sc, chunk_pairs=chunk)),
                         ("pairs_pinned", lambda: ctx.align_batch(*pr, scoring=sc, chunk_pairs=chunk))):
            s, _, _ = fn()
            if ref is None:
                ref = s
            assert np.array_equal(s, ref)
            best = 1e9
            for _ in range(args.reps):
                t = time.perf_counter()
                fn()
                best = min(best, time.perf_counter() - t)
            print(json.dumps({"config": args.config, "variant": name, "chunk": chunk,
                              "ms": round(best * 1e3, 3), "gcups": round(cells / best / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
