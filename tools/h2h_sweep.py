#!/usr/bin/env python3
"""Config-3 host-to-host rate vs chunk size (bench.py's configs_extra.config3
host_to_host leg, genome_pinned form): 1 M pairs of 150 x 300, affine + best
cell, reads + window positions in pinned host memory, the windows' genome
resident in HBM, chunked async H2D / kernels / readback through
msw_align_reads; best of 3 per chunk size, checked against one HBM-resident
run.  One JSON line per chunk size and round (`--reps`).
  python3 tools/h2h_sweep.py --chunks 32768,65536,131072,262144 > out.jsonl"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="32768,65536,131072,262144,524288")
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=1)
    args = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (binds the HIP runtime first)

    from mini_parallel_amd import AFFINE, Context
    from mini_parallel_amd.aligner import pinned_empty
    from mini_parallel_amd.synthetic import config_batch

    b = config_batch(3, n_pairs=args.pairs)
    ctx = Context(0)

    def pinned(a):
        p = pinned_empty(a.shape, a.dtype)
        p[...] = a
        return p
    ws = b.wins.shape[1]
    genome = ctx.load_genome(np.ascontiguousarray(b.wins).reshape(-1))
    reads, rl, wl = pinned(b.reads), pinned(b.read_len), pinned(b.win_len)
    pos = pinned(np.arange(b.n_pairs, dtype=np.int64) * ws)
    want = ctx.align_reads(genome, reads, rl, pos, wl, scoring=AFFINE, chunk_pairs=b.n_pairs)
    for rep in range(args.reps):
        for chunk in [int(x) for x in args.chunks.split(",")]:
            for _ in (0,):
                got = ctx.align_reads(genome, reads, rl, pos, wl, scoring=AFFINE, chunk_pairs=chunk)
                ok = all(np.array_equal(g, w) for g, w in zip(got, want))
                best = 1e30
                for _ in range(3):
                    ctx.synchronize()
                    t0 = time.perf_counter()
                    ctx.align_reads(genome, reads, rl, pos, wl, scoring=AFFINE, chunk_pairs=chunk)
                    best = min(best, time.perf_counter() - t0)
                print(json.dumps({"chunk_pairs": chunk, "rep": rep, "ms": round(best * 1e3, 3),
                                  "gcups": round(b.cells / best / 1e9, 1), "bit_exact": ok}), flush=True)
    genome.close()
    ctx.close()


if __name__ == "__main__":
    main()
