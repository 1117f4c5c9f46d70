#!/usr/bin/env python3
"""GPU lane reader alone (msw_gfastq_*: inflate, CRC, parse, emit) over one
BGZF FASTQ lane file: reads/s and inflated GB/s per pass, no scoring.  Run
it under `rocprofv3 --kernel-trace --stats` for the reader's kernels without
the scoring worker beside them.
  python tools/gfastq_bench.py --reads 2000000 --passes 3 [--with-pos]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--qual", default="binned")
    ap.add_argument("--level", type=int, default=6)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--with-pos", action="store_true")
    ap.add_argument("--dir", default="/tmp/msw_gfastq_bench")
    args = ap.parse_args()
    from mini_parallel_amd import Context
    from mini_parallel_amd._lib import check, lib
    from mini_parallel_amd.fastq import GpuFastqReader
    from mini_parallel_amd.synthetic import write_wgs_dataset
    t = time.perf_counter()
    ds = write_wgs_dataset(args.dir, lanes=1, reads_per_lane=1, reads_per_file=args.reads, keep_batches=False,
                           qual=args.qual, compresslevel=args.level, bgzf=True)
    path = ds["files"][0]
    print(f"dataset {os.path.getsize(path) / 1e6:.1f} MB gz in {time.perf_counter() - t:.1f} s", flush=True)
    ctx = Context(0)
    rd = GpuFastqReader(ctx, path, max_reads=args.batch, with_pos=args.with_pos)
    for p in range(args.passes):
        if p:
            check(lib().msw_gfastq_reset(rd._h, path.encode()))
        t = time.perf_counter()
        n = 0
        while True:
            d = rd.next_batch(host=False)
            if d.n == 0:
                break
            n += d.n
        check(lib().msw_synchronize(ctx.handle))
        dt = time.perf_counter() - t
        s = rd.stats()
        print(f"pass {p}: {n} reads in {dt * 1e3:.1f} ms: {n / dt / 1e6:.1f} M reads/s, "
              f"{s['bytes_out'] / dt / 1e9:.1f} GB/s inflated ({s['bytes_in'] / 1e6:.0f} MB in, "
              f"{s['bytes_out'] / 1e6:.0f} MB out)", flush=True)
    rd.close()
    ctx.close()


if __name__ == "__main__":
    main()
