#!/usr/bin/env python3
"""GPU BGZF inflate throughput vs the number of members in one launch
(MSW_GZ_TIMING=1 prints the inflate / CRC kernel times of each launch).
  MSW_GZ_TIMING=1 python tools/inflate_bench.py --qual binned --level 6"""
import argparse
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qual", default="binned")
    ap.add_argument("--level", type=int, default=6)
    ap.add_argument("--members", default="1,16,256,1024,2534,8192")
    ap.add_argument("--strategy", default="default", choices=["default", "huffman_only", "rle", "fixed", "stored"])
    args = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401
    from mini_parallel_amd import Context
    from mini_parallel_amd.fastq import bgzf_inflate
    from mini_parallel_amd.synthetic import bgzf_compress, write_wgs_dataset
    ds = write_wgs_dataset("/tmp/msw_inflate_bench", lanes=1, reads_per_lane=1, reads_per_file=40_000,
                           keep_batches=False, qual=args.qual, compresslevel=1, bgzf=False)
    import gzip
    text = gzip.decompress(open(ds["files"][0], "rb").read())
    blk = 0xFF00
    one = [text[k:k + blk] for k in range(0, len(text) - blk, blk)]
    strat = {"default": 0, "huffman_only": zlib.Z_HUFFMAN_ONLY, "rle": zlib.Z_RLE, "fixed": zlib.Z_FIXED,
             "stored": 0}[args.strategy]
    level = 0 if args.strategy == "stored" else args.level
    members = [bgzf_compress(m, level, strat, eof_block=False) for m in one]
    ctx = Context(0)
    for n in [int(x) for x in args.members.split(",")]:
        blob = b"".join(members[k % len(members)] for k in range(n))
        want = b"".join(one[k % len(one)] for k in range(n))
        bgzf_inflate(ctx, blob)  # warm
        t = time.perf_counter()
        got = bgzf_inflate(ctx, blob)
        dt = time.perf_counter() - t
        assert got == want
        print(f"members {n}: {len(blob) / 1e6:.1f} MB in, {len(want) / 1e6:.1f} MB out, host-to-host {dt * 1e3:.1f} ms",
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
