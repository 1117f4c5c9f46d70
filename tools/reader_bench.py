#!/usr/bin/env python3
"""FASTQ reader throughput (C++ reader through ctypes) on one lane file, for
gzip / BGZF lane files and several MSW_INFLATE_THREADS values.
  python tools/reader_bench.py --reads 1000000 --threads 1,4,16"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(path, threads):
    os.environ["MSW_INFLATE_THREADS"] = str(threads)
    from mini_parallel_amd.fastq import FastqReader
    import numpy as np
    seqs = np.zeros((65536, 256), np.uint8)
    t = time.perf_counter()
    n = 0
    from mini_parallel_amd._lib import lib
    import ctypes
    lens = np.zeros(65536, np.uint16)
    pos = np.zeros(65536, np.int64)
    with FastqReader(path) as r:
        while True:
            k = ctypes.c_uint64(0)
            lib().msw_fastq_next(r._h, seqs.ctypes.data, lens.ctypes.data, 256, 65536, ctypes.byref(k),
                                 pos.ctypes.data)
            if k.value == 0:
                break
            n += k.value
    return n, time.perf_counter() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/tmp/msw_reader")
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--threads", default="1,4,16")
    ap.add_argument("--child", nargs=2)
    a = ap.parse_args()
    if a.child:
        n, dt = child(a.child[0], int(a.child[1]))
        print(json.dumps({"reads": n, "s": round(dt, 4)}))
        return
    from mini_parallel_amd.synthetic import write_wgs_dataset
    for bgzf in (False, True):
        d = os.path.join(a.dir, "bgzf" if bgzf else "gz")
        ds = write_wgs_dataset(d, lanes=1, reads_per_lane=1, reads_per_file=a.reads, genome_bases=1 << 24,
                               keep_batches=False, bgzf=bgzf)
        for t in [int(x) for x in a.threads.split(",")]:
            out = subprocess.run([sys.executable, __file__, "--child", ds["files"][0], str(t)], capture_output=True,
                                 text=True, check=True).stdout.strip().splitlines()[-1]
            r = json.loads(out)
            print(json.dumps({"bgzf": bgzf, "inflate_threads": t, "reads": r["reads"], "s": r["s"],
                              "M_reads_per_s": round(r["reads"] / r["s"] / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
