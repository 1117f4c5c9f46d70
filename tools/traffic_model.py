#!/usr/bin/env python3
"""Bytes of HBM lines the scoring kernels must touch, by buffer, for the bench
workloads of configs 2 and 5 (the layouts of mini_parallel_amd.synthetic:
one padded row per pair), at line granularities of 16..128 bytes -- the
model the measured split (tools/traffic_split.py) is compared against in
DESIGN.md 4.3.  Rows are loaded in 16-byte chunks up to round16(length).
  python3 tools/traffic_model.py > profiles/r03/traffic/line_model.txt"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mini_parallel_amd.synthetic import config_batch  # noqa: E402


def touched(stride, lens, g):
    """Bytes of the distinct g-byte lines covering row i's [0, round16(len_i))."""
    L = (lens + 15) // 16 * 16
    st = np.arange(len(lens), dtype=np.int64) * stride
    keep = L > 0
    a, e = st[keep] // g, (st[keep] + L[keep] - 1) // g
    # rows may share a line when the stride is not a multiple of g: merge
    tot, cur_a, cur_e = 0, None, None
    for x, y in zip(a, e):
        if cur_e is None or x > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_a + 1
            cur_a, cur_e = x, y
        else:
            cur_e = max(cur_e, y)
    if cur_e is not None:
        tot += cur_e - cur_a + 1
    return tot * g


def main():
    for k in (2, 5):
        b = config_batch(k)
        m = b.read_len.astype(np.int64)
        n = b.win_len.astype(np.int64)
        rs, ws = b.reads.shape[1], b.wins.shape[1]
        print(f"config {k}: B={len(m)} rs={rs} ws={ws} alg reads {m.sum() / 1e6:.2f} MB windows {n.sum() / 1e6:.2f} MB")
        for g in (16, 32, 64, 128):
            print(f"  g={g:3d}: reads {touched(rs, m, g) / 1e6:.2f} MB, windows {touched(ws, n, g) / 1e6:.2f} MB")
    # config 5 before the per-pair clamp: every window loaded to its length
    # bucket's longest (KR = ceil(m / 16) buckets)
    b = config_batch(5)
    m = b.read_len.astype(np.int64)
    n = b.win_len.astype(np.int64)
    kr = (m + 15) // 16
    nmax = np.zeros_like(n)
    for k in np.unique(kr):
        nmax[kr == k] = n[kr == k].max()
    for g in (64, 128):
        print(f"windows loaded to the bucket max, g={g}: {touched(b.wins.shape[1], nmax, g) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
