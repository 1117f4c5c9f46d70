#!/usr/bin/env python3
"""Kernel time of one batch shape (device-resident, HIP events on the launch
stream), for A/B of kernel variants (MSW_LIB_PATH) and for best-case proxies
of layouts the kernel does not implement: e.g. a row split of
10k 150 bp pairs over two waves is bounded below by 20k pairs of 75 bp reads
run as ordinary waves (no hand-off, no lag).  Prints one JSON line.

Usage: python tools/lever_probe.py --read-len 150 --win-len 300 --pairs 10000
       [--group-lanes G] [--layout pairs|split|mixed] [--affine] [--coords]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--win-len", type=int, default=300)
    ap.add_argument("--pairs", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--group-lanes", type=int, default=0)
    ap.add_argument("--layout", default="")
    ap.add_argument("--affine", action="store_true")
    ap.add_argument("--coords", action="store_true")
    ap.add_argument("--label", default="")
    ap.add_argument("--check", type=int, default=512, help="pairs checked against the oracle (0 = none)")
    args = ap.parse_args()
    if args.layout:
        os.environ["MSW_LAYOUT"] = args.layout
    if args.group_lanes:
        os.environ["MSW_GROUP_LANES"] = str(args.group_lanes)

    import numpy as np
    import torch
    from mini_parallel_amd import Context, Scoring
    from mini_parallel_amd.synthetic import make_pairs

    r16 = lambda v: max(16, (v + 15) // 16 * 16)  # noqa: E731
    b = make_pairs(args.pairs, args.read_len, args.win_len / args.read_len, seed=77,
                   read_stride=r16(args.read_len + 2), win_stride=r16(args.win_len))
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    reads, wins = t(b.reads), t(b.wins)
    rl, wl = t(b.read_len.view(np.int16)), t(b.win_len.view(np.int16))
    score = torch.zeros(b.n_pairs, dtype=torch.int32, device=dev)
    ei = torch.zeros(b.n_pairs, dtype=torch.int16, device=dev)
    ej = torch.zeros(b.n_pairs, dtype=torch.int16, device=dev)
    sc = Scoring(gap_open=3 if args.affine else 0, gap_extend=1 if args.affine else 2, affine=args.affine,
                 want_coords=args.coords)
    ctx = Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    step = ctx.prepare_device_launch(reads.data_ptr(), rl.data_ptr(), wins.data_ptr(), wl.data_ptr(),
                                     b.reads.shape[1], b.wins.shape[1], b.n_pairs, score.data_ptr(),
                                     int(b.read_len.max()), int(b.win_len.max()), sc, ei.data_ptr(), ej.data_ptr(),
                                     stream.cuda_stream)
    for _ in range(5):
        step()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.reps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / args.reps
    out = {"label": args.label, "read_len": args.read_len, "win_len": args.win_len, "pairs": args.pairs,
           "group_lanes": args.group_lanes or "auto", "layout": args.layout or "auto",
           "kind": ("affine" if args.affine else "linear") + ("+coords" if args.coords else ""),
           "avg_us": round(us, 2), "gcups": round(b.cells / (us * 1e-6) / 1e9, 1),
           "lib": os.path.basename(os.environ.get("MSW_LIB_PATH", "libmsw.so"))}
    if args.check:
        from oracle import oracle_lib
        n = min(args.check, b.n_pairs)
        s, i, j = oracle_lib.sw_batch(b.reads[:n], b.read_len[:n], b.wins[:n], b.win_len[:n], match=2, mismatch=-1,
                                      gap_open=sc.gap_open, gap_extend=sc.gap_extend, affine=sc.affine, threads=8)
        g = score.cpu().numpy()[:n]
        bad = int((g != s).sum())
        if args.coords:
            bad += int(((ei.cpu().numpy()[:n] != i) | (ej.cpu().numpy()[:n] != j)).sum())
        out["checked"], out["mismatches"] = n, bad
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
