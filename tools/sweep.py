#!/usr/bin/env python3
"""Kernel-time sweep over batch sizes and lane layouts (one process, device
resident inputs, HIP events on the launch stream).  Prints one JSON line per
point.  Usage: python tools/sweep.py [--config 2] [--sizes 1024,2048,...]"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--sizes", default="1024,2048,4096,8192,10000,12288,16384,32768,65536")
    ap.add_argument("--layouts", default="pairs,split,mixed,auto")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--affine", action="store_true")
    ap.add_argument("--coords", action="store_true")
    ap.add_argument("--group-lanes", default="0", help="comma list of forced G (0 = runtime choice)")
    args = ap.parse_args()

    import numpy as np
    import torch
    from mini_parallel_amd import Context, Scoring
    from mini_parallel_amd.synthetic import config_batch

    sizes = [int(x) for x in args.sizes.split(",")]
    b = config_batch(args.config, n_pairs=max(sizes))
    dev = torch.device("cuda", 0)
    reads = torch.from_numpy(b.reads).to(dev)
    wins = torch.from_numpy(b.wins).to(dev)
    rl = torch.from_numpy(b.read_len.view(np.int16)).to(dev)
    wl = torch.from_numpy(b.win_len.view(np.int16)).to(dev)
    score = torch.zeros(b.n_pairs, dtype=torch.int32, device=dev)
    ei = torch.zeros(b.n_pairs, dtype=torch.int16, device=dev)
    ej = torch.zeros(b.n_pairs, dtype=torch.int16, device=dev)
    sc = Scoring(gap_open=3 if args.affine else 0, gap_extend=1 if args.affine else 2,
                 affine=args.affine, want_coords=args.coords)
    ctx = Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    for layout in args.layouts.split(","):
      for gl in args.group_lanes.split(","):
        if layout == "auto":
            os.environ.pop("MSW_LAYOUT", None)
        else:
            os.environ["MSW_LAYOUT"] = layout
        if int(gl):
            os.environ["MSW_GROUP_LANES"] = gl
        else:
            os.environ.pop("MSW_GROUP_LANES", None)
        for n in sizes:
            cells = int((b.read_len[:n].astype(np.int64) * b.win_len[:n]).sum())
            step = ctx.prepare_device_launch(reads.data_ptr(), rl.data_ptr(), wins.data_ptr(), wl.data_ptr(),
                                             b.reads.shape[1], b.wins.shape[1], n, score.data_ptr(),
                                             int(b.read_len.max()), int(b.win_len.max()), sc,
                                             ei.data_ptr(), ej.data_ptr(), stream.cuda_stream)
            for _ in range(3):
                step()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.reps):
                step()
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            print(json.dumps({"layout": layout, "G": int(gl), "pairs": n, "ms": round(ms, 4),
                              "gcups": round(cells / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
