#!/usr/bin/env python3
"""A/B: config-2 steps back to back on one stream vs alternating over two
streams (each with its own score buffer), so a step's first waves start while
the previous step's last waves drain and the launch gap is hidden.

  python3 tools/step_overlap.py [--steps 200] [--reps 5] > out.jsonl

Per variant and repetition: wall per step (barrier-free: synchronize, K
launches, synchronize) and the mean per-launch kernel time from event pairs
around every launch on its own stream; the scores of both buffers are checked
equal to the one-stream run."""
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
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--pairs", type=int, default=10_000)
    a = ap.parse_args()
    import torch
    from mini_parallel_amd import Context, Scoring
    from mini_parallel_amd.synthetic import config_shard
    b = config_shard(2, 0, a.pairs)
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    t = lambda x, dt=None: torch.from_numpy(np.ascontiguousarray(x if dt is None else x.view(dt))).to(dev)  # noqa
    r, w, rl, wl = t(b.reads), t(b.wins), t(b.read_len, np.int16), t(b.win_len, np.int16)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    outs = [torch.zeros(b.n_pairs, dtype=torch.int32, device=dev) for _ in range(2)]
    steps = [ctx.prepare_device_launch(r.data_ptr(), rl.data_ptr(), w.data_ptr(), wl.data_ptr(), b.reads.shape[1],
                                       b.wins.shape[1], b.n_pairs, o.data_ptr(), int(b.read_len.max()),
                                       int(b.win_len.max()), Scoring(), stream=s.cuda_stream)
             for o, s in zip(outs, streams)]
    cells = b.cells

    def run(nstreams, events):
        evs = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.steps):
            i = k % nstreams
            if events:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(streams[i])
                steps[i]()
                e1.record(streams[i])
                evs.append((e0, e1))
            else:
                steps[i]()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.steps
        kern = float(np.mean([x.elapsed_time(y) for x, y in evs])) * 1e-3 if evs else None
        return wall, kern

    for _ in range(3):
        run(2, False)
    ref = None
    for rep in range(a.reps):
        for ns in (1, 2):
            for ev in (False, True):
                outs[0].zero_()
                outs[1].zero_()
                wall, kern = run(ns, ev)
                s0 = outs[0].cpu().numpy()
                ref = s0 if ref is None else ref
                ok = bool(np.array_equal(s0, ref) and (ns == 1 or np.array_equal(outs[1].cpu().numpy(), ref)))
                print(json.dumps({"rep": rep, "streams": ns, "events": ev, "us_per_step": round(wall * 1e6, 2),
                                  "gcups": round(cells / wall / 1e9, 1),
                                  "kernel_us": None if kern is None else round(kern * 1e6, 2), "scores_equal": ok}),
                      flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
