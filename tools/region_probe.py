#!/usr/bin/env python3
"""How much of bench.py's config-2 step time at K = 20 is the timed region's
two ends (host latency before the first launch runs, and after the last one
ends until the closing synchronize returns), by way of ending the region:
  sync     torch.cuda.synchronize()                      (bench.py's form)
  ev_sync  ev1.synchronize(), then torch.cuda.synchronize()
  stream   stream.synchronize(), then torch.cuda.synchronize()
Each variant runs R regions of K steps after the bench's preheat, variants
interleaved; prints per variant the median and spread of wall µs per step,
event µs per step, and wall - events (the two ends) per region.

  python3 tools/region_probe.py [--k 20] [--regions 60]
"""
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
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--regions", type=int, default=60)
    a = ap.parse_args()
    import torch
    from mini_parallel_amd import Context, Scoring
    from mini_parallel_amd.synthetic import config_shard
    b = config_shard(2, 0, 10_000)
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    t = lambda x, dt=None: torch.from_numpy(np.ascontiguousarray(x if dt is None else x.view(dt))).to(dev)  # noqa
    r, w, rl, wl = t(b.reads), t(b.wins), t(b.read_len, np.int16), t(b.win_len, np.int16)
    out = torch.zeros(b.n_pairs, dtype=torch.int32, device=dev)
    step = ctx.prepare_device_launch(r.data_ptr(), rl.data_ptr(), w.data_ptr(), wl.data_ptr(), b.reads.shape[1],
                                     b.wins.shape[1], b.n_pairs, out.data_ptr(), int(b.read_len.max()),
                                     int(b.win_len.max()), Scoring(), stream=stream.cuda_stream)

    def preheat(seconds=0.1):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            for _ in range(20):
                step()
            torch.cuda.synchronize(dev)

    def region(end):
        torch.cuda.synchronize(dev)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(a.k):
            step()
        e1.record(stream)
        if end == "ev_sync":
            e1.synchronize()
        elif end == "stream":
            stream.synchronize()
        torch.cuda.synchronize(dev)
        wall = (time.perf_counter() - t0) * 1e6
        ev = e0.elapsed_time(e1) * 1e3
        return wall / a.k, ev / a.k, wall - ev

    variants = ("sync", "ev_sync", "stream")
    res = {v: [] for v in variants}
    preheat()
    for i in range(a.regions):
        for v in variants:
            res[v].append(region(v))
            preheat(0.02)
    for v in variants:
        x = np.array(res[v])
        print(json.dumps({"end": v, "k": a.k, "regions": a.regions,
                          "wall_us_per_step": {"median": round(float(np.median(x[:, 0])), 2),
                                               "p10": round(float(np.percentile(x[:, 0], 10)), 2),
                                               "p90": round(float(np.percentile(x[:, 0], 90)), 2)},
                          "event_us_per_step_median": round(float(np.median(x[:, 1])), 2),
                          "ends_us": {"median": round(float(np.median(x[:, 2])), 1),
                                      "p90": round(float(np.percentile(x[:, 2], 90)), 1)}}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
