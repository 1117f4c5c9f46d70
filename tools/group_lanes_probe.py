#!/usr/bin/env python3
"""Lanes per pair group for large batches of 150 bp reads x 300 bp windows:
the layout model's choice (G = 8, KR = 19 once 17..24 packed rows are
allowed for any G) against 16-lane groups (KR = 10),
forced with MSW_GROUP_LANES, alternating three times (the clock drifts over
seconds of load, so a fixed order biases later settings).  Device-resident
batches, HIP events over R launches after a preheat; scores (and
coordinates) must agree across G.

  python3 tools/group_lanes_probe.py [--reps 20]
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--sizes", default="65536,131072,262144,1048576", help="pairs per launch, comma-separated")
    ap.add_argument("--settings", default="auto,16", help="two MSW_GROUP_LANES settings to alternate ('auto' = model)")
    ap.add_argument("--schemes", default="linear,linear_coords,affine_coords")
    a = ap.parse_args()
    sizes = [int(x) for x in a.sizes.split(",")]
    settings = a.settings.split(",")
    schemes = a.schemes.split(",")
    import torch
    from mini_parallel_amd import Context
    from mini_parallel_amd.aligner import AFFINE, LINEAR, LINEAR_COORDS
    from mini_parallel_amd.synthetic import config_shard
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    for n in sizes:
        b = config_shard(3, 0, n)  # 150 bp reads (indels: 149-151) x 300 bp windows
        t = lambda x, dt=None: torch.from_numpy(np.ascontiguousarray(x if dt is None else x.view(dt))).to(dev)  # noqa
        r, w, rl, wl = t(b.reads), t(b.wins), t(b.read_len, np.int16), t(b.win_len, np.int16)
        for name, sc in (("linear", LINEAR), ("linear_coords", LINEAR_COORDS), ("affine_coords", AFFINE)):
            if name not in schemes:
                continue
            ref = None
            for g in settings * 3:  # alternating: clocks drift under load
                if g == "auto":
                    os.environ.pop("MSW_GROUP_LANES", None)
                else:
                    os.environ["MSW_GROUP_LANES"] = g
                out = torch.zeros(n, dtype=torch.int32, device=dev)
                ei = torch.zeros(n, dtype=torch.int16, device=dev)
                ej = torch.zeros(n, dtype=torch.int16, device=dev)
                step = ctx.prepare_device_launch(r.data_ptr(), rl.data_ptr(), w.data_ptr(), wl.data_ptr(),
                                                 b.reads.shape[1], b.wins.shape[1], n, out.data_ptr(),
                                                 int(b.read_len.max()), int(b.win_len.max()), sc,
                                                 end_i_ptr=ei.data_ptr() if sc.want_coords else 0,
                                                 end_j_ptr=ej.data_ptr() if sc.want_coords else 0,
                                                 stream=stream.cuda_stream)
                t0 = time.perf_counter()
                while time.perf_counter() - t0 < 0.1:
                    step()
                    torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.reps):
                    step()
                e1.record(stream)
                torch.cuda.synchronize(dev)
                ms = e0.elapsed_time(e1) / a.reps
                got = (out.cpu().numpy(), ei.cpu().numpy(), ej.cpu().numpy())
                if ref is None:
                    ref = got
                same = all(np.array_equal(x, y) for x, y in zip(got, ref))
                print(json.dumps({"pairs": n, "scheme": name, "group_lanes": g, "ms_per_launch": round(ms, 4),
                                  "tcups": round(b.cells / (ms * 1e-3) / 1e12, 3), "equal_to_auto": same}),
                      flush=True)
    os.environ.pop("MSW_GROUP_LANES", None)
    ctx.close()


if __name__ == "__main__":
    main()
