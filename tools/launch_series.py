#!/usr/bin/env python3
"""Why the config-2 launch time depends on how many launches run back to
back (bench.py: 48.5 us per launch at K = 20, 45.1 at 200, 43.0 at 2000):
per-launch kernel times (an event pair around every launch) and the host's
enqueue time per launch, over a series of K launches started after an idle
gap, for several gaps; optionally with an nccl process group created first
(bench.py creates one), and the two-stream overlap with that group.

  python3 tools/launch_series.py [--nccl] > out.jsonl
"""
import argparse
import json
import os
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nccl", action="store_true")
    ap.add_argument("--k", type=int, default=300)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    if a.nccl:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        dist.barrier()
    from mini_parallel_amd import Context, Scoring
    from mini_parallel_amd.synthetic import config_shard
    b = config_shard(2, 0, 10_000)
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
    for _ in range(500):
        steps[0]()
    torch.cuda.synchronize()
    for gap in (0.0, 0.001, 0.01, 0.1):
        time.sleep(gap)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.k)]
        host = []
        for e0, e1 in evs:
            h0 = time.perf_counter()
            e0.record(streams[0])
            steps[0]()
            e1.record(streams[0])
            host.append(time.perf_counter() - h0)
        torch.cuda.synchronize()
        d = np.array([x.elapsed_time(y) * 1e3 for x, y in evs])
        gaps = np.array([evs[i][1].elapsed_time(evs[i + 1][0]) * 1e3 for i in range(a.k - 1)])
        print(json.dumps({"gap_s": gap, "nccl": a.nccl, "kernel_us_first10": [round(x, 1) for x in d[:10]],
                          "kernel_us_by_50": [round(float(d[i:i + 50].mean()), 2) for i in range(0, a.k, 50)],
                          "between_us_mean": round(float(gaps.mean()), 2),
                          "host_enqueue_us_mean": round(float(np.mean(host)) * 1e6, 2)}), flush=True)
    # bench.py's bracket after a long warm-up: K = 20 launches right after
    # (a) sync only, (b) sync + barrier + sync (nccl runs only)
    for variant in ("sync", "barrier"):
        if variant == "barrier" and not a.nccl:
            continue
        for _ in range(2000):
            steps[0]()
        torch.cuda.synchronize()
        tb = time.perf_counter()
        if variant == "barrier":
            dist.barrier()
            torch.cuda.synchronize()
        fence_us = (time.perf_counter() - tb) * 1e6
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(streams[0])
        for _ in range(20):
            steps[0]()
        e1.record(streams[0])
        torch.cuda.synchronize()
        print(json.dumps({"after_warmup_2000": variant, "nccl": a.nccl, "fence_us": round(fence_us, 1),
                          "wall_us_per_step": round((time.perf_counter() - t0) * 1e6 / 20, 2),
                          "event_us_per_step": round(e0.elapsed_time(e1) * 1e3 / 20, 2)}), flush=True)
    # two streams, no events, K launches alternating, vs one stream
    for ns in (1, 2, 1, 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.k):
            steps[k % ns]()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.k
        print(json.dumps({"streams": ns, "nccl": a.nccl, "us_per_step": round(dt * 1e6, 2)}), flush=True)
    ctx.close()
    if a.nccl:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
