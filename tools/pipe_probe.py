#!/usr/bin/env python3
"""Why bench.py's pipelined_two_streams does not overlap while
tools/stream_queues.py does: bench.py's own objects (Job, GpuWorkload,
pipelined_steps) under variants of its setup.

  python3 tools/pipe_probe.py VARIANT   (VARIANT: bench | no_set_stream | no_pg | gather_first | timed_first)
"""
import datetime
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    v = sys.argv[1]
    import torch
    import torch.distributed as dist
    if v != "no_pg":
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{bench._free_port()}", rank=0, world_size=1,
                                timeout=datetime.timedelta(minutes=5))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from mini_parallel_amd import Context
    from mini_parallel_amd.synthetic import config_shard
    ctx = Context(0)
    stream, stream2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    if v != "no_set_stream":
        torch.cuda.set_stream(stream)
    batch = config_shard(2, 0, 10_000)
    sc = bench.scoring_of(2)
    work = bench.GpuWorkload(ctx, dev, stream, 2, batch, sc)
    job = bench.Job(0, 1, 0, True, dev, stream)
    args = bench.parse(["--steps", "400", "--warmup", "5"])
    if v in ("gather_first", "timed_first"):
        from mini_parallel_amd import dist as mdist
        if v == "timed_first":
            job.preheat(work.step)
            job.fence()
            for _ in range(20):
                work.step()
            job.stop()
        job.max([1.0])
        job.sum([1])
        mdist.gather_results(work.score, work.ei, work.ej)
    for _ in range(3):
        p = bench.pipelined_steps(job, ctx, 2, batch, sc, work, stream2, args)
        job.preheat(work.step)
        job.fence()
        t0 = time.perf_counter()
        for _ in range(400):
            work.step()
        wall = job.stop() - t0
        print(json.dumps({"variant": v, "pipelined_us": p["ms_per_step"] * 1e3, "serial_us": round(wall / 400 * 1e6, 2)}),
              flush=True)
    ctx.close()
    if v != "no_pg":
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
