#!/usr/bin/env python3
"""Do two HIP streams run config-2 launches concurrently?  It depends on
which hardware queues they land on (GPU_MAX_HW_QUEUES, 4 on the box: HIP
maps streams onto its queues as they are created): create `pre` streams
first, then the pair, and time K launches alternating over the pair.

  python3 tools/stream_queues.py > out.jsonl
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from mini_parallel_amd import Context, Scoring
    from mini_parallel_amd.synthetic import config_shard
    b = config_shard(2, 0, 10_000)
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    t = lambda x, dt=None: torch.from_numpy(np.ascontiguousarray(x if dt is None else x.view(dt))).to(dev)  # noqa
    r, w, rl, wl = t(b.reads), t(b.wins), t(b.read_len, np.int16), t(b.win_len, np.int16)
    outs = [torch.zeros(b.n_pairs, dtype=torch.int32, device=dev) for _ in range(2)]
    keep = []
    print(json.dumps({"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}), flush=True)
    for pre in range(0, 6):
        extra = [torch.cuda.Stream(dev) for _ in range(pre)]
        pair = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        keep += extra + pair
        steps = [ctx.prepare_device_launch(r.data_ptr(), rl.data_ptr(), w.data_ptr(), wl.data_ptr(), b.reads.shape[1],
                                           b.wins.shape[1], b.n_pairs, o.data_ptr(), int(b.read_len.max()),
                                           int(b.win_len.max()), Scoring(), stream=s.cuda_stream)
                 for o, s in zip(outs, pair)]
        for _ in range(300):
            steps[0]()
            steps[1]()
        res = {}
        for ns in (1, 2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(400):
                steps[k % ns]()
            torch.cuda.synchronize()
            res[ns] = round((time.perf_counter() - t0) / 400 * 1e6, 2)
        print(json.dumps({"streams_created_before_pair": pre, "total_streams_so_far": len(keep) + 5,
                          "us_per_step_1": res[1], "us_per_step_2": res[2]}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
