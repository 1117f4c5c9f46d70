#!/usr/bin/env python3
"""Config-2 steps issued one by one vs as one captured HIP graph of K
launches (torch.cuda.CUDAGraph around the library's launches on the capture
stream), after a preheat: wall per step for K = 20 and 200.

  python3 tools/graph_probe.py > out.jsonl
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
    s = torch.cuda.Stream(dev)
    out = torch.zeros(b.n_pairs, dtype=torch.int32, device=dev)
    step = ctx.prepare_device_launch(r.data_ptr(), rl.data_ptr(), w.data_ptr(), wl.data_ptr(), b.reads.shape[1],
                                     b.wins.shape[1], b.n_pairs, out.data_ptr(), int(b.read_len.max()),
                                     int(b.win_len.max()), Scoring(), stream=s.cuda_stream)
    graphs = {}
    for K in (20, 200):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(K):
                step()
        graphs[K] = g
    ref = None
    for rep in range(3):
        for K in (20, 200):
            for mode in ("launches", "graph"):
                t0 = time.perf_counter()
                while time.perf_counter() - t0 < 0.1:  # preheat
                    for _ in range(20):
                        step()
                    torch.cuda.synchronize()
                out.zero_()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if mode == "graph":
                    graphs[K].replay()
                else:
                    for _ in range(K):
                        step()
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / K
                sc = out.cpu().numpy()
                ref = sc if ref is None else ref
                print(json.dumps({"rep": rep, "K": K, "mode": mode, "us_per_step": round(dt * 1e6, 2),
                                  "scores_equal": bool(np.array_equal(sc, ref)), "nonzero": int((sc != 0).sum())}),
                      flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
