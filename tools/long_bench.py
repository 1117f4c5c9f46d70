"""Long-pair kernel throughput (sw_long_kernel, msw_long.hip) on device-resident
batches: GCUPS per shape and scoring kind, timed with HIP events on the launch
stream; MSW_FORCE_LONG=1 also times it on the packed kernels' config-2 shape
for comparison.  One JSON line per case.
  python3 tools/long_bench.py [--reps 20]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="", help="run the cases whose name contains this")
    args = ap.parse_args()
    import torch
    from mini_parallel_amd import Context, Scoring
    from mini_parallel_amd.synthetic import make_pairs
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()  # a real stream handle: launches and events on the same stream
    kinds = {"linear": Scoring(), "affine_coords": Scoring(affine=True, gap_open=3, gap_extend=1, want_coords=True)}
    cases = [("300x600", 40_000, 300, 2.0, False), ("1000x2000", 4_000, 1000, 2.0, False),
             ("150x5000", 8_000, 150, 5000 / 150, False), ("150x300_forced", 10_000, 150, 2.0, True),
             ("150x300_packed", 10_000, 150, 2.0, False), ("mixed_257-2000x2", 8_000, (257, 2000), 2.0, False),
             ("mixed_500-2000x2", 8_000, (500, 2000), 2.0, False), ("mixed_75-384x2", 100_000, (75, 384), 2.0, False)]
    for name, n, m, wf, force in cases:
        if args.only not in name:
            continue
        b = make_pairs(n, m, win_factor=wf, seed=4242)
        t = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in
             (b.reads, b.wins, b.read_len.view(np.int16), b.win_len.view(np.int16))]
        score = torch.zeros(n, dtype=torch.int32, device=dev)
        ei = torch.zeros(n, dtype=torch.int16, device=dev)
        ej = torch.zeros(n, dtype=torch.int16, device=dev)
        cells = float((b.read_len.astype(np.int64) * b.win_len).sum())
        mixed = isinstance(m, tuple)
        if force:
            os.environ["MSW_FORCE_LONG"] = "1"
        for kname, sc in kinds.items():
            if mixed:  # mixed lengths: a plan (length buckets, one launch per long-pair R)
                launch = ctx.prepare_planned_launch(t[0].data_ptr(), t[2].data_ptr(), t[1].data_ptr(),
                                                    t[3].data_ptr(), b.reads.shape[1], b.wins.shape[1], b.read_len,
                                                    b.win_len, score.data_ptr(), sc, ei.data_ptr(), ej.data_ptr(),
                                                    stream=st.cuda_stream)
            else:
                launch = ctx.prepare_device_launch(t[0].data_ptr(), t[2].data_ptr(), t[1].data_ptr(),
                                                   t[3].data_ptr(), b.reads.shape[1], b.wins.shape[1], n,
                                                   score.data_ptr(), int(b.read_len.max()), int(b.win_len.max()), sc,
                                                   ei.data_ptr(), ej.data_ptr(), stream=st.cuda_stream)
            for _ in range(3):
                launch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.reps):
                launch()
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            print(json.dumps({"case": name, "kind": kname, "pairs": n, "avg_launch_ms": round(ms, 4),
                              "gcups": round(cells / (ms * 1e6), 1)}), flush=True)
        os.environ.pop("MSW_FORCE_LONG", None)
    ctx.close()


if __name__ == "__main__":
    main()
