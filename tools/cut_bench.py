#!/usr/bin/env python3
"""HBM roofline of the window-cut kernel alone (bench.py's cut_windows_roofline
leg), for A/B builds via MSW_LIB_PATH.  python tools/cut_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    sys.argv = [sys.argv[0]]
    import bench
    from mini_parallel_amd import Context
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = Context(0)
    for _ in range(3):
        print(json.dumps(bench.cut_roofline(ctx, dev, stream)), flush=True)


if __name__ == "__main__":
    main()
