#!/usr/bin/env python3
"""A/B of two rustseq_mini builds on bench.py's full-size config-4 lane set
(tools/c4_full.py's dataset and per-file oracle check), runs alternating:

  python3 tools/c4_ab.py --cli-b tools/_variants/r03/rustseq_mini --out gpurun_out/T/ab.jsonl [--reps 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
from c4_full import run_cli  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cli-b", required=True)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dir", default="/tmp/msw_bench_c4")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    out_dir = os.path.dirname(os.path.abspath(a.out))
    os.makedirs(out_dir, exist_ok=True)
    args = bench.parse(["--c4-dir", a.dir])
    bench.ensure_c4_dataset(args)
    d, files, _ = bench.c4_layout(args)
    clis = {"a_head": os.path.join(ROOT, "mini_parallel_amd", "rustseq_mini"), "b": os.path.abspath(a.cli_b)}
    with open(a.out, "w") as f:
        for rep in range(a.reps):
            for tag, cli in clis.items():
                row = run_cli(d, files, "1", f"{tag}_{rep}", out_dir, cli=cli)
                row["cli"] = cli
                f.write(json.dumps(row) + "\n")
                f.flush()
                print(f"[c4_ab] {tag} rep {rep}: {row['reads_per_second'] / 1e6:.1f} M reads/s, wall "
                      f"{row['wall_ms']:.0f} ms, bit_exact {row['bit_exact']}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
