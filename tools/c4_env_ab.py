#!/usr/bin/env python3
"""A/B of one rustseq_mini build under two environment settings on
bench.py's full-size config-4 lane set, runs alternating (every run's
per-file sums checked against the oracle, tools/c4_full.run_cli):

  python3 tools/c4_env_ab.py --b MSW_GFASTQ_BATCH=524288 --out gpurun_out/T/ab.jsonl [--reps 3]
  python3 tools/c4_env_ab.py --cli-b tools/bin/VARIANT/rustseq_mini --out ...
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
    ap.add_argument("--b", action="append", default=[], help="NAME=VALUE set for the b runs (repeatable)")
    ap.add_argument("--cli-b", default=None, help="another rustseq_mini build for the b runs (repo-relative)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dir", default="/tmp/msw_bench_c4")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    out_dir = os.path.dirname(os.path.abspath(a.out))
    os.makedirs(out_dir, exist_ok=True)
    args = bench.parse(["--c4-dir", a.dir])
    bench.ensure_c4_dataset(args)
    d, files, _ = bench.c4_layout(args)
    env_b = dict(kv.split("=", 1) for kv in a.b)
    with open(a.out, "w") as f:
        for rep in range(a.reps):
            for tag in ("a", "b"):
                saved = {k: os.environ.get(k) for k in env_b}
                if tag == "b":
                    os.environ.update(env_b)
                try:
                    row = run_cli(d, files, "1", f"{tag}_{rep}", out_dir,
                                  cli=os.path.join(ROOT, a.cli_b) if tag == "b" and a.cli_b else None)
                finally:
                    for k, v in saved.items():
                        if v is None:
                            os.environ.pop(k, None)
                        else:
                            os.environ[k] = v
                row["env"] = env_b if tag == "b" else {}
                row["cli"] = a.cli_b if tag == "b" and a.cli_b else "in-tree"
                f.write(json.dumps(row) + "\n")
                f.flush()
                print(f"[c4_env_ab] {tag} rep {rep}: {row['reads_per_second'] / 1e6:.1f} M reads/s, "
                      f"bit_exact {row['bit_exact']}", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
