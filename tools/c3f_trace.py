#!/usr/bin/env python3
"""Where config 3 from FASTQ spends its ~25 ms (bench.py's
configs_extra.config3.fastq: 2 BGZF lane files x 500k reads, affine + best
cell, --scores-out): bench's dataset, then the product's --full-wgs driver run
directly with the reader's span trace (MSW_GFASTQ_TRACE=1) and inflate timing
(MSW_GZ_TIMING=1), several times; prints the run records' timing fields and
the trace lines as JSON.

  python3 tools/c3f_trace.py --out gpurun_out/TAG/c3f_trace.jsonl [--runs 3]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--dir", default="/tmp/msw_bench_c4")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    args = bench.parse(["--c4-dir", a.dir])
    bench.ensure_c3f_dataset(args, 1)
    d, files, per = bench.c3f_layout(args, 1)
    cli = os.path.join(ROOT, "mini_parallel_amd", "rustseq_mini")
    with open(a.out, "w") as out:
        for k in range(a.runs):
            wd = tempfile.mkdtemp(prefix="c3ftrace_")
            env = dict(os.environ, WGS_DATA_DIR=d, WGS_SAMPLE_ID="SYN", WGS_LANES="1",
                       WGS_READS_PER_LANE=str(bench.C3F_RPL), GPU_CHUNK_SIZE_READS="65536",
                       MSW_GFASTQ_TRACE="1", MSW_GZ_TIMING="1", WGS_RUN_ID=f"c3ftrace{k}")
            cmd = [cli, "--full-wgs", "--gpu", "--score-mode", "sw", "--reference", os.path.join(d, "reference.fa"),
                   "--window", str(bench.C4_WINDOW), "--checkpoint-dir", wd, "--json", os.path.join(wd, "rec.json"),
                   "--num-gpus", "1", "--gap-model", "affine", "--scores-out", wd]
            t0 = time.perf_counter()
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
            proc_ms = (time.perf_counter() - t0) * 1e3
            if r.returncode:
                raise SystemExit(f"run {k}: rc {r.returncode}\n{r.stderr[-3000:]}")
            rec = json.load(open(os.path.join(wd, "rec.json")))
            row = {"run": k, "process_ms": round(proc_ms, 1),
                   **{f: rec.get(f) for f in ("wall_ms", "setup_ms", "teardown_ms", "kernel_ms", "setup_phases",
                                              "gpu_busy_fraction", "total_reads")},
                   "trace": [ln for ln in r.stderr.splitlines() if ln.startswith("[g")]}
            out.write(json.dumps(row) + "\n")
            out.flush()
            print(json.dumps({k2: v for k2, v in row.items() if k2 != "trace"}), flush=True)


if __name__ == "__main__":
    main()
