#!/usr/bin/env python3
"""Config 3 from FASTQ (bench.py's N = 1 lane set: one lane's R1/R2 BGZF
files of 500k reads, affine + best cell, per-read records) through the
--full-wgs driver under several environment settings, runs alternating
(settings in turn, `--reps` rounds); every run's records are compared with
the oracle's.  One JSON line per run: the timed wall, setup, and reads/s.

  python3 tools/c3f_env_ab.py --out gpurun_out/T/c3f_ab.jsonl \\
      --setting base= --setting batch131k=MSW_GFASTQ_BATCH=131072 [--reps 3]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--setting", action="append", required=True,
                    help="NAME=VAR=VALUE[,VAR=VALUE...] (NAME= for no change; CLI=path runs another build "
                         "of rustseq_mini, relative to the repo)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--sleep", type=float, default=0.0, help="seconds idle before each run (lets the previous "
                    "process's GPU teardown finish in the kernel)")
    ap.add_argument("--dir", default="/tmp/msw_bench_c4")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    args = bench.parse(["--c4-dir", a.dir])
    bench.ensure_c3f_dataset(args, 1)
    d, files, per = bench.c3f_layout(args, 1)
    settings = []
    for s in a.setting:
        name, _, rest = s.partition("=")
        env = dict(kv.split("=", 1) for kv in rest.split(",") if kv)
        settings.append((name, env))
    want = {}
    for p in files:
        z = np.load(p + ".oracle.npz")
        want[os.path.basename(p)] = (z["score"], z["end_i"], z["end_j"])
    cli = os.path.join(ROOT, "mini_parallel_amd", "rustseq_mini")
    with open(a.out, "w") as out:
        for rep in range(a.reps):
            for name, extra in settings:
                wd = tempfile.mkdtemp(prefix="c3fab_")
                extra = dict(extra)
                exe = os.path.join(ROOT, extra.pop("CLI")) if "CLI" in extra else cli
                env = dict(os.environ, WGS_DATA_DIR=d, WGS_SAMPLE_ID="SYN", WGS_LANES="1",
                           WGS_READS_PER_LANE=str(bench.C3F_RPL), GPU_CHUNK_SIZE_READS="65536",
                           WGS_RUN_ID=f"c3fab_{name}_{rep}", **extra)
                cmd = [exe, "--full-wgs", "--gpu", "--score-mode", "sw", "--reference", os.path.join(d, "reference.fa"),
                       "--window", str(bench.C4_WINDOW), "--checkpoint-dir", wd, "--json", os.path.join(wd, "rec.json"),
                       "--num-gpus", "1", "--gap-model", "affine", "--scores-out", wd]
                time.sleep(a.sleep)
                t0 = time.perf_counter()
                t_launch = time.time_ns()
                r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
                t_end = time.time_ns()
                proc_ms = (time.perf_counter() - t0) * 1e3
                if r.returncode:
                    raise SystemExit(f"{name} rep {rep}: rc {r.returncode}\n{r.stderr[-3000:]}")
                rec = json.load(open(os.path.join(wd, "rec.json")))
                tm, tr = rec.get("t_main_unix_ns"), rec.get("t_record_unix_ns")
                phases = {"start_ms": round((tm - t_launch) * 1e-6, 1), "main_to_record_ms": round((tr - tm) * 1e-6, 1),
                          "exit_ms": round((t_end - tr) * 1e-6, 1)} if tm and tr else None
                bad = 0
                for base, (s, i, j) in want.items():
                    g = np.fromfile(os.path.join(wd, base + ".scores"), dtype=[("s", "<i4"), ("i", "<i2"), ("j", "<i2")])
                    bad += int((g["s"] != s).sum() + (g["i"] != i).sum() + (g["j"] != j).sum()) if g.size == s.size \
                        else s.size
                row = {"setting": name, "env": extra, "rep": rep, "wall_ms": round(rec["wall_ms"], 2),
                       "setup_ms": round(rec["setup_ms"], 1),
                       "reads_per_s": round(rec["total_reads"] / (rec["wall_ms"] * 1e-3)),
                       "reads_per_s_incl_setup": round(rec["total_reads"] / ((rec["wall_ms"] + rec["setup_ms"]) * 1e-3)),
                       "kernel_ms": rec.get("kernel_ms"), "teardown_ms": rec.get("teardown_ms"),
                       "process_wall_ms": round(proc_ms, 1), "setup_phases": rec.get("setup_phases"),
                       "process_phases": phases, "mismatches": bad}
                out.write(json.dumps(row) + "\n")
                out.flush()
                print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
