#!/usr/bin/env python3
"""CPU-side cost of `bench.py --gpus N`, measured on
this host without a GPU: everything the bench does on host cores before,
between and after its GPU work, at the driver's sizes.

  python3 tools/n8_readiness.py --world 8 --c4-dir /tmp/msw_n8 > out.json

Phases timed:
  prepare        bench.prepare_datasets at world N (config-4 pool of 32 x 1 M
                 scored segments + assembly of 16 lane files, config-3 FASTQ
                 lane files: two generated and scored, 2N - 2 copies)
  shard_gen      one rank's synthetic shards (config 2: 10k, config 3: 1M,
                 config 5: 100k pairs); N ranks run these side by side
  cpu_legs       rank 0's CPU baselines (bounded by --cpu-seconds, as in the
                 bench) and parity samples of every shard at world N
  c3f_parity     rank 0's check of all N x 1 M per-read records against the
                 oracle files (here against the oracle files themselves)
Prints one JSON object; DESIGN.md 6 turns it into the predicted N = 8 wall.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--c4-dir", default="/tmp/msw_n8")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--skip-prepare", action="store_true")
    a = ap.parse_args()
    import bench
    from mini_parallel_amd import dist as mdist
    from mini_parallel_amd.synthetic import config_shard
    N = a.world
    args = bench.parse(["--gpus", str(N), "--c4-dir", a.c4_dir, "--cpu-seconds", str(a.cpu_seconds)])
    out = {"world": N, "host_cpus": bench.host_cpus(), "cpu_model": open("/proc/cpuinfo").read().split(
        "model name")[1].split("\n")[0].strip(": ")}
    t0 = time.perf_counter()
    if not a.skip_prepare:
        bench.prepare_datasets(args, [3, 4], N)
    out["prepare_s"] = round(time.perf_counter() - t0, 1)
    out["c4_meta"] = {k: v for k, v in (args._c4_meta or {}).items() if k in ("gen_seconds", "assemble_seconds",
                                                                              "oracle_thread_seconds", "reused")}
    out["c3f_meta"] = {k: v for k, v in (args._c3f_meta or {}).items() if k != "sizes"}
    gen = {}
    for cfg, per in ((2, 10_000), (3, 1_000_000), (5, 100_000)):
        lo, hi = mdist.shard_range(per * N, N - 1, N)
        t0 = time.perf_counter()
        b = config_shard(cfg, lo, hi)
        gen[f"config{cfg}"] = round(time.perf_counter() - t0, 2)
    out["shard_gen_s_per_rank"] = gen
    # rank 0's CPU baselines and the all-shard parity samples (oracle scores
    # stand in for the gathered GPU results)
    t0 = time.perf_counter()
    legs = {}
    for cfg, per in ((2, 10_000), (3, 1_000_000), (5, 100_000)):
        sc = bench.scoring_of(cfg)
        b = config_shard(cfg, 0, per)
        from oracle import oracle_lib
        oracle_lib.build()
        t1 = time.perf_counter()
        s, i, j, _ = oracle_lib.sw_batch_simd(b.reads[:4096], b.read_len[:4096], b.wins[:4096], b.win_len[:4096],
                                              threads=bench.host_cpus()[2], coords=sc.want_coords,
                                              **bench._oracle_kw(sc))
        legs[f"config{cfg}_oracle_4096_s"] = round(time.perf_counter() - t1, 2)
        secs = args.cpu_seconds if cfg == 2 else max(1.0, args.cpu_seconds / 2)
        g = np.zeros(per, np.int32)
        t1 = time.perf_counter()
        bench.cpu_baseline(args, b, sc, g, np.zeros(per, np.int16), np.zeros(per, np.int16), seconds=secs)
        legs[f"config{cfg}_cpu_baseline_s"] = round(time.perf_counter() - t1, 1)
        n_total = per * N
        gs = np.zeros(n_total, np.int32)
        t1 = time.perf_counter()
        bench.parity_sample(cfg, sc, n_total, N, gs, np.zeros(n_total, np.int16), np.zeros(n_total, np.int16))
        legs[f"config{cfg}_parity_sample_s"] = round(time.perf_counter() - t1, 1)
    t1 = time.perf_counter()
    bench.cpu_baseline_c4(args)
    legs["config4_cpu_baseline_s"] = round(time.perf_counter() - t1, 1)
    out["rank0_cpu_legs"] = legs
    out["rank0_cpu_legs_s"] = round(time.perf_counter() - t0, 1)
    # config-3 FASTQ parity at world N: every record of the 2N files
    d, files, per = bench.c3f_layout(args, N)
    t0 = time.perf_counter()
    n = 0
    for p in files:
        z = np.load(p + ".oracle.npz")
        want = np.stack([z["score"], z["end_i"], z["end_j"]], 1).astype(np.int64)
        got = want.copy()
        n += int((got != want).any(axis=1).sum() == 0) * want.shape[0]
    out["c3f_parity_s"] = round(time.perf_counter() - t0, 2)
    out["c3f_records"] = n
    du = 0
    for root, _, fs in os.walk(a.c4_dir):
        du += sum(os.path.getsize(os.path.join(root, f)) for f in fs)
    out["dataset_bytes"] = du
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
