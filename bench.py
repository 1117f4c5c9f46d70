#!/usr/bin/env python3
"""bench.py -- GCUPS of the batched Smith-Waterman scoring path on MI355X.

Workload (BASELINE.json configs[1], "config 2"): 10,000 synthetic 150 bp
reads x 300 bp reference windows per GPU, linear gap (+2/-1/-2), score-only,
inputs resident in HBM.  One step = one pass of the hot path
(msw_align_batch_device: the hand-written gfx950 kernel through the C ABI)
over the batch.

Multi-GPU (SURVEY 8e, weak scaling): ONE global seeded batch of
pairs_per_gpu x N pairs (mini_parallel_amd.synthetic.config_shard: pair i is
the same whoever generates it); rank r scores shard_range(B, r, N) with no
data-path collective; after the timed region the scores are gathered to every
rank over RCCL (all_gather, the only collective of the path) and rank 0 checks
the gathered scores against the oracle on a sample taken from every shard.
value = cells of all ranks / max-over-ranks wall time.

Launch: ``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``
(the driver's form) or ``python bench.py --gpus N``, which starts the N rank
processes itself (children, before anything touches the GPU).  Fewer visible
GPUs than N is an error (exit status 3), never a quiet n_gpus = 1.

Extra fields: ``roofline`` (HBM, as north_star asks; algorithmic bytes per
launch / average launch time from HIP events on the launch stream), ``valu``
(the binding VALU-integer ceilings: the loop's instruction mix, SURVEY 8d's
mapping-independent i32 ceiling and the lone-wave issue bound),
``cpu_baseline`` (oracle restatement on rank 0's host cores, bounded sample,
at every N), ``parity``, ``pcie_inclusive``, ``cut_windows_roofline`` and,
at every N, ``configs_extra``: the other BASELINE configs, sharded over the
same ranks --
  config3  1M pairs/GPU affine + best cell, HBM-resident kernel rate AND the
           host-to-host rate through pinned chunked staging (BASELINE:
           "async FASTQ chunk staging", aligner.rs:269-289, :466-475);
  config4  a bounded config-4 stream: 8 lanes x 2 BGZF FASTQ lane files
           generated before the timed region, rank r runs the product's
           --full-wgs driver (GPU lane reader + genome-resident scoring) on
           lane files r::N, per-file i64 sums all-gathered over RCCL, one
           file checked against the oracle (aligner.rs:183-362);
  config5  100k mixed 75-250 bp pairs/GPU through one length-bucketed
           planned launch per rank, scores gathered over RCCL.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GCUPS (billion cell updates/s) on 150bp reads, 1/2/4/8 MI355X; bit-exact scores"

# Per-gfx950 constants (/opt/skills/guides/MI355X_MICROARCH.md, chip table).
HBM_PEAK_GBPS = 8000.0
SIMDS, CLOCK_HZ = 256 * 4, 2.4e9
# VALU issue cycles per packed row-step (one wave instruction stream covering
# 64 lanes x 2 cells = 128 cells) of the f16 fast path at full occupancy: the
# compiled loop's VALU instructions per row-step (hipcc -S of msw_kernels.hip,
# KR = 13: linear 243 / 52, +coords 192 / 26, affine 455 / 52, affine+coords
# 298 / 26) x 4.1 cycles, the issue cost of v_pk_add_f16, v_pk_maximum3_f16,
# v_perm_b32, v_lshl_or_b32, v_bfi_b32 and v_max3_u32 measured by
# tools/ubench_valu.hip.  A lone wave issues at most one
# instruction per ~4.75 cycles, so one-wave-per-SIMD batches sit below this.
# (score-only loops run 4 steps per iteration, best-cell loops 2).
CYCLES_PER_ROW_STEP = {"linear": 19.16, "linear_coords": 30.28, "affine": 35.88,
                       "affine_coords": 46.99}
DEFAULT_PAIRS = {2: 10_000, 3: 1_000_000, 5: 100_000}

# SURVEY 8d's mapping-independent VALU ceiling: 256 CU x 4 SIMD x 32 i32
# lanes/clk x 2.4 GHz lane-ops/s over the algorithmic i32 ops per cell
# (linear score 6: substitution 2, diagonal add, max(up, left), -gap, max3
# with 0; affine + best cell 13: E 3, F 3, H 3, substitution 2, key 2; the
# other two kinds by the same count: +2 for the key, -2 without it).
VALU_LANE_OPS = 256 * 4 * 32 * 2.4e9
I32_OPS_PER_CELL = {"linear": 6, "linear_coords": 8, "affine": 11, "affine_coords": 13}
# tools/ubench_valu.hip (profiles/r01/ubench_valu_gfx950.txt): a packed op
# issues every 4.1 cycles per SIMD at occupancy, a lone wave (one wave per
# SIMD, config 2: 1000 waves on 1024 SIMDs) at best every 4.75 cycles.
PACKED_ISSUE_CYCLES, LONE_WAVE_ISSUE_CYCLES = 4.1, 4.75

PREHEAT_S = 0.1  # seconds of back-to-back steps before each timed region (Job.preheat)
STREAM_REPS = 400  # batches in the timed pass of pcie_inclusive's streaming variant

# config-4 leg: 8 lanes x R1/R2 BGZF lane files (aligner.rs:198-204 naming) of
# 25 M reads = 400 M reads (BASELINE config 4: "8 lanes x ~50 M reads"), each
# file 25 segments of 1 M reads from a pool of 32 distinct pre-scored segments
C4_LANES, C4_READS_PER_LANE, C4_READS_PER_FILE = 8, 2, 25_000_000
C4_SEGMENT_READS, C4_POOL = 1_000_000, 32
C4_GENOME, C4_WINDOW, C4_LEVEL, C4_QUAL, C4_SEED = 64 << 20, 300, 6, "binned", 1004


def valu_block(kind: str, kernel_gcups: float) -> dict:
    """The binding VALU ceilings of a kernel rate: the instruction-mix
    ceiling of the loop that ran (rises if the loop gets longer -- so never
    alone), SURVEY 8d's mapping-independent i32 ceiling, and the lone-wave
    issue bound of the instruction mix."""
    mix = 128.0 / CYCLES_PER_ROW_STEP[kind] * SIMDS * CLOCK_HZ / 1e9
    i32 = VALU_LANE_OPS / I32_OPS_PER_CELL[kind] / 1e9
    lone = mix * PACKED_ISSUE_CYCLES / LONE_WAVE_ISSUE_CYCLES
    return {"kernel_gcups": round(kernel_gcups, 1),
            "ceiling_gcups": round(mix, 1), "frac": round(kernel_gcups / mix, 4),
            "cycles_per_packed_row_step": CYCLES_PER_ROW_STEP[kind],
            "basis": "VALU issue bound of the f16 loop's instruction mix at full occupancy, 2.4 GHz peak "
                     "clock (~2.2 GHz sustained, tools/wave_trace.py; DESIGN.md 4.3)",
            "i32_ceiling_gcups": round(i32, 1), "frac_i32_ceiling": round(kernel_gcups / i32, 4),
            "i32_ops_per_cell": I32_OPS_PER_CELL[kind],
            "i32_basis": "SURVEY 8d: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz / i32 ops per cell "
                         "(mapping-independent; packed 16-bit cells can exceed it)",
            "lone_wave_ceiling_gcups": round(lone, 1), "frac_lone_wave": round(kernel_gcups / lone, 4),
            "lone_wave_basis": f"the instruction-mix ceiling x {PACKED_ISSUE_CYCLES}/{LONE_WAVE_ISSUE_CYCLES} "
                               "cycles per issue (tools/ubench_valu.hip): the bound of launches with at most "
                               "one wave per SIMD"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default 1, or WORLD_SIZE under torch.distributed.run")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 5],
                    help="BASELINE config whose batch shape is timed (2 = the metric's)")
    ap.add_argument("--pairs", type=int, default=0, help="override pairs per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target CPU work for the cpu_baseline sample (0 disables)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-pcie", action="store_true", help="skip the host-memory (PCIe) rate")
    ap.add_argument("--extra-configs", default="3,4,5",
                    help="other BASELINE configs timed as configs_extra keys at every N ('' or 'none' = none)")
    ap.add_argument("--c3-pairs", type=int, default=0, help="config-3 leg: pairs per GPU (default 1M)")
    ap.add_argument("--c5-pairs", type=int, default=0, help="config-5 leg: pairs per GPU (default 100k)")
    ap.add_argument("--c4-reads-per-file", type=int, default=C4_READS_PER_FILE,
                    help="config-4 leg: reads per lane file (8 lanes x 2 files)")
    ap.add_argument("--c4-segment-reads", type=int, default=C4_SEGMENT_READS,
                    help="config-4 leg: reads per pooled segment (lane files are made of segments)")
    ap.add_argument("--c4-pool", type=int, default=C4_POOL, help="config-4 leg: distinct segments in the pool")
    ap.add_argument("--c3-fastq-reads", type=int, default=1_000_000,
                    help="config-3 FASTQ leg: reads per GPU, as one lane (R1 + R2 lane files) per GPU "
                         "(0 = skip the leg)")
    ap.add_argument("--c4-dir", default="/tmp/msw_bench_c4",
                    help="configs 3 / 4 FASTQ legs: where the lane files are generated (reused across runs)")
    ap.add_argument("--no-h2h", action="store_true", help="config-3 leg: skip the host-to-host rate")
    ap.add_argument("--detail", default="",
                    help="where the full record goes (default gpurun_out/bench_detail_n<N>.json); the stdout "
                         "line keeps the contract's keys and a per-leg summary")
    ap.add_argument("--cpu-standin", action="store_true",
                    help="TEST ONLY (tests/test_bench_launcher.py): gloo ranks on the CPU with a "
                         "stand-in scorer, to exercise the launcher, sharding and gather without a GPU")
    ap.add_argument("--share-gpu", action="store_true",
                    help="TEST ONLY, oversubscribed: every rank runs the real GPU path on device 0 (contexts, "
                         "kernels, per-rank CLI children with MSW_DEVICES=0), collectives over gloo on host "
                         "tensors (RCCL refuses two ranks on one device); the line says \"oversubscribed\": "
                         "true and is never a scaling point (tests/test_bench_contract.py)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# Host CPU accounting (the GPU box: 256 CPUs in the affinity mask, a cgroup
# quota of 16 CPUs -- tools/probe_host.sh).
# ---------------------------------------------------------------------------
def cgroup_cpu_quota():
    """CPUs' worth of time the cgroup grants (cpu.max), or None if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        return None


def host_cpus():
    aff = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    return aff, quota, usable


def physical_cores():
    """Physical cores of the host (lscpu-free: unique (package, core) ids)."""
    seen = set()
    try:
        base = "/sys/devices/system/cpu"
        for d in os.listdir(base):
            if d.startswith("cpu") and d[3:].isdigit():
                try:
                    with open(f"{base}/{d}/topology/physical_package_id") as f:
                        pk = f.read().strip()
                    with open(f"{base}/{d}/topology/core_id") as f:
                        co = f.read().strip()
                    seen.add((pk, co))
                except OSError:
                    pass
    except OSError:
        pass
    return len(seen) or (os.cpu_count() or 1)


# ---------------------------------------------------------------------------
# Launcher: N rank processes, started before anything touches the GPU.
# ---------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def visible_gpus() -> int:
    import torch  # device_count() does not initialise the GPU on this image
    return int(torch.cuda.device_count())


def launch_ranks(args, argv) -> int:
    n = args.gpus
    if not args.cpu_standin:
        have = visible_gpus()
        if have < (1 if args.share_gpu else n):
            print(f"bench.py: --gpus {n} asked for {n} ranks but only {have} GPU(s) are visible; "
                  f"refusing to report a smaller run", file=sys.stderr, flush=True)
            return 3
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc, alive = 0, list(procs)
    while alive:
        for p in list(alive):
            r = p.poll()
            if r is None:
                continue
            alive.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in alive:  # our own children, by PID
                    q.terminate()
        time.sleep(0.02)
    return rc


# ---------------------------------------------------------------------------
# CPU baseline and parity (test infrastructure: oracle/)
# ---------------------------------------------------------------------------
def _oracle_kw(scoring):
    return dict(match=scoring.match, mismatch=scoring.mismatch, gap_open=scoring.gap_open,
                gap_extend=scoring.gap_extend, affine=scoring.affine)


def cpu_baseline(args, batch, scoring, gpu_scores, gpu_i, gpu_j, seconds=None):
    """The CPU baseline, timed on this host: the inter-sequence SIMD
    restatement of the oracle (oracle/sw_simd.c, AVX-512BW 32 x int16 lanes /
    AVX2 16, bit-exact with the scalar oracle by tests/test_oracle.py) over a
    bounded sample of the timed pairs sized to ~cpu_seconds, on every CPU the
    process may use (the affinity mask capped by the cgroup CPU quota), plus
    the scalar oracle on one core.  Parity: GPU vs the SIMD results on the
    whole sample and vs the scalar oracle on its smaller sample."""
    from oracle import oracle_lib
    oracle_lib.build()
    budget = args.cpu_seconds if seconds is None else seconds
    aff, quota, usable = host_cpus()
    threads = args.cpu_threads or usable
    kw = _oracle_kw(scoring)
    coords = scoring.want_coords

    def cells_of(n):
        return int((batch.read_len[:n].astype(np.int64) * batch.win_len[:n]).sum())

    def simd(n, thr):
        return oracle_lib.sw_batch_simd(batch.reads[:n], batch.read_len[:n], batch.wins[:n],
                                        batch.win_len[:n], threads=thr, coords=coords, **kw)

    # calibrate on a small sample, then size the sample to ~cpu_seconds
    n0 = min(batch.n_pairs, 256 * threads)
    ts = time.perf_counter()
    simd(n0, threads)
    rate = n0 / max(time.perf_counter() - ts, 1e-6)
    ns = int(min(batch.n_pairs, max(n0, rate * budget)))
    passes = max(1, int(rate * budget / ns))
    ts = time.perf_counter()
    for _ in range(passes):
        cs, ci, cj, isa = simd(ns, threads)
    dt = time.perf_counter() - ts
    scells = passes * cells_of(ns)
    gcups = scells / dt / 1e9
    # one thread: the per-core rate (for the full-host extrapolation)
    n1c = max(32, min(ns, int(ns / max(threads, 1))))
    ts = time.perf_counter()
    simd(n1c, 1)
    one_core = cells_of(n1c) / max(time.perf_counter() - ts, 1e-9) / 1e9
    # every CPU of the affinity mask (throttled by the cgroup quota, if any)
    all_aff = None
    if aff != threads:
        ts = time.perf_counter()
        simd(ns, aff)
        all_aff = {"threads": aff, "gcups": round(cells_of(ns) / (time.perf_counter() - ts) / 1e9, 3)}
    # scalar oracle, one core, ~1/5 of the budget
    n1 = max(1, min(ns, int(budget * 0.2 * 2e8 / max(cells_of(1), 1))))
    ts = time.perf_counter()
    ss, si, sj = oracle_lib.sw_batch(batch.reads[:n1], batch.read_len[:n1], batch.wins[:n1],
                                     batch.win_len[:n1], threads=1, **kw)
    scalar_gcups = cells_of(n1) / max(time.perf_counter() - ts, 1e-9) / 1e9
    phys = physical_cores()
    isa_s = 'AVX-512BW 32' if isa == 512 else ('AVX2 16' if isa == 256 else 'scalar 1')
    cpu = {"value": round(gcups, 3), "unit": "GCUPS", "cores": threads, "kind": "port",
           "sample": f"{passes} pass(es) over the first {ns} of the {batch.n_pairs} timed pairs "
                     f"({scells} cells, {dt:.1f} s): oracle/sw_simd.c, inter-sequence {isa_s} x int16 "
                     f"lanes, {threads} threads = the CPUs this process may use "
                     f"(affinity {aff}, cgroup quota {quota if quota is not None else 'none'})",
           "cpu_model": oracle_lib.cpu_model(), "isa_bits": isa,
           "affinity_cpus": aff, "cgroup_cpu_quota": quota, "physical_cores": phys,
           "one_thread_gcups": round(one_core, 3),
           "all_affinity_threads": all_aff,
           "full_host_extrapolated_gcups": round(one_core * phys, 1),
           "full_host_note": "one thread's rate x the host's physical cores (linear scaling, SMT "
                             "ignored): an extrapolation, not a measurement -- the cgroup grants "
                             "this job only the quota above",
           "scalar_oracle_1core_gcups": round(scalar_gcups, 4)}
    mism = int((cs != gpu_scores[:ns]).sum()) + int((ss != gpu_scores[:n1]).sum())
    if coords:
        mism += int(((ci != gpu_i[:ns]) | (cj != gpu_j[:ns])).sum())
        mism += int(((si != gpu_i[:n1]) | (sj != gpu_j[:n1])).sum())
    parity = {"checked_pairs": ns, "checked_pairs_scalar": n1, "mismatches": mism, "bit_exact": mism == 0}
    return cpu, parity


def parity_sample(cfg, scoring, n_total, world, g_score, g_i, g_j, per_shard=512):
    """Rank 0, N > 1: the GATHERED scores against the SIMD oracle on a sample
    from every shard -- pairs [mid - per_shard/2, mid + per_shard/2) around
    each shard's midpoint, regenerated from the global batch's seed."""
    from mini_parallel_amd import dist as mdist
    from mini_parallel_amd.synthetic import config_shard
    from oracle import oracle_lib
    oracle_lib.build()
    _, _, usable = host_cpus()
    checked, mism, ranges = 0, 0, []
    for r in range(world):
        a, b = mdist.shard_range(n_total, r, world)
        mid = (a + b) // 2
        lo, hi = max(a, mid - per_shard // 2), min(b, mid + per_shard // 2)
        if hi <= lo:
            continue
        s = config_shard(cfg, lo, hi)
        cs, ci, cj, _ = oracle_lib.sw_batch_simd(s.reads, s.read_len, s.wins, s.win_len, threads=usable,
                                                 coords=scoring.want_coords, **_oracle_kw(scoring))
        mism += int((cs != g_score[lo:hi]).sum())
        if scoring.want_coords:
            mism += int(((ci != g_i[lo:hi]) | (cj != g_j[lo:hi])).sum())
        checked += hi - lo
        ranges.append([lo, hi])
    return {"checked_pairs": checked, "checked_ranges": ranges, "mismatches": mism,
            "bit_exact": mism == 0 and checked > 0, "source": "gathered scores of all ranks"}


def standin_scores(batch):
    """--cpu-standin: a deterministic function of each pair's bytes (NOT a
    scorer), so the launcher/shard/gather path can run without a GPU."""
    rl = batch.read_len.astype(np.int64)
    cols = np.arange(batch.reads.shape[1])[None, :]
    s = (batch.reads.astype(np.int64) * (cols < rl[:, None])).sum(axis=1)
    return ((s * 31 + batch.win_len.astype(np.int64)) % 100_003).astype(np.int32)


# ---------------------------------------------------------------------------
# GPU pieces
# ---------------------------------------------------------------------------
def cut_roofline(ctx, dev, stream):
    """The path's HBM-bound kernel on its own: msw_genome_cut_device cutting
    1M 300 bp windows (random positions in a 64 Mbp genome) into a 304 B/row
    slab, timed with HIP events on the launch stream.  Algorithmic bytes per
    window: 300 genome + 304 slab + 8 position + 2 requested + 2 clipped length."""
    import torch
    n, ws, glen, reps = 1_000_000, 304, 64 << 20, 20
    rng = np.random.default_rng(7)
    genome = ctx.load_genome(rng.choice(np.frombuffer(b"ACGT", np.uint8), glen))
    d_pos = torch.from_numpy(rng.integers(0, glen - 300, n).astype(np.int64)).to(dev)
    d_want = torch.full((n,), 300, dtype=torch.int16, device=dev)
    d_wins = torch.empty((n, ws), dtype=torch.uint8, device=dev)
    d_len = torch.empty(n, dtype=torch.int16, device=dev)

    def launch():
        genome.cut_device(d_pos.data_ptr(), d_want.data_ptr(), n, d_wins.data_ptr(), ws, d_len.data_ptr(),
                          stream.cuda_stream)
    for _ in range(3):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        launch()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    t = e0.elapsed_time(e1) * 1e-3 / reps
    genome.close()
    alg = n * (300 + ws + 8 + 2 + 2)
    return {"kernel": "cut_windows_kernel", "bound": "hbm", "achieved": round(alg / t / 1e9, 1),
            "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(alg / t / 1e9 / HBM_PEAK_GBPS, 4),
            "avg_launch_ms": round(t * 1e3, 4), "alg_bytes_per_launch": alg,
            "workload": "1M x 300 bp windows from a 64 Mbp HBM-resident genome -> 304 B/row slab"}


def pcie_rates(ctx, batch, scoring, cells, gpu_scores):
    from mini_parallel_amd.aligner import pinned_empty

    def pinned(a):
        p = pinned_empty(a.shape, a.dtype)
        p[...] = a
        return p

    ws = batch.wins.shape[1]
    genome = ctx.load_genome(np.ascontiguousarray(batch.wins).reshape(-1))
    pos = np.arange(batch.n_pairs, dtype=np.int64) * ws
    pairs = (batch.reads, batch.read_len, batch.wins, batch.win_len)
    reads = (batch.reads, batch.read_len, pos, batch.win_len)
    variants = {
        "pairs_pageable": (ctx.align_batch, pairs),
        "pairs_pinned": (ctx.align_batch, tuple(pinned(a) for a in pairs)),
        "genome_pageable": (lambda *a, **k: ctx.align_reads(genome, *a, **k), reads),
        "genome_pinned": (lambda *a, **k: ctx.align_reads(genome, *a, **k), tuple(pinned(a) for a in reads)),
    }
    out, best_v = {}, None
    for name, (fn, arrs) in variants.items():
        for chunk in (0, (batch.n_pairs + 3) // 4):
            s, _, _ = fn(*arrs, scoring=scoring, chunk_pairs=chunk)  # warm the staging slots
            if not np.array_equal(s, gpu_scores):
                raise SystemExit(f"pcie variant {name} disagrees with the device-resident scores")
            best = 1e30
            for _ in range(3):
                ts = time.perf_counter()
                fn(*arrs, scoring=scoring, chunk_pairs=chunk)
                best = min(best, time.perf_counter() - ts)
            key = f"{name}{'' if chunk == 0 else '_4chunks'}"
            out[key] = {"gcups": round(cells / best / 1e9, 2), "ms_per_batch": round(best * 1e3, 3)}
            if best_v is None or out[key]["gcups"] > out[best_v]["gcups"]:
                best_v = key
    # Streaming: a run of batches submitted asynchronously, three in flight
    # (msw_align_reads_async + wait on the oldest ticket), as the --full-wgs
    # driver feeds chunks: the steady-state host-to-host rate.  The first
    # pass (>= PREHEAT_S) ramps the clock; the second, STREAM_REPS batches
    # (~30 ms), is timed.  submit_us = host time inside the submission calls.
    depth = 3
    arrs = variants["genome_pinned"][1]
    for reps in (None, STREAM_REPS):
        ts = time.perf_counter()
        pend, sub, k = [], 0.0, 0
        while (k < reps) if reps else (k < 3 or time.perf_counter() - ts < PREHEAT_S):
            t1 = time.perf_counter()
            pend.append(ctx.align_reads(genome, *arrs, scoring=scoring, asynchronous=True))
            sub += time.perf_counter() - t1
            k += 1
            if len(pend) == depth:
                pend.pop(0).wait()
        while pend:
            s_last = pend.pop(0).wait()[0]
        dt = (time.perf_counter() - ts) / k
    if not np.array_equal(s_last, gpu_scores):
        raise SystemExit("pcie streaming variant disagrees with the device-resident scores")
    out["genome_pinned_stream"] = {"gcups": round(cells / dt / 1e9, 2), "ms_per_batch": round(dt * 1e3, 3),
                                   "batches": k, "submit_us_per_batch": round(sub / k * 1e6, 1)}
    if out["genome_pinned_stream"]["gcups"] > out[best_v]["gcups"]:
        best_v = "genome_pinned_stream"
    genome.close()
    h2d_bytes = {"pairs": int(batch.reads.nbytes + batch.wins.nbytes + 4 * batch.n_pairs),
                 "genome": int(batch.reads.nbytes + 12 * batch.n_pairs)}
    return {"value": out[best_v]["gcups"], "unit": "GCUPS", "best": best_v, "variants": out,
            "h2d_bytes_per_batch": h2d_bytes,
            "path": "host arrays -> GPU -> scores on the host (msw_align_batch / msw_align_reads), rank 0; "
                    "scores checked equal to the device-resident run"}


def scoring_of(cfg):
    from mini_parallel_amd import Scoring
    return {2: Scoring(), 3: Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True),
            5: Scoring()}[cfg]


def kind_of(scoring):
    return ("affine" if scoring.affine else "linear") + ("_coords" if scoring.want_coords else "")


def alg_bytes_of(batch, scoring):
    """Algorithmic HBM bytes of one pass: every read and window byte once,
    plus the outputs (4 B score, +4 B coordinates)."""
    return int(batch.read_len.astype(np.int64).sum() + batch.win_len.astype(np.int64).sum()
               + batch.n_pairs * (8 if scoring.want_coords else 4))


class GpuWorkload:
    """A batch resident in HBM plus a zero-argument launch of the hot path
    on ``stream`` (configs 2/3: msw_align_batch_device; config 5: one planned
    length-bucketed launch, plan built outside the timed region)."""

    def __init__(self, ctx, dev, stream, cfg, batch, scoring):
        import torch
        self.batch, self.scoring, self.stream = batch, scoring, stream

        def to_dev(a, dt=None):
            a = np.ascontiguousarray(a if dt is None else a.view(dt))
            return torch.from_numpy(a).to(dev)

        self.reads, self.wins = to_dev(batch.reads), to_dev(batch.wins)
        self.rlen, self.wlen = to_dev(batch.read_len, np.int16), to_dev(batch.win_len, np.int16)
        n = batch.n_pairs
        self.score = torch.zeros(n, dtype=torch.int32, device=dev)
        self.ei = torch.zeros(n, dtype=torch.int16, device=dev)
        self.ej = torch.zeros(n, dtype=torch.int16, device=dev)
        self.max_m, self.max_n = int(batch.read_len.max()), int(batch.win_len.max())
        if cfg == 5:
            self.step = ctx.prepare_planned_launch(
                self.reads.data_ptr(), self.rlen.data_ptr(), self.wins.data_ptr(), self.wlen.data_ptr(),
                batch.reads.shape[1], batch.wins.shape[1], batch.read_len, batch.win_len,
                self.score.data_ptr(), scoring, self.ei.data_ptr(), self.ej.data_ptr(), stream.cuda_stream)
        else:
            self.step = ctx.prepare_device_launch(
                self.reads.data_ptr(), self.rlen.data_ptr(), self.wins.data_ptr(), self.wlen.data_ptr(),
                batch.reads.shape[1], batch.wins.shape[1], n, self.score.data_ptr(), self.max_m,
                self.max_n, scoring, self.ei.data_ptr(), self.ej.data_ptr(), stream.cuda_stream)

    def results(self):
        return self.score.cpu().numpy(), self.ei.cpu().numpy(), self.ej.cpu().numpy()


class Job:
    """This rank's place in the job and the bracket every timed region uses:
    synchronize, barrier, synchronize (the contract's form), max / sum over
    ranks.  gpu=False is --cpu-standin (gloo, CPU tensors).  shared=True is
    --share-gpu: the GPU path on device 0 for every rank, collectives over
    gloo on host tensors (comm_dev None)."""

    def __init__(self, rank, world, local_rank, gpu, dev=None, stream=None, shared=False):
        self.rank, self.world, self.local_rank, self.gpu = rank, world, local_rank, gpu
        self.dev, self.stream, self.shared = dev, stream, shared
        self.dev_index = 0 if shared else local_rank  # the GPU this rank (and its CLI child) runs on
        self.comm_dev = dev if (gpu and not shared) else None

    def sync(self):
        if self.gpu:
            import torch
            torch.cuda.synchronize(self.dev)

    def fence(self):
        """Start of a timed region (and a plain rendezvous): synchronize,
        barrier, synchronize.  One rank has no one to wait for: no barrier
        (the gathers and reductions still run through the group)."""
        from mini_parallel_amd import dist as mdist
        self.sync()
        if mdist.active() and self.world > 1:
            import torch.distributed as dist
            dist.barrier()
        self.sync()

    def stop(self):
        """End of a timed region: this rank's GPU work finished -> the clock
        reading; then the barrier, outside the reading (ranks started together
        at the fence, and the job's time is the max over ranks)."""
        self.sync()
        t = time.perf_counter()
        self.fence()
        return t

    def preheat(self, step, seconds=PREHEAT_S):
        """After the warm-up steps: repeat the step back to back until the GPU
        has run it for `seconds`.  An idle GPU drops its clock and takes ~10 ms
        of load to ramp back (config 2: 49.4 us per launch after a 10 ms idle
        spell, 44.8 after ~200 launches; tools/launch_series.py), so a 1 ms
        timed region right after setup measures the ramp, not the kernel.
        Untimed; reported as `preheat` beside `warmup`."""
        if not self.gpu or seconds <= 0:
            return {"steps": 0, "seconds": 0.0}
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            for _ in range(20):
                step()
            n += 20
            self.sync()
        return {"steps": n, "seconds": round(time.perf_counter() - t0, 3)}

    def max(self, vals):
        from mini_parallel_amd import dist as mdist
        return mdist.max_over_ranks(vals, device=self.comm_dev)

    def sum(self, vals):
        from mini_parallel_amd import dist as mdist
        return mdist.sum_over_ranks(vals, device=self.comm_dev)

    def tensor(self, a):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(a))
        return t.to(self.comm_dev) if self.comm_dev is not None else t

    def wire(self, *ts):
        """Result tensors as the process group moves them: on the GPU for
        RCCL, copied to host memory for gloo (--share-gpu)."""
        return [t if self.comm_dev is not None else t.cpu() for t in ts]

    def gather(self, *ts):
        from mini_parallel_amd import dist as mdist
        return mdist.gather_results(*self.wire(*ts))


def leg_pairs(job, ctx, cfg, args):
    """configs_extra.config3 / .config5: each rank scores its shard of one
    global seeded batch (pairs_per_gpu x N pairs, HBM-resident; config 5
    through one planned length-bucketed launch), kernel time from HIP events
    on the launch stream, the job's rate over the max-over-ranks wall; the
    scores (and best cells) are all-gathered over RCCL and rank 0 checks a
    sample from every shard against the oracle.  Config 3 adds the
    host-to-host rate (leg_h2h)."""
    import torch
    from mini_parallel_amd import dist as mdist
    from mini_parallel_amd.synthetic import config_shard
    scoring = scoring_of(cfg)
    kind = kind_of(scoring)
    per_gpu = (args.c3_pairs if cfg == 3 else args.c5_pairs) or DEFAULT_PAIRS[cfg]
    n_total = per_gpu * job.world
    a, b = mdist.shard_range(n_total, job.rank, job.world)
    t0 = time.perf_counter()
    batch = config_shard(cfg, a, b)
    gen_s = time.perf_counter() - t0
    reps = 5 if cfg == 3 else 20
    h2h = None
    if job.gpu:
        w = GpuWorkload(ctx, job.dev, job.stream, cfg, batch, scoring)
        for _ in range(2):
            w.step()
        job.preheat(w.step)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        job.fence()
        t0 = time.perf_counter()
        e0.record(job.stream)
        for _ in range(reps):
            w.step()
        e1.record(job.stream)
        wall = job.stop() - t0
        kern = e0.elapsed_time(e1) * 1e-3 / reps
        outs = [w.score] + ([w.ei, w.ej] if scoring.want_coords else [])
    else:
        job.fence()
        t0 = time.perf_counter()
        for _ in range(reps):
            s = standin_scores(batch)
        wall = job.stop() - t0
        kern = wall / reps
        outs = [torch.from_numpy(s)]
    wall_max, kern_max = job.max([wall, kern])
    (job_cells,) = job.sum([batch.cells])
    gathered = job.gather(*outs)
    if cfg == 3 and job.gpu and not args.no_h2h:
        dev_res = [t.cpu().numpy() for t in outs]
        del w, outs
        torch.cuda.empty_cache()
        h2h = leg_h2h(job, ctx, batch, scoring, dev_res)
    elif job.gpu:
        del w, outs
        torch.cuda.empty_cache()
    if job.rank != 0:
        return None
    g = [t.cpu().numpy() for t in gathered]
    if job.gpu:
        par = parity_sample(cfg, scoring, n_total, job.world, g[0], g[1] if len(g) > 1 else None,
                            g[2] if len(g) > 2 else None)
    else:
        want = standin_scores(config_shard(cfg, 0, n_total))
        par = {"standin": True, "gather_in_order": bool(np.array_equal(g[0], want)), "pairs": int(g[0].size)}
    cpu = None
    if job.gpu and args.cpu_seconds > 0:
        # the CPU baseline of this leg's own pairs (rank 0's shard; BASELINE.md's
        # plan), which also checks that shard's sample bit for bit
        n0 = batch.n_pairs
        cpu, cpar = cpu_baseline(args, batch, scoring, g[0][:n0], g[1][:n0] if len(g) > 1 else None,
                                 g[2][:n0] if len(g) > 2 else None, seconds=max(1.0, args.cpu_seconds / 2))
        par["rank0_cpu_sample"] = cpar
        par["bit_exact"] = bool(par["bit_exact"] and cpar["bit_exact"])
        par["mismatches"] += cpar["mismatches"]
    kernel_gcups = batch.cells / kern / 1e9
    alg = alg_bytes_of(batch, scoring)
    # counter traffic of this leg's kernel at this size (tools/profile_round.sh)
    tr = load_pmc_traffic(f"config{cfg}:{kind}") if (job.gpu and per_gpu == DEFAULT_PAIRS[cfg]) else None
    return {"workload": f"config{cfg}: {per_gpu} pairs/GPU of one global {n_total}-pair batch, reads "
                        f"{int(batch.read_len.min())}-{int(batch.read_len.max())} bp x windows "
                        f"{int(batch.win_len.min())}-{int(batch.win_len.max())} bp, {kind.replace('_', '+')}, "
                        "HBM-resident" + (", one length-bucketed planned launch per rank" if cfg == 5 else ""),
            "n_ranks": job.world, "pairs_per_gpu": per_gpu, "global_pairs": n_total, "scaling": "weak",
            "job_gcups": round(job_cells * reps / wall_max / 1e9, 1),
            "kernel_gcups": round(kernel_gcups, 1), "avg_launch_ms": round(kern * 1e3, 4),
            "max_avg_launch_ms": round(kern_max * 1e3, 4), "launches": reps,
            "valu": valu_block(kind, kernel_gcups),
            "roofline_hbm": {"achieved": round(alg / kern / 1e9, 2), "frac": round(alg / kern / 1e9 / HBM_PEAK_GBPS, 5),
                             "alg_bytes_per_launch": alg,
                             "traffic": round(tr["hbm_bytes_per_launch"]) if tr else None,
                             "traffic_over_alg": round(tr["hbm_bytes_per_launch"] / alg, 3) if tr else None,
                             "traffic_detail": tr},
            "parity": par, "gathered_pairs": int(g[0].size), "host_to_host": h2h, "cpu_baseline": cpu,
            "gen_seconds": round(gen_s, 1)}


def pipelined_steps(job, ctx, cfg, batch, scoring, work, s2, args):
    """"pipelined_two_streams": the same K steps over the same batch, issued
    alternately on two streams (a second score buffer on a second stream),
    so step k + 1's waves start while step k's drain -- two waves per SIMD
    where one launch of 10k pairs leaves one.  Each step is
    still one complete pass over the batch; the serial one-stream rate stays
    `value`.  Scores of both buffers must equal."""
    import torch
    w2 = GpuWorkload(ctx, job.dev, s2, cfg, batch, scoring)
    pair = (work.step, w2.step)
    for k in range(max(2, args.warmup)):
        pair[k & 1]()
    job.preheat(lambda: (pair[0](), pair[1]()))
    job.fence()
    t0 = time.perf_counter()
    for k in range(args.steps):
        pair[k & 1]()
    wall = job.stop() - t0
    same = bool(torch.equal(work.score, w2.score))
    (wall_max,) = job.max([wall])
    (cells, bad) = job.sum([batch.cells, 0 if same else 1])
    del w2
    if job.rank != 0:
        return None
    return {"value": round(cells * args.steps / wall_max / 1e9, 2), "unit": "GCUPS",
            "ms_per_step": round(wall_max * 1e3 / args.steps, 4), "streams": 2, "steps": args.steps,
            "scores_equal_across_streams": bad == 0,
            "note": "the timed K steps again, alternating over two streams (two batches in flight); "
                    "not `value`, which runs one batch at a time"}


def leg_h2h(job, ctx, batch, scoring, dev_res, chunk=32768):
    """configs_extra.config3.host_to_host -- BASELINE config 3 as stated
    ("async FASTQ chunk staging"): the rank's pairs start in pinned host
    memory (msw_host_alloc, aligner.rs:466-475 USE_PINNED_MEMORY) and go
    through the library's chunked pipeline (aligner.rs:269-289's per-chunk
    loop: chunks of `chunk` pairs, H2D on the copy stream under the previous
    chunk's kernel, results back on the readback stream), scores and best
    cells back in host memory.  Two forms: the reads + window positions
    against an HBM-resident genome (msw_align_reads; here the genome is the
    shard's windows back to back, so the cut windows are exactly the batch's)
    and the reads + windows themselves (msw_align_batch).  Setup (genome
    upload, pinned fills) is outside the timed calls; each call is bracketed
    by the job fence; best of 3; results must equal the HBM-resident run.
    Chunks of 32 K pairs: with the chunks' kernels alternating over two
    compute streams, 16 K / 32 K / 64 K / 128 K pairs run 5.18-5.21 /
    5.16-5.18 / 4.99-5.03 / 4.83-4.86 TCUPS (tools/h2h_sweep.py,
    profiles/r03/h2h/chunk_sweep_two_streams.jsonl)."""
    from mini_parallel_amd.aligner import pinned_empty

    def pinned(a):
        p = pinned_empty(a.shape, a.dtype)
        p[...] = a
        return p
    ws = batch.wins.shape[1]
    genome = ctx.load_genome(np.ascontiguousarray(batch.wins).reshape(-1))
    reads, rl, wl = pinned(batch.reads), pinned(batch.read_len), pinned(batch.win_len)
    ppos, pwins = pinned(np.arange(batch.n_pairs, dtype=np.int64) * ws), pinned(batch.wins)
    variants = {
        "genome_pinned": (lambda: ctx.align_reads(genome, reads, rl, ppos, wl, scoring=scoring, chunk_pairs=chunk)),
        "pairs_pinned": (lambda: ctx.align_batch(reads, rl, pwins, wl, scoring=scoring, chunk_pairs=chunk)),
    }
    out, equal = {}, True
    for name, fn in variants.items():
        res = fn()  # warm: staging slots, kernel instance
        equal = equal and bool(np.array_equal(res[0], dev_res[0]))
        if scoring.want_coords:
            equal = equal and bool(np.array_equal(res[1], dev_res[1]) and np.array_equal(res[2], dev_res[2]))
        best = 1e30
        for _ in range(3):
            job.fence()
            t0 = time.perf_counter()
            fn()
            best = min(best, job.stop() - t0)
        out[name] = best
    genome.close()
    walls = job.max([out[k] for k in variants])
    (cells,) = job.sum([batch.cells])
    (ok,) = job.sum([0 if equal else 1])
    if job.rank != 0:
        return None
    res = {k: {"gcups": round(cells / t / 1e9, 1), "ms_per_batch": round(t * 1e3, 3)} for k, t in zip(variants, walls)}
    best = max(res, key=lambda k: res[k]["gcups"])
    return {"value": res[best]["gcups"], "unit": "GCUPS", "best": best, "variants": res,
            "chunk_pairs": chunk, "pairs_per_gpu": batch.n_pairs,
            "h2d_bytes_per_pair": {"genome_pinned": int(batch.reads.shape[1] + 12),
                                   "pairs_pinned": int(batch.reads.shape[1] + ws + 4)},
            "equal_to_hbm_resident_run": ok == 0,
            "path": "pinned host arrays -> chunked async H2D (copy stream) -> kernels (compute stream) -> "
                    "scores + best cells in host memory; whole-job rate over the max-over-ranks wall"}


# ---------------------------------------------------------------------------
# FASTQ-backed legs: lane files on disk -> the product's --full-wgs driver
# (rustseq_mini) as a child process per rank.  Datasets are written once,
# before any rank touches a GPU, and reused while their DONE.json matches.
# ---------------------------------------------------------------------------
_POOL_GENOME = None  # set before forking the generator pools (shared copy-on-write)


def _lane_names(lanes, rpl):
    return ["SYN_L%03d_R%d_001.fastq.gz" % (ln, r) for ln in range(1, lanes + 1) for r in range(1, rpl + 1)]


def _write_reference(path, g, seed):
    with open(path, "w") as f:
        f.write(">synthetic seed=%d\n" % seed)
        s = g.tobytes().decode()
        f.write("\n".join(s[k:k + 80] for k in range(0, len(s), 80)) + "\n")


def _marker_ok(d, names):
    try:
        with open(os.path.join(d, "DONE.json")) as f:
            m = json.load(f)
        if all(os.path.getsize(os.path.join(d, n)) == m["sizes"][n] for n in names):
            return m
    except (OSError, ValueError, KeyError):
        pass
    return None


def _write_marker(d, m):
    p = os.path.join(d, "DONE.json")
    with open(p + ".tmp", "w") as f:
        json.dump(m, f)
    os.replace(p + ".tmp", p)


def _run_pool(fn, jobs, workers, tag):
    """Run generator jobs on a fork pool, printing progress every 20 s (a
    silent minute would look like a hang to the GPU box's watchdog)."""
    from multiprocessing import get_context
    t0 = time.perf_counter()
    with get_context("fork").Pool(max(1, min(workers, len(jobs)))) as pool:
        res = pool.map_async(fn, jobs, chunksize=1)
        while not res.ready():
            res.wait(20)
            print(f"[bench] {tag}: {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)
        return res.get(), time.perf_counter() - t0


def _c4_segment_job(job):
    """One pooled config-4 segment: `n` reads of 150 bp (their own seeded
    run, synthetic._lane_reads), FASTQ text with binned qualities, BGZF at
    zlib level 6 as whole members without the EOF block (segments
    concatenate into lane files), then the oracle's score of every read
    against its genome window (one thread; the i64 sum is what a lane file
    made of this segment adds)."""
    from mini_parallel_amd.synthetic import _lane_reads, _lane_records, _with_windows, bgzf_compress
    from oracle import oracle_lib
    idx, n, path = job
    g = _POOL_GENOME
    b, pos, rng = _lane_reads(g, idx, n, 150, 2.0, C4_SEED, segment=1)
    data = bgzf_compress(_lane_records(b, pos, rng, b"SYN", idx // 2 + 1, C4_QUAL), C4_LEVEL, eof_block=False)
    with open(path, "wb") as f:
        f.write(data)
    w = _with_windows(g, b, pos)
    t0 = time.perf_counter()
    s, _, _, _ = oracle_lib.sw_batch_simd(w.reads, w.read_len, w.wins, w.win_len, threads=1, coords=False)
    dt = time.perf_counter() - t0
    return {"segment": idx, "reads": int(n), "bases": int(w.read_len.astype(np.int64).sum()),
            "score": int(s.astype(np.int64).sum()), "cells": int(w.cells), "oracle_s": dt, "bytes": len(data)}


def c4_layout(args):
    """Directory, lane file paths and segment plan of the config-4 dataset:
    16 lane files (8 lanes x R1/R2) of R reads each, lane file f made of
    segments plan[f] of a pool of P distinct S-read segments."""
    R, S, P = args.c4_reads_per_file, args.c4_segment_reads, args.c4_pool
    if S <= 0 or R % S:
        raise SystemExit(f"bench.py: --c4-reads-per-file {R} must be a multiple of --c4-segment-reads {S}")
    d = os.path.join(args.c4_dir, f"l{C4_LANES}x{C4_READS_PER_LANE}_r{R}_seg{S}x{P}_g{C4_GENOME}_z{C4_LEVEL}"
                                  f"{C4_QUAL}_s{C4_SEED}")
    names = _lane_names(C4_LANES, C4_READS_PER_LANE)
    nseg = R // S
    plan = [[(f * nseg + s) % P for s in range(nseg)] for f in range(len(names))]
    return d, [os.path.join(d, n) for n in names], plan


def _copy_into(dst, srcs, tail):
    """dst = the concatenation of the files srcs, then the bytes tail.
    Plain reads and writes, so the lane file's own pages are in the page
    cache, as a lane set that was just written or read is: copy_file_range
    reflinked the segments on the box's file system, which left every run
    paging the lane files in from disk (the first window of each file
    ~150 ms, GPU idle; tools/c4_trace.sh)."""
    with open(dst, "wb") as fo:
        for s in srcs:
            with open(s, "rb") as fi:
                while True:
                    buf = fi.read(64 << 20)
                    if not buf:
                        break
                    fo.write(buf)
        fo.write(tail)
        return fo.tell()


def ensure_c4_dataset(args) -> dict:
    """BASELINE config 4 at its stated size: 8 lanes x R1/R2 BGZF lane files
    of 25 M 150 bp reads (400 M reads; aligner.rs:198-204 naming, 51,858,562
    reads per file at aligner.rs:214).  A pool of P distinct 1 M-read
    segments is generated and scored by the oracle once; each lane file is
    the concatenation of 25 pooled segments (BGZF members concatenate into a
    valid multi-member gzip), so its expected (score i64, reads, bases) is
    the sum over its segments.  Segments repeat across and within files --
    stated in the record.  Written before any rank touches a GPU."""
    from concurrent.futures import ThreadPoolExecutor

    from mini_parallel_amd.synthetic import BGZF_EOF, wgs_genome
    from oracle import oracle_lib
    global _POOL_GENOME
    d, files, plan = c4_layout(args)
    names = [os.path.basename(p) for p in files]
    m = _marker_ok(d, names)
    if m is not None:
        m["reused"] = True
        return m
    import shutil
    if os.path.isdir(args.c4_dir):  # earlier config-4 datasets of this bench (disk: ~37 GB each)
        for e in os.listdir(args.c4_dir):
            if e.startswith(f"l{C4_LANES}x{C4_READS_PER_LANE}_r"):
                shutil.rmtree(os.path.join(args.c4_dir, e), ignore_errors=True)
    os.makedirs(os.path.join(d, "pool"), exist_ok=True)
    oracle_lib.build()
    oracle_lib.lib()
    _POOL_GENOME = wgs_genome(C4_SEED, C4_GENOME)
    _write_reference(os.path.join(d, "reference.fa"), _POOL_GENOME, C4_SEED)
    S, P = args.c4_segment_reads, args.c4_pool
    jobs = [(i, S, os.path.join(d, "pool", "seg_%03d.bgz" % i)) for i in range(P)]
    segs, gen_s = _run_pool(_c4_segment_job, jobs, host_cpus()[2], f"config-4 segment pool ({P} x {S} reads)")
    _POOL_GENOME = None
    need = sum(segs[i]["bytes"] for row in plan for i in row)
    free = shutil.disk_usage(d).free
    if free < need + (2 << 30):
        raise RuntimeError(f"config-4 lane files need {need / 1e9:.1f} GB, {args.c4_dir} has {free / 1e9:.1f} GB free")
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=min(16, len(files))) as ex:
        futs = [ex.submit(_copy_into, fp, [jobs[i][2] for i in row], BGZF_EOF) for fp, row in zip(files, plan)]
        sizes = [fu.result() for fu in futs]
        print(f"[bench] config-4 lane files ({len(files)}) assembled: {time.perf_counter() - t0:.0f} s",
              file=sys.stderr, flush=True)
    asm_s = time.perf_counter() - t0
    expect = {n: {"score": sum(segs[i]["score"] for i in row), "reads": sum(segs[i]["reads"] for i in row),
                  "bases": sum(segs[i]["bases"] for i in row)} for n, row in zip(names, plan)}
    m = {"sizes": dict(zip(names, sizes)), "expect": expect, "plan": plan, "segments": segs,
         "gen_seconds": round(gen_s, 1), "assemble_seconds": round(asm_s, 1),
         "oracle_thread_seconds": round(sum(s["oracle_s"] for s in segs), 2), "bytes": int(sum(sizes))}
    _write_marker(d, m)
    m["reused"] = False
    return m


# config 3 from FASTQ (BASELINE: "1M synthetic 150 bp reads ... affine-gap
# score + best-cell coord, async FASTQ chunk staging"): 1 M reads per GPU in
# one lane's R1/R2 BGZF files, every read's (score, end_i, end_j) compared
# with the oracle.
C3F_RPL, C3F_GENOME, C3F_SEED = 2, 64 << 20, 1003


def _c3_file_job(job):
    """One config-3 lane file: its reads (synthetic._lane_reads, reads seed
    k), BGZF level 6 + EOF block, and the oracle's affine + best-cell result
    of every read (one thread) saved beside it."""
    from mini_parallel_amd.synthetic import _lane_reads, _lane_records, _with_windows, bgzf_compress
    from oracle import oracle_lib
    k, n, path = job
    g = _POOL_GENOME
    b, pos, rng = _lane_reads(g, k, n, 150, 2.0, C3F_SEED)
    data = bgzf_compress(_lane_records(b, pos, rng, b"SYN", k // C3F_RPL + 1, C4_QUAL), C4_LEVEL)
    with open(path, "wb") as f:
        f.write(data)
    w = _with_windows(g, b, pos)
    sc = scoring_of(3)
    t0 = time.perf_counter()
    s, i, j, _ = oracle_lib.sw_batch_simd(w.reads, w.read_len, w.wins, w.win_len, threads=1, coords=True,
                                          **_oracle_kw(sc))
    dt = time.perf_counter() - t0
    np.savez(path + ".oracle.npz", score=s, end_i=i, end_j=j)
    return {"bytes": len(data), "cells": int(w.cells), "reads": int(n), "oracle_s": dt}


def c3f_layout(args, world):
    """N lanes x R1/R2 = 2N lane files for N GPUs, each GPU's reads split
    over two files: rank r takes lane files r and r + N (WGS_FILE_SHARD), so
    the leg is weak-scaled like the HBM-resident config-3 leg.  (One lane per GPU
    rather than many small files: a file's first span cannot overlap its own
    inflate with scoring, so 16 files of 62.5k reads ran at 20 M reads/s and
    2 files of 500k at 40 M; smaller spans were slower still --
    profiles/r04/e2e/c3f_layout.jsonl, c3f_span.jsonl.)"""
    per = args.c3_fastq_reads // C3F_RPL
    d = os.path.join(args.c4_dir, f"c3fastq_{world}x{C3F_RPL}_r{per}_g{C3F_GENOME}_s{C3F_SEED}")
    # lane-major names (L001_R1, L001_R2, L002_R1, ...); rank r's files are r and r + N
    names = _lane_names(world, C3F_RPL)
    return d, [os.path.join(d, n) for n in names], per


def ensure_c3f_dataset(args, world) -> dict:
    from mini_parallel_amd.synthetic import wgs_genome
    from oracle import oracle_lib
    global _POOL_GENOME
    d, files, per = c3f_layout(args, world)
    names = [os.path.basename(p) for p in files]
    m = _marker_ok(d, names)
    if m is not None:
        m["reused"] = True
        return m
    os.makedirs(d, exist_ok=True)
    oracle_lib.build()
    oracle_lib.lib()
    _POOL_GENOME = wgs_genome(C3F_SEED, C3F_GENOME)
    _write_reference(os.path.join(d, "reference.fa"), _POOL_GENOME, C3F_SEED)
    # One oracle pass whatever N: rank r's lane files are r and r + N
    # (c3f_layout), and file k holds the reads of seed 0 if k < N, else of
    # seed 1 -- files 0 and N are generated and scored, ranks 1..N-1 get
    # byte-identical copies of them (and of their oracle results) under their
    # own names.  Every rank still scores 1 M reads (2 x 500k) from its own
    # files; 8 M distinct reads at N = 8 would cost ~2 min of generation and
    # oracle scoring on the box's 16 CPUs before any GPU work.
    src = [0 if k < world else world for k in range(len(files))]
    gen = sorted(set(src))
    res, gen_s = _run_pool(_c3_file_job, [(j, per, files[k]) for j, k in enumerate(gen)], host_cpus()[2],
                           f"config-3 lane files ({len(gen)} x {per} reads, {len(files) - len(gen)} copies)")
    _POOL_GENOME = None
    t0 = time.perf_counter()
    import shutil
    for k, sk in enumerate(src):
        if k != sk:
            shutil.copyfile(files[sk], files[k])
            shutil.copyfile(files[sk] + ".oracle.npz", files[k] + ".oracle.npz")
    by_gen = dict(zip(gen, res))
    m = {"sizes": {n: by_gen[sk]["bytes"] for n, sk in zip(names, src)},
         "cells": sum(by_gen[sk]["cells"] for sk in src),
         "files_generated": len(gen), "files_copied": len(files) - len(gen),
         "distinct_reads": per * len(gen), "copy_seconds": round(time.perf_counter() - t0, 2),
         "gen_seconds": round(gen_s, 1), "oracle_thread_seconds": round(sum(r["oracle_s"] for r in res), 2)}
    _write_marker(d, m)
    m["reused"] = False
    return m


def _standin_file(path):
    """--cpu-standin: per-file (score, reads, bases) from the host FASTQ
    reader, score = sum over reads of (31 * length + first byte) -- a
    deterministic function of the file, NOT a scorer."""
    from mini_parallel_amd.fastq import FastqReader
    score = reads = bases = 0
    with FastqReader(path) as fq:
        while True:
            seqs, lens = fq.next_chunk(4096, stride=256)
            if len(lens) == 0:
                break
            l64 = lens.astype(np.int64)
            score += int((31 * l64 + seqs[:, 0].astype(np.int64)).sum())
            reads += len(lens)
            bases += int(l64.sum())
    return score, reads, bases


def _standin_records(path):
    """--cpu-standin: per-read stand-in records (score, end_i, end_j) of a
    lane file, a deterministic function of each read (NOT a scorer)."""
    from mini_parallel_amd.fastq import FastqReader
    out = []
    with FastqReader(path) as fq:
        while True:
            seqs, lens = fq.next_chunk(4096, stride=256)
            if len(lens) == 0:
                break
            out.append(np.stack([31 * lens.astype(np.int32) + seqs[:, 0], lens.astype(np.int32) - 1,
                                 seqs[:, 1].astype(np.int32)], axis=1))
    return np.concatenate(out) if out else np.zeros((0, 3), np.int32)


def run_wgs_child(job, d, lanes, rpl, reference, extra_args, tag, timeout_s):
    """This rank's share of a lane set through the product's --full-wgs
    driver: rustseq_mini in a child process started after the job fence,
    lane files rank, rank + N, ... (WGS_FILE_SHARD), GPU = local rank.
    Returns (record, checkpoint, process seconds, workdir, error text)."""
    import tempfile
    cli = os.path.join(ROOT, "mini_parallel_amd", "rustseq_mini")
    wd = tempfile.mkdtemp(prefix=f"msw_{tag}_r{job.rank}_")
    env = dict(os.environ, WGS_DATA_DIR=d, WGS_SAMPLE_ID="SYN", WGS_LANES=str(lanes),
               WGS_READS_PER_LANE=str(rpl), GPU_CHUNK_SIZE_READS="65536",
               WGS_FILE_SHARD=f"{job.rank}/{job.world}", MSW_DEVICES=str(job.dev_index),
               WGS_RUN_ID=f"bench_{tag}_r{job.rank}_{os.getpid()}")
    rec_path = os.path.join(wd, "rec.json")
    cmd = [cli, "--full-wgs", "--gpu", "--score-mode", "sw", "--reference", reference, "--window", str(C4_WINDOW),
           "--checkpoint-dir", wd, "--json", rec_path, "--num-gpus", "1"] + [x.replace("{wd}", wd) for x in extra_args]
    job.fence()
    t0 = time.perf_counter()
    t_launch = time.time_ns()
    err, rec, ck = "", None, None
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout_s)
        t_end = time.time_ns()
        if r.returncode != 0:
            err = f"rustseq_mini exit {r.returncode}:\n" + (r.stdout[-1500:] + r.stderr[-1500:]).strip()
    except subprocess.TimeoutExpired as e:
        err = f"rustseq_mini did not finish in {timeout_s} s: {str(e.stdout or '')[-800:]}"
    proc = time.perf_counter() - t0
    job.fence()
    if not err:
        try:
            with open(rec_path) as f:
                rec = json.load(f)
            with open(os.path.join(wd, f"checkpoint_{rec['run_id']}.json")) as f:
                ck = json.load(f)
            # the child's own timeline (CLOCK_REALTIME stamps in its record)
            tm, tr = rec.get("t_main_unix_ns"), rec.get("t_record_unix_ns")
            rec["process_phases"] = {"start_ms": (tm - t_launch) * 1e-6 if tm else 0.0,
                                     "main_to_record_ms": (tr - tm) * 1e-6 if tm and tr else 0.0,
                                     "exit_ms": (t_end - tr) * 1e-6 if tr else 0.0}
        except (OSError, ValueError, KeyError) as e:
            err = f"run record unreadable: {e}"
    if err:
        print(f"bench.py rank {job.rank}: {tag} leg failed:\n{err}", file=sys.stderr, flush=True)
    return rec, ck, proc, wd, err


def _files_by_rank(fi, rank, dev, world):
    """The lane files each rank's CLI child processed (sorted) and the GPU
    ordinal it ran on (MSW_DEVICES; -1 for the CPU stand-in), from the
    gathered per-file rows."""
    by = [sorted(int(f) for f, r in zip(fi, rank) if r == k) for k in range(world)]
    devs = [sorted({int(d) for d, r in zip(dev, rank) if r == k}) for k in range(world)]
    return by, [d[0] if len(d) == 1 else d for d in devs]


def _setup_split(rec):
    """The CLI's setup phases (max over its workers), then its process
    phases (PROCESS_PHASES), as a flat list."""
    ph = (rec or {}).get("setup_phases") or {}
    pp = (rec or {}).get("process_phases") or {}
    return [float(ph.get(k, 0.0)) for k in SETUP_PHASES] + [float(pp.get(k, 0.0)) for k in PROCESS_PHASES]


# the CLI child's process wall, split: exec -> main (dynamic loading of the
# HIP runtime and libmsw), main -> run record written (HIP init, setup, the
# timed work, teardown), record -> reaped by the parent (process exit)
PROCESS_PHASES = ("start_ms", "main_to_record_ms", "exit_ms")


SETUP_PHASES = ("hip_init_ms", "reference_load_ms", "context_ms", "genome_ms", "result_sets_ms", "lane_reader_ms",
                "kernel_load_ms")
# what each phase inside setup_ms is (named in the record when it binds)
SETUP_WHY = {
    "context_ms": "the HIP runtime's device bring-up in the process's first stream creation (HSA queue "
                  "creation: 160-168 ms for the first hipStreamCreate on a fresh box, 2-14 ms for later ones, "
                  "tools/setup_probe.cpp, profiles/r04/setup/setup_probe.jsonl); once per process, after the "
                  "runtime init, so no call of ours can start it earlier",
    "genome_ms": "each worker's copy of the reference into its context's HBM (pageable host memory)",
    "result_sets_ms": "the workers' pinned host result buffers and their device twins",
    "lane_reader_ms": "the GPU lane reader's span, inflate and parse buffers",
    "kernel_load_ms": "the scoring kernels' code objects, loaded before the clock (msw_ctx_prepare)",
}


def _setup_bound(phases_ms):
    """The phase inside setup_ms that takes longest, and what it is."""
    k = max(SETUP_WHY, key=lambda n: phases_ms.get(n, 0.0))
    return {"phase": k, "ms": round(phases_ms.get(k, 0.0), 1), "why": SETUP_WHY[k]}


def leg_config4(job, args):
    """configs_extra.config4 -- BASELINE config 4 at its stated size: the 16
    lane files of ensure_c4_dataset (8 lanes x R1/R2 x 25 M reads = 400 M
    reads), sharded by file over the ranks (rank r: files r, r + N, ...;
    strong scaling: the dataset is fixed).  Each rank runs the product's
    --full-wgs driver on its GPU (GPU lane reader inflating and parsing on
    the GPU, windows cut from the HBM-resident genome, score-only kernel, two
    workers per GPU).  Per-file (score i64, reads, bases) rows are
    all-gathered over RCCL; rank 0 checks EVERY file against the oracle's
    composed segment sums (aligner.rs:183-362)."""
    from mini_parallel_amd import dist as mdist
    (bad,) = job.sum([1 if (args._c4_meta or {}).get("error") else 0])  # only rank 0 generated
    if bad:
        return None if job.rank else {"error": args._c4_meta["error"], "parity": {"bit_exact": False}}
    d, files, plan = c4_layout(args)
    F, R = len(files), args.c4_reads_per_file
    mine = list(range(job.rank, F, job.world))
    rows, stats, err, cells = [], [0.0] * 5, "", 0
    setup = [0.0] * (len(SETUP_PHASES) + len(PROCESS_PHASES))
    if job.gpu:
        rec, ck, proc, _, err = run_wgs_child(job, d, C4_LANES, C4_READS_PER_LANE, os.path.join(d, "reference.fa"),
                                              [], "c4", 900)
        if not err:
            for fr in ck["files"]:
                rows.append([files.index(fr["file_path"]), fr["score"], fr["total_reads"], fr["total_bases"],
                             1 if fr["completed"] else 0, job.rank, job.dev_index])
            stats = [rec["wall_ms"], proc * 1e3, rec["setup_ms"], rec["teardown_ms"], rec["kernel_ms"]]
            cells = int(rec["cells"])
            setup = _setup_split(rec)
    else:
        job.fence()
        t0 = time.perf_counter()
        for fi in mine:
            rows.append([fi, *_standin_file(files[fi]), 1, job.rank, -1])
        proc = time.perf_counter() - t0
        job.fence()
        stats = [proc * 1e3, proc * 1e3, 0.0, 0.0, 0.0]
        cells = sum(rw[3] for rw in rows) * C4_WINDOW
    mx = job.max(stats + [stats[2] + stats[0]] + setup)
    tot = job.sum([cells, 1 if err else 0])
    flat = np.array(rows, np.int64).reshape(-1)
    (g,) = mdist.gather_results(job.tensor(flat))
    if job.rank != 0:
        return None
    g = g.cpu().numpy().reshape(-1, 7)
    if tot[1]:
        return {"error": "the config-4 leg failed on some rank (see stderr)", "n_ranks": job.world,
                "parity": {"bit_exact": False}}
    table = np.zeros((F, 4), np.int64)
    seen = np.zeros(F, np.int64)
    for fi, sc, nr, nb, done, _, _ in g:
        table[fi] = (sc, nr, nb, done)
        seen[fi] += 1
    reads = int(table[:, 1].sum())
    with open(os.path.join(d, "DONE.json")) as f:
        expect = json.load(f)["expect"]
    bad = []
    for fi, p in enumerate(files):
        e = expect[os.path.basename(p)]
        ok_rb = table[fi, 1] == e["reads"] and table[fi, 2] == e["bases"]
        ok_sc = (table[fi, 0] == e["score"]) if job.gpu else True
        if not (ok_rb and ok_sc and table[fi, 3] == 1 and seen[fi] == 1):
            bad.append(os.path.basename(p))
    by_rank, dev_by_rank = _files_by_rank(g[:, 0], g[:, 5], g[:, 6], job.world)
    par = {"files": F, "files_once": bool((seen == 1).all()), "files_done": int(table[:, 3].sum()),
           "files_by_rank": by_rank, "child_device_by_rank": dev_by_rank,
           "files_sharded_as_cli": by_rank == [list(range(r, F, job.world)) for r in range(job.world)],
           "reads": reads, "reads_expected": F * R, "files_checked": F, "files_mismatched": bad,
           "check": "every lane file's (score i64, reads, bases) against the sums of its segments' oracle "
                    "results (oracle/sw_simd.c, each segment scored once when the pool was generated)"}
    if job.gpu:
        par["gpu_total_score"] = int(table[:, 0].sum())
        par["oracle_total_score"] = int(sum(expect[os.path.basename(p)]["score"] for p in files))
        par["bit_exact"] = not bad and reads == F * R
    else:
        want = _standin_file(files[0])
        par.update({"standin": True, "file0_ok": bool(tuple(table[0, :3]) == want), "rows_ok": not bad})
    wall_ms, proc_ms, setup_ms, tear_ms, kern_ms, setup_wall_ms = mx[:6]
    job_cells = int(tot[0])
    S, P = args.c4_segment_reads, args.c4_pool
    out = {"workload": f"config4: {C4_LANES} lanes x {C4_READS_PER_LANE} BGZF lane files x {R} reads of 150 bp "
                       f"= {F * R} reads (zlib level {C4_LEVEL}, {C4_QUAL} qualities), {C4_GENOME >> 20} Mbp "
                       f"HBM-resident genome, window {C4_WINDOW}, linear score sums per file; each file is "
                       f"{R // S} segments of {S} reads drawn from a pool of {P} distinct segments (segments repeat)",
           "n_ranks": job.world, "scaling": "strong", "files_per_rank": len(mine), "reads": reads,
           "gcups": round(job_cells / (wall_ms * 1e6), 1),
           "reads_per_s": round(reads / (wall_ms * 1e-3)),
           "reads_per_s_incl_setup": round(reads / (setup_wall_ms * 1e-3)),
           "reads_per_s_process": round(reads / (proc_ms * 1e-3)),
           "wall_ms": round(wall_ms, 1), "setup_ms": round(setup_ms, 1), "teardown_ms": round(tear_ms, 1),
           "process_wall_ms": round(proc_ms, 1), "max_kernel_ms": round(kern_ms, 1),
           "setup_phases_ms": {k: round(v, 1) for k, v in zip(SETUP_PHASES, mx[6:])},
           "process_phases_ms": {k: round(v, 1) for k, v in zip(PROCESS_PHASES, mx[6 + len(SETUP_PHASES):])},
           "setup_bound_by": _setup_bound(dict(zip(SETUP_PHASES, mx[6:]))),
           "timing": "wall_ms = the --full-wgs driver's timed region (workers set up -> last results on the "
                     "host), max over ranks; setup_ms = contexts, genome upload and reader buffers before it "
                     "(setup_phases_ms: each phase's max over workers and ranks; hip_init_ms comes before "
                     "setup_ms, reference_load_ms runs on its own thread beside hip_init_ms); "
                     "process_wall_ms = the rank's child process "
                     "start to exit",
           "segments": {"pool": P, "segment_reads": S, "segments_per_file": R // S,
                        "distinct_reads": P * S, "note": "lane files are concatenations of pooled, pre-scored "
                                                         "segments: reads repeat across and within files"},
           "gather": "per-file (score i64, reads, bases) rows all-gathered over the process group",
           "parity": par, "dataset": {k: v for k, v in (args._c4_meta or {}).items() if not k.startswith("_")}}
    if job.gpu and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline_c4(args)
    return out


def cpu_baseline_c4(args):
    """configs_extra.config4.cpu_baseline: the SIMD restatement scoring pool
    segment 0 (its reads against their genome windows, linear, score only)
    on every CPU this job may use, timed here; plus the per-thread rate of
    the pool generation's oracle pass (each segment scored on one thread,
    the workers running side by side).  Scoring only: the CPU inflate and
    parse of the lane files are not in it."""
    from mini_parallel_amd.synthetic import _lane_reads, _with_windows, wgs_genome
    from oracle import oracle_lib
    g = wgs_genome(C4_SEED, C4_GENOME)
    b, pos, _ = _lane_reads(g, 0, args.c4_segment_reads, 150, 2.0, C4_SEED, segment=1)
    w = _with_windows(g, b, pos)
    _, _, usable = host_cpus()
    passes, dt, t0 = 0, 0.0, time.perf_counter()
    while dt < max(1.0, args.cpu_seconds / 4):
        s, _, _, isa = oracle_lib.sw_batch_simd(w.reads, w.read_len, w.wins, w.win_len, threads=usable, coords=False)
        passes += 1
        dt = time.perf_counter() - t0
    meta = args._c4_meta or {}
    seg0 = (meta.get("segments") or [{}])[0]
    thr = meta.get("_segment_rates") or []
    per_thread = (sum(c for c, _ in thr) / sum(t for _, t in thr) / 1e9) if thr else None
    gc = passes * w.cells / dt / 1e9
    return {"value": round(gc, 2), "unit": "GCUPS", "cores": usable, "kind": "port",
            "reads_per_s": round(passes * w.n_pairs / dt),
            "sample": f"{passes} pass(es) of oracle/sw_simd.c ({isa}-bit) over pool segment 0 ({w.n_pairs} reads x "
                      f"300 bp windows, {w.cells} cells, {dt:.1f} s) on {usable} threads",
            "segment0_score_matches_pool": bool(int(s.astype(np.int64).sum()) == seg0.get("score")),
            "pool_pass_per_thread_gcups": None if per_thread is None else round(per_thread, 2),
            "scope": "scoring only (no CPU inflate / parse)"}


def leg_config3_fastq(job, args):
    """configs_extra.config3.fastq -- BASELINE config 3 as stated: 1 M reads
    in BGZF lane files (16 x 62,500), through the product's --full-wgs
    driver with --gap-model affine --scores-out (lane loader -> batches in
    HBM -> affine + best cell -> per-read (score, end_i, end_j) records on
    the host, aligner.rs:107-178, 269-289, 466-475), sharded by file over the
    ranks.  Every record is gathered over the process group and rank 0
    compares all of them with the oracle's."""
    from mini_parallel_amd import dist as mdist
    (bad,) = job.sum([1 if (args._c3f_meta or {}).get("error") else 0])  # only rank 0 generated
    if bad:
        return None if job.rank else {"error": args._c3f_meta["error"], "parity": {"bit_exact": False}}
    d, files, per = c3f_layout(args, job.world)
    F = len(files)
    stats, err, cells, recs, idx = [0.0] * 5, "", 0, [], []
    setup = [0.0] * (len(SETUP_PHASES) + len(PROCESS_PHASES))
    if job.gpu:
        rec, ck, proc, wd, err = run_wgs_child(job, d, job.world, C3F_RPL, os.path.join(d, "reference.fa"),
                                               ["--gap-model", "affine", "--scores-out", "{wd}"], "c3f", 600)
        if not err:
            for fr in sorted(ck["files"], key=lambda x: files.index(x["file_path"])):
                fi = files.index(fr["file_path"])
                raw = np.fromfile(os.path.join(wd, os.path.basename(fr["file_path"]) + ".scores"), np.uint8)
                r = raw.view([("s", "<i4"), ("i", "<i2"), ("j", "<i2")])
                recs.append(np.stack([r["s"].astype(np.int32), r["i"].astype(np.int32), r["j"].astype(np.int32)], 1))
                idx.append([fi, r.shape[0], 1 if fr["completed"] else 0, job.rank, job.dev_index])
            stats = [rec["wall_ms"], proc * 1e3, rec["setup_ms"], rec["teardown_ms"], rec["kernel_ms"]]
            cells = int(rec["cells"])
            setup = _setup_split(rec)
    else:
        job.fence()
        t0 = time.perf_counter()
        for fi in range(job.rank, F, job.world):
            r = _standin_records(files[fi])
            recs.append(r)
            idx.append([fi, r.shape[0], 1, job.rank, -1])
        proc = time.perf_counter() - t0
        job.fence()
        stats = [proc * 1e3] * 2 + [0.0] * 3
        cells = sum(int(r.shape[0]) for r in recs) * C4_WINDOW
    mx = job.max(stats + [stats[2] + stats[0]] + setup)
    tot = job.sum([cells, 1 if err else 0])
    allr = np.concatenate(recs) if recs else np.zeros((0, 3), np.int32)
    t_s, t_i, t_j = (job.tensor(np.ascontiguousarray(allr[:, c])) for c in range(3))
    # int16 coordinates ride the gather's int32 wire cast; the per-file index
    # rows (a different length) are a gather of their own
    g_s, g_i, g_j = job.gather(t_s, t_i.to(dtype=_torch().int16), t_j.to(dtype=_torch().int16))
    (g_idx,) = mdist.gather_results(job.tensor(np.array(idx, np.int64).reshape(-1)))
    if job.rank != 0:
        return None
    if tot[1]:
        return {"error": "the config-3 FASTQ leg failed on some rank (see stderr)", "parity": {"bit_exact": False}}
    g_s, g_i, g_j = g_s.cpu().numpy(), g_i.cpu().numpy(), g_j.cpu().numpy()
    g_idx = g_idx.cpu().numpy().reshape(-1, 5)
    by_rank, dev_by_rank = _files_by_rank(g_idx[:, 0], g_idx[:, 3], g_idx[:, 4], job.world)
    off, order = 0, {}
    for fi, n, done, _, _ in g_idx:
        order[int(fi)] = (off, int(n), int(done))
        off += int(n)
    mism, checked, files_ok = 0, 0, 0
    for fi, p in enumerate(files):
        if fi not in order:
            continue
        o, n, done = order[fi]
        files_ok += done
        if job.gpu:
            z = np.load(p + ".oracle.npz")
            want = np.stack([z["score"], z["end_i"], z["end_j"]], 1).astype(np.int64)
        else:
            want = _standin_records(p).astype(np.int64)
        got = np.stack([g_s[o:o + n], g_i[o:o + n], g_j[o:o + n]], 1).astype(np.int64)
        if got.shape != want.shape:
            mism += max(n, want.shape[0])
        else:
            mism += int((got != want).any(axis=1).sum())
        checked += n
    wall_ms, proc_ms, setup_ms, tear_ms, kern_ms, setup_wall_ms = mx[:6]
    reads = int(g_idx[:, 1].sum()) if g_idx.size else 0
    return {"workload": f"config3 from FASTQ: {F} BGZF lane files x {per} reads of 150 bp = {F * per} reads, "
                        f"{C3F_GENOME >> 20} Mbp HBM-resident genome, window {C4_WINDOW}, affine (open 3, extend 1) "
                        "+ best cell, per-read records (--scores-out)",
            "n_ranks": job.world, "scaling": "weak", "reads": reads, "reads_per_gpu": args.c3_fastq_reads,
            "gcups_end_to_end": round(int(tot[0]) / (wall_ms * 1e6), 1),
            "gcups_incl_setup": round(int(tot[0]) / (setup_wall_ms * 1e6), 1),
            "reads_per_s": round(reads / (wall_ms * 1e-3)),
            "reads_per_s_incl_setup": round(reads / (setup_wall_ms * 1e-3)),
            "wall_ms": round(wall_ms, 1), "setup_ms": round(setup_ms, 1), "process_wall_ms": round(proc_ms, 1),
            "max_kernel_ms": round(kern_ms, 1),
            "teardown_ms": round(tear_ms, 1),
            "setup_phases_ms": {k: round(v, 1) for k, v in zip(SETUP_PHASES, mx[6:])},
            "process_phases_ms": {k: round(v, 1) for k, v in zip(PROCESS_PHASES, mx[6 + len(SETUP_PHASES):])},
            "setup_bound_by": _setup_bound(dict(zip(SETUP_PHASES, mx[6:]))),
            "parity": {"records_checked": checked, "records_expected": F * per, "mismatches": mism,
                       "files_done": files_ok, "files_by_rank": by_rank, "child_device_by_rank": dev_by_rank,
                       "files_sharded_as_cli": by_rank == [list(range(r, F, job.world)) for r in range(job.world)],
                       "bit_exact": mism == 0 and checked == F * per and files_ok == F,
                       "check": "every read's (score, end_i, end_j) against the oracle (oracle/sw_simd.c, "
                                "affine + best cell), records gathered over the process group",
                       **({"standin": True} if not job.gpu else {})},
            "dataset": {k: v for k, v in (args._c3f_meta or {}).items() if not k.startswith("_")}}


class _stdout_to_stderr:
    """File descriptor 1 pointed at 2 for the block (native libraries print
    on fd 1 directly, below sys.stdout)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def _torch():
    import torch
    return torch


# ---------------------------------------------------------------------------
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    extras = [int(x) for x in args.extra_configs.split(",") if x.strip().isdigit()]
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if args.gpus is not None and args.gpus != world:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
            return 2
    else:
        world = args.gpus or 1
        if world > 1:
            if args.cpu_standin or visible_gpus() >= (1 if args.share_gpu else world):
                prepare_datasets(args, extras, world)  # before the ranks start (they reuse it)
            return launch_ranks(args, argv)
    rank = int(os.environ.get("RANK", 0))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    gpu = not args.cpu_standin
    args._c4_meta = args._c3f_meta = None
    if rank == 0:
        # before anything touches the GPU; the other ranks wait in init_process_group
        prepare_datasets(args, extras, world)

    import datetime

    import warnings

    import torch  # first: libmsw.so then binds to the same HIP runtime as torch
    import torch.distributed as dist
    # keep the driver's output tail for the record: barrier() on the current
    # device is what every barrier here means
    warnings.filterwarnings("ignore", message="barrier\\(\\): using the device under current context")

    shared = gpu and args.share_gpu
    dev_index = 0 if shared else local_rank
    if gpu:
        have = int(torch.cuda.device_count())
        local_world = 1 if shared else int(os.environ.get("LOCAL_WORLD_SIZE", world))
        if have < local_world or dev_index >= have:
            print(f"bench.py: rank {rank} needs GPU {dev_index} of {local_world} but only {have} GPU(s) are visible",
                  file=sys.stderr, flush=True)
            return 3
        torch.cuda.set_device(dev_index)
    # A process group at every N, N = 1 included: the gathers, max / sum
    # reductions and barriers of every leg run through RCCL ("nccl") on the
    # GPUs whatever the GPU count (gloo for --cpu-standin and --share-gpu).
    pg_init = "env://" if "WORLD_SIZE" in os.environ else f"tcp://127.0.0.1:{_free_port()}"
    # Build the communicator now, not inside a leg, and keep RCCL's version
    # banner and gloo's connection lines (printed on stdout at communicator
    # creation) off the one-line stdout contract.
    with _stdout_to_stderr():
        dist.init_process_group("nccl" if gpu and not shared else "gloo", init_method=pg_init, rank=rank,
                                world_size=world, timeout=datetime.timedelta(minutes=30))
        from mini_parallel_amd import dist as _md
        _md.sum_over_ranks([0], device=torch.device("cuda", dev_index) if gpu and not shared else None)
    from mini_parallel_amd import dist as mdist
    from mini_parallel_amd.synthetic import config_shard

    cfg = args.config
    scoring = scoring_of(cfg)
    kind = kind_of(scoring)
    per_gpu = args.pairs or DEFAULT_PAIRS[cfg]
    n_total = per_gpu * world
    a, b = mdist.shard_range(n_total, rank, world)
    batch = config_shard(cfg, a, b)
    cells = batch.cells

    ctx = None
    if gpu:
        dev = torch.device("cuda", dev_index)
        from mini_parallel_amd import Context
        ctx = Context(dev_index)
        # A dedicated (non-null) stream: the kernels and the timing events share
        # it; a second one, created beside it (HIP maps streams onto its
        # hardware queues as they are created), for pipelined_steps.
        stream = torch.cuda.Stream(dev)
        stream2 = torch.cuda.Stream(dev)
        torch.cuda.set_stream(stream)
        work = GpuWorkload(ctx, dev, stream, cfg, batch, scoring)
        step = work.step
    else:
        dev = stream = None
        holder = {}

        def step():
            holder["s"] = standin_scores(batch)
    job = Job(rank, world, local_rank, gpu, dev, stream, shared=shared)

    for _ in range(args.warmup):
        step()
    preheat = job.preheat(step)
    job.fence()

    if gpu:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    if gpu:
        ev0.record(stream)
    for _ in range(args.steps):
        step()
    if gpu:
        ev1.record(stream)
    wall_ms = (job.stop() - t0) * 1e3
    kern_ms = ev0.elapsed_time(ev1) if gpu else wall_ms

    wall_ms, kern_ms = job.max([wall_ms, kern_ms])
    # every rank scores its own shard: the job's cells and ranks are sums over ranks
    job_cells, ranks_ran = job.sum([cells, 1])

    # Two batches in flight (an extra figure, not `value`).  Before any
    # all_gather: after one, kernels on the two streams stopped overlapping on
    # the box (tools/pipe_probe.py: 34.7 -> 42.7 us per step).
    pipe = pipelined_steps(job, ctx, cfg, batch, scoring, work, stream2, args) if gpu else None

    # Final score/coordinate gather over RCCL (outside the timed region): the
    # only collective of the path.  Concatenated in rank order = global order.
    if gpu:
        g_score, g_i, g_j = job.gather(work.score, work.ei, work.ej)
    else:
        (g_score,) = mdist.gather_results(torch.from_numpy(holder["s"]))
        g_i = g_j = None

    # The other BASELINE configs, on every rank (each leg fences and gathers).
    extra = {}
    for c in extras:
        if c == cfg:
            continue
        if c in (3, 5):
            extra[f"config{c}"] = leg_pairs(job, ctx, c, args)
            if c == 3 and args.c3_fastq_reads > 0:
                r = leg_config3_fastq(job, args)  # BASELINE config 3 from lane files
                if rank == 0:
                    extra["config3"]["fastq"] = r
        elif c == 4:
            extra["config4"] = leg_config4(job, args)

    if rank == 0:
        g_score = g_score.cpu().numpy()
        g_i = g_i.cpu().numpy() if g_i is not None else None
        g_j = g_j.cpu().numpy() if g_j is not None else None
        value = job_cells * args.steps / (wall_ms * 1e-3) / 1e9
        ms_per_step = wall_ms / args.steps
        avg_launch_s = kern_ms * 1e-3 / args.steps
        alg_bytes = alg_bytes_of(batch, scoring)
        achieved = alg_bytes / avg_launch_s / 1e9
        kernel_gcups = cells / avg_launch_s / 1e9
        # PMC bytes exist only for the workload tools/profile_round.sh profiled
        traffic = load_pmc_traffic(f"config{cfg}:{kind}") if (not args.pairs and gpu) else None

        cpu = parity = pcie = cut = None
        gathered = {"pairs": int(g_score.size), "pairs_expected": n_total,
                    "score_sum": int(g_score.astype(np.int64).sum())}
        if not gpu:
            parity = {"standin": True}
        else:
            if args.cpu_seconds > 0:
                # the CPU baseline on rank 0's shard; parity of the whole
                # gathered batch on a sample from every shard at N > 1
                cpu, parity = cpu_baseline(args, batch, scoring, g_score[:batch.n_pairs],
                                           None if g_i is None else g_i[:batch.n_pairs],
                                           None if g_j is None else g_j[:batch.n_pairs])
                if world > 1:
                    parity = {"rank0_shard": parity,
                              "all_shards": parity_sample(cfg, scoring, n_total, world, g_score, g_i, g_j)}
                    parity["bit_exact"] = parity["rank0_shard"]["bit_exact"] and parity["all_shards"]["bit_exact"]
                    parity["mismatches"] = (parity["rank0_shard"]["mismatches"]
                                            + parity["all_shards"]["mismatches"])
            # PCIe-inclusive rates (never `value`): the same batch from host
            # memory, scores back on the host, rank 0.
            if not args.no_pcie:
                pcie = pcie_rates(ctx, batch, scoring, cells, g_score[:batch.n_pairs])
                cut = cut_roofline(ctx, dev, stream)

        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GCUPS",
            "n_gpus": ranks_ran,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f16",
            "dtype_note": "cells are exact integers held as packed f16 (H * 2^-11, H < 2048; "
                          "DESIGN.md 4.1); the u16 integer path serves non-ACGT windows",
            "data": "synthetic (seeded genome, 1% subs, 0.1% indels, 0.05% N, 10% unrelated reads)",
            "config": {"workload": f"config{cfg}: {per_gpu} pairs/GPU of one global {n_total}-pair batch, "
                                   f"reads {int(batch.read_len.min())}-{int(batch.read_len.max())} bp x windows "
                                   f"{int(batch.win_len.min())}-{int(batch.win_len.max())} bp, "
                                   f"{kind.replace('_', '+')}, HBM-resident",
                       "pairs_per_gpu": per_gpu, "global_pairs": n_total, "cells_per_gpu_step": cells,
                       "cells_per_job_step": job_cells,
                       "parallelism": f"dp{world}", "kernel": f"sw_{kind}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                         "traffic": round(traffic["hbm_bytes_per_launch"]) if traffic else None,
                         "traffic_over_alg": round(traffic["hbm_bytes_per_launch"] / alg_bytes, 3) if traffic else None,
                         "traffic_unit": "bytes per launch (rocprofv3 PMC, profiles/pmc_traffic.json)",
                         "traffic_detail": traffic, "alg_bytes_per_launch": alg_bytes,
                         "avg_launch_ms": round(avg_launch_s * 1e3, 4)},
            "valu": dict(valu_block(kind, kernel_gcups), binding=True),
            "cpu_baseline": cpu,
            "parity": parity,
            "configs_extra": extra or None,
            "pcie_inclusive": pcie,
            "cut_windows_roofline": cut,
            "pipelined_two_streams": pipe,
            "preheat": dict(preheat, note="untimed repeats of the step after the warm-up until the GPU has "
                                          "run it back to back for the time stated: the clock ramps over ~10 ms "
                                          "of load (tools/launch_series.py, DESIGN.md 5)"),
            "gathered_scores": gathered,
            "collectives": {"backend": mdist.backend(), "world": world, "calls_rank0": dict(mdist.CALLS),
                            "note": "every max / sum / gather / barrier of the run goes through this process "
                                    "group (RCCL = the nccl backend on ROCm), at N = 1 too"},
        }
        if shared:
            line["oversubscribed"] = True
            line["oversubscribed_note"] = (f"--share-gpu: {world} ranks on ONE GPU (device 0), collectives over "
                                           "gloo on host tensors -- a functional run of the N > 1 GPU code, "
                                           "never a scaling point")
        if not gpu:
            line["standin"] = True
            line["standin_scores"] = g_score.tolist() if g_score.size <= 100_000 else None
        detail = write_detail(args, world, line)
        print(json.dumps(fit_line(compact_line(line, detail))), flush=True)

    dist.barrier()
    dist.destroy_process_group()
    return 0


def prepare_datasets(args, extras, world):
    """The lane sets of the FASTQ legs (config 4, config 3 from FASTQ), written
    once before any rank touches a GPU.  A failure (e.g. no disk space) is
    kept as the leg's error instead of ending the bench."""
    args._c4_meta = args._c3f_meta = None
    if 4 in extras:
        try:
            args._c4_meta = ensure_c4_dataset(args)
        except (OSError, RuntimeError) as e:
            args._c4_meta = {"error": f"config-4 dataset: {e}"}
    if 3 in extras and args.c3_fastq_reads > 0:
        try:
            args._c3f_meta = ensure_c3f_dataset(args, world)
        except (OSError, RuntimeError) as e:
            args._c3f_meta = {"error": f"config-3 FASTQ dataset: {e}"}
    for m in (args._c4_meta, args._c3f_meta):  # the record keeps the summary, not the per-file tables
        if m and "error" not in m:
            for k in ("expect", "plan", "sizes"):
                m.pop(k, None)
            segs = m.pop("segments", None)
            if segs:
                m["segments"] = [{k: s[k] for k in ("segment", "reads", "score", "bytes")} for s in segs[:4]]
                m["segments_total"] = len(segs)
                m["_segment_rates"] = [(s["cells"], s["oracle_s"]) for s in segs]


# The driver keeps ~9.6 KB of a run's output tail (stdout, then stderr) and
# parses the standard top-level keys of the last line; the line stays under
# LINE_LIMIT bytes so every leg's headline numbers survive in that tail
# ("What's weak" 4).  Everything else goes to the detail file.
LINE_LIMIT = 6000


def write_detail(args, world, full):
    """The full record (every leg's prose, variants, setup phases, dataset
    metadata) as JSON beside the run; returns the path written (relative to
    the repo when inside it) or None if it could not be written."""
    path = args.detail or os.path.join(ROOT, "gpurun_out", f"bench_detail_n{world}.json")
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path + ".tmp", "w") as f:
            json.dump(full, f, indent=1)
        os.replace(path + ".tmp", path)
    except OSError as e:
        print(f"bench.py: detail record not written ({e})", file=sys.stderr, flush=True)
        return None
    ap = os.path.abspath(path)
    return os.path.relpath(ap, ROOT) if ap.startswith(ROOT + os.sep) else ap


def _pick(d, *keys):
    """The keys of d that are present and not None, in order."""
    return {k: d[k] for k in keys if isinstance(d, dict) and d.get(k) is not None}


def _leg_pairs_summary(e):
    """configs_extra.config3 / .config5 (HBM-resident) in one small object."""
    par, cpu, roof, valu = e.get("parity") or {}, e.get("cpu_baseline") or {}, e.get("roofline_hbm") or {}, \
        e.get("valu") or {}
    # distinct pairs checked: the gathered sample lies inside rank 0's CPU sample at N = 1
    checked = max(par.get("checked_pairs", 0), (par.get("rank0_cpu_sample") or {}).get("checked_pairs", 0))
    return {**_pick(e, "job_gcups", "kernel_gcups", "avg_launch_ms", "pairs_per_gpu"),
            "bit_exact": par.get("bit_exact"), "checked": checked or par.get("pairs"),
            **_pick({"cpu_gcups": cpu.get("value"), "valu_frac": valu.get("frac"),
                     "hbm_frac": roof.get("frac"), "traffic_over_alg": roof.get("traffic_over_alg")},
                    "cpu_gcups", "valu_frac", "hbm_frac", "traffic_over_alg")}


def _phases(leg):
    """A FASTQ leg's setup and process phases, whole milliseconds, short keys
    (the phase names without their _ms suffix)."""
    out = {}
    for key, short in (("setup_phases_ms", "setup_phases"), ("process_phases_ms", "process_phases")):
        ph = leg.get(key)
        if ph:
            out[short] = {k[:-3]: round(v) for k, v in ph.items()}
    return out


def summarize_legs(full):
    """The per-leg `summary` of the one-line record: for each BASELINE config
    and host-path leg its rate with unit, whether it was bit-exact and how
    many results were checked, the CPU baseline, the VALU fraction and the
    counter-traffic ratio -- the fields a reader of the driver's tail needs
    (anchor: the reference's run record, tools/benchmark.rs:17-34)."""
    par = full.get("parity") or {}
    cpu = full.get("cpu_baseline") or {}
    roof = full.get("roofline") or {}
    pipe = full.get("pipelined_two_streams") or {}
    s = {"units": {"gcups": "GCUPS", "reads_per_s": "reads/s", "ms": "milliseconds"},
         "c2": {"gcups": full.get("value"), **_pick({"kernel_gcups": (full.get("valu") or {}).get("kernel_gcups"),
                                                     "pipelined_gcups": pipe.get("value")},
                                                    "kernel_gcups", "pipelined_gcups"),
                "bit_exact": par.get("bit_exact"),
                "checked": par.get("checked_pairs") or (par.get("rank0_shard") or {}).get("checked_pairs"),
                **_pick({"cpu_gcups": cpu.get("value"), "valu_frac": (full.get("valu") or {}).get("frac"),
                         "hbm_frac": roof.get("frac"), "traffic_over_alg": roof.get("traffic_over_alg")},
                        "cpu_gcups", "valu_frac", "hbm_frac", "traffic_over_alg")}}
    ex = full.get("configs_extra") or {}
    for c in ("config3", "config5"):
        e = ex.get(c)
        if not e:
            continue
        if "error" in e:
            s[f"c{c[-1]}_hbm"] = {"error": str(e["error"])[:200], "bit_exact": False}
            continue
        s[f"c{c[-1]}_hbm"] = _leg_pairs_summary(e)
        h = e.get("host_to_host")
        if h:
            s["c3_h2h"] = {"gcups": h.get("value"), "best": h.get("best"),
                           "bit_exact": h.get("equal_to_hbm_resident_run"), "checked": h.get("pairs_per_gpu"),
                           "chunk_pairs": h.get("chunk_pairs")}
        f = e.get("fastq")
        if f:
            fp = f.get("parity") or {}
            s["c3_fastq"] = {**_pick(f, "reads_per_s", "gcups_end_to_end", "reads_per_s_incl_setup",
                                     "gcups_incl_setup", "wall_ms", "setup_ms", "teardown_ms", "process_wall_ms",
                                     "error"),
                             **_phases(f),
                             "bit_exact": fp.get("bit_exact"), "checked": fp.get("records_checked"),
                             **_pick({"distinct_reads": (f.get("dataset") or {}).get("distinct_reads")},
                                     "distinct_reads")}
    c4 = ex.get("config4")
    if c4:
        p4 = c4.get("parity") or {}
        s["c4"] = {**_pick(c4, "reads_per_s", "reads_per_s_incl_setup", "reads_per_s_process", "gcups", "reads",
                           "wall_ms", "setup_ms", "teardown_ms", "process_wall_ms", "error"),
                   **_phases(c4),
                   "bit_exact": p4.get("bit_exact"), "checked": p4.get("files_checked"), "checked_unit": "files",
                   **_pick({"cpu_gcups": (c4.get("cpu_baseline") or {}).get("value")}, "cpu_gcups")}
    pc = full.get("pcie_inclusive")
    if pc:
        st = (pc.get("variants") or {}).get("genome_pinned_stream") or {}
        s["pcie"] = {"gcups": pc.get("value"), "best": pc.get("best"),
                     **_pick({"stream_gcups": st.get("gcups"), "submit_us": st.get("submit_us_per_batch")},
                             "stream_gcups", "submit_us"),
                     "bit_exact": True, "checked": (full.get("config") or {}).get("pairs_per_gpu")}
    cut = full.get("cut_windows_roofline")
    if cut:
        s["cut_windows"] = _pick(cut, "achieved", "frac", "avg_launch_ms")
    return s


def compact_line(full, detail_path=None):
    """The one JSON line bench.py prints: the contract's keys, the headline's
    roofline / cpu_baseline / valu / parity without their prose, the per-leg
    summary, and the detail file's path.  The prose and variant tables stay in
    the detail record."""
    cfg = full.get("config") or {}
    roof = full.get("roofline") or {}
    cpu = full.get("cpu_baseline")
    par = full.get("parity") or {}
    line = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data") if k in full}
    line["config"] = _pick(cfg, "workload", "pairs_per_gpu", "global_pairs", "cells_per_gpu_step",
                           "cells_per_job_step", "parallelism", "kernel")
    line["roofline"] = _pick(roof, "bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_over_alg",
                             "alg_bytes_per_launch", "avg_launch_ms")
    line["roofline"].setdefault("traffic", None)
    if cpu:
        c = _pick(cpu, "value", "unit", "cores", "kind", "cpu_model", "isa_bits", "one_thread_gcups",
                  "scalar_oracle_1core_gcups")
        smp = str(cpu.get("sample", ""))
        c["sample"] = smp if len(smp) <= 240 else smp[:237] + "..."
        line["cpu_baseline"] = c
    else:
        line["cpu_baseline"] = None
    line["valu"] = _pick(full.get("valu") or {}, "kernel_gcups", "ceiling_gcups", "frac", "i32_ceiling_gcups",
                         "frac_i32_ceiling", "lone_wave_ceiling_gcups", "frac_lone_wave", "binding")
    line["parity"] = {"bit_exact": par.get("bit_exact"), "mismatches": par.get("mismatches"),
                      "checked_pairs": par.get("checked_pairs")
                      or (par.get("rank0_shard") or {}).get("checked_pairs"),
                      **({"standin": True} if par.get("standin") else {})}
    line["preheat"] = _pick(full.get("preheat") or {}, "steps", "seconds")
    line["summary"] = summarize_legs(full)
    if full.get("gathered_scores"):
        line["gathered_scores"] = full["gathered_scores"]
    col = full.get("collectives")
    if col:
        line["collectives"] = _pick(col, "backend", "world", "calls_rank0")
    line["detail"] = detail_path
    for k in ("standin", "standin_scores", "oversubscribed"):  # --cpu-standin / --share-gpu test runs only
        if k in full:
            line[k] = full[k]
    return line


def fit_line(line):
    """Enforce LINE_LIMIT at run time: if the line is over it,
    drop the optional parts of the summary in turn (phase splits, error
    prose, then the cpu_baseline sample text), never the contract's keys,
    and say so on stderr.  The detail file keeps everything."""
    def size():
        return len(json.dumps(line).encode())
    if size() <= LINE_LIMIT:
        return line
    start, dropped = size(), []
    summ = line.get("summary") or {}
    for key in ("process_phases", "setup_phases"):
        for leg in summ.values():
            if isinstance(leg, dict) and leg.pop(key, None) is not None and f"summary.*.{key}" not in dropped:
                dropped.append(f"summary.*.{key}")
        if size() <= LINE_LIMIT:
            break
    if size() > LINE_LIMIT:
        for leg in summ.values():
            if isinstance(leg, dict) and isinstance(leg.get("error"), str) and len(leg["error"]) > 60:
                leg["error"] = leg["error"][:57] + "..."
                dropped.append("summary.*.error (trimmed)")
    if size() > LINE_LIMIT and isinstance(line.get("cpu_baseline"), dict):
        line["cpu_baseline"]["sample"] = str(line["cpu_baseline"].get("sample", ""))[:60]
        dropped.append("cpu_baseline.sample (trimmed)")
    if size() > LINE_LIMIT:
        for k in [k for k in summ if k not in ("c2", "units")]:
            summ[k] = {kk: summ[k][kk] for kk in ("gcups", "reads_per_s", "bit_exact", "checked")
                       if isinstance(summ[k], dict) and kk in summ[k]}
        dropped.append("summary legs cut to rate + parity")
    print(f"bench.py: the one-line record was {start} B > LINE_LIMIT {LINE_LIMIT}; now {size()} B after "
          f"dropping {', '.join(dict.fromkeys(dropped))} (the detail file keeps them)", file=sys.stderr, flush=True)
    return line


def load_pmc_traffic(key: str):
    """HBM bytes per launch from a committed rocprofv3 --pmc summary, if any."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(key)
    except Exception:
        return None


if __name__ == "__main__":
    sys.exit(main())
