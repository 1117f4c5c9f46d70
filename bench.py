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

# config-4 leg: 8 lanes x R1/R2 BGZF lane files (aligner.rs:198-204 naming)
C4_LANES, C4_READS_PER_LANE, C4_READS_PER_FILE = 8, 2, 2_000_000
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
    ap.add_argument("--c4-dir", default="/tmp/msw_bench_c4",
                    help="config-4 leg: where the lane files are generated (reused across runs)")
    ap.add_argument("--no-h2h", action="store_true", help="config-3 leg: skip the host-to-host rate")
    ap.add_argument("--cpu-standin", action="store_true",
                    help="TEST ONLY (tests/test_bench_launcher.py): gloo ranks on the CPU with a "
                         "stand-in scorer, to exercise the launcher, sharding and gather without a GPU")
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
        if have < n:
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


def cpu_baseline(args, batch, scoring, gpu_scores, gpu_i, gpu_j):
    """The CPU baseline, timed on this host: the inter-sequence SIMD
    restatement of the oracle (oracle/sw_simd.c, AVX-512BW 32 x int16 lanes /
    AVX2 16, bit-exact with the scalar oracle by tests/test_oracle.py) over a
    bounded sample of the timed pairs sized to ~cpu_seconds, on every CPU the
    process may use (the affinity mask capped by the cgroup CPU quota), plus
    the scalar oracle on one core.  Parity: GPU vs the SIMD results on the
    whole sample and vs the scalar oracle on its smaller sample."""
    from oracle import oracle_lib
    oracle_lib.build()
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
    ns = int(min(batch.n_pairs, max(n0, rate * args.cpu_seconds)))
    passes = max(1, int(rate * args.cpu_seconds / ns))
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
    n1 = max(1, min(ns, int(args.cpu_seconds * 0.2 * 2e8 / max(cells_of(1), 1))))
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
    # driver feeds chunks: the steady-state host-to-host rate.
    reps, depth = 24, 3
    arrs = variants["genome_pinned"][1]
    for _ in range(2):
        ts = time.perf_counter()
        pend = []
        for _ in range(reps):
            pend.append(ctx.align_reads(genome, *arrs, scoring=scoring, asynchronous=True))
            if len(pend) == depth:
                pend.pop(0).wait()
        while pend:
            s_last = pend.pop(0).wait()[0]
        dt = (time.perf_counter() - ts) / reps
    if not np.array_equal(s_last, gpu_scores):
        raise SystemExit("pcie streaming variant disagrees with the device-resident scores")
    out["genome_pinned_stream"] = {"gcups": round(cells / dt / 1e9, 2), "ms_per_batch": round(dt * 1e3, 3)}
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
    ranks.  gpu=False is --cpu-standin (gloo, CPU tensors)."""

    def __init__(self, rank, world, local_rank, gpu, dev=None, stream=None):
        self.rank, self.world, self.local_rank, self.gpu = rank, world, local_rank, gpu
        self.dev, self.stream = dev, stream

    def sync(self):
        if self.gpu:
            import torch
            torch.cuda.synchronize(self.dev)

    def fence(self):
        self.sync()
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier()
        self.sync()

    def max(self, vals):
        from mini_parallel_amd import dist as mdist
        return mdist.max_over_ranks(vals, device=self.dev)

    def sum(self, vals):
        from mini_parallel_amd import dist as mdist
        return mdist.sum_over_ranks(vals, device=self.dev)

    def tensor(self, a):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(a))
        return t.to(self.dev) if self.gpu else t


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
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        job.fence()
        t0 = time.perf_counter()
        e0.record(job.stream)
        for _ in range(reps):
            w.step()
        e1.record(job.stream)
        job.fence()
        wall = time.perf_counter() - t0
        kern = e0.elapsed_time(e1) * 1e-3 / reps
        outs = [w.score] + ([w.ei, w.ej] if scoring.want_coords else [])
    else:
        job.fence()
        t0 = time.perf_counter()
        for _ in range(reps):
            s = standin_scores(batch)
        job.fence()
        wall = time.perf_counter() - t0
        kern = wall / reps
        outs = [torch.from_numpy(s)]
    wall_max, kern_max = job.max([wall, kern])
    (job_cells,) = job.sum([batch.cells])
    gathered = mdist.gather_results(*outs)
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
    kernel_gcups = batch.cells / kern / 1e9
    alg = alg_bytes_of(batch, scoring)
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
                             "alg_bytes_per_launch": alg},
            "parity": par, "gathered_pairs": int(g[0].size), "host_to_host": h2h,
            "gen_seconds": round(gen_s, 1)}


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
            job.fence()
            best = min(best, time.perf_counter() - t0)
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
# config-4 leg: the --full-wgs stream over BGZF lane files
# ---------------------------------------------------------------------------
def c4_layout(args):
    R = args.c4_reads_per_file
    d = os.path.join(args.c4_dir, f"l{C4_LANES}x{C4_READS_PER_LANE}_r{R}_g{C4_GENOME}_z{C4_LEVEL}{C4_QUAL}_s{C4_SEED}")
    files = [os.path.join(d, "SYN_L%03d_R%d_001.fastq.gz" % (ln, r))
             for ln in range(1, C4_LANES + 1) for r in range(1, C4_READS_PER_LANE + 1)]
    return d, files


def ensure_c4_dataset(args) -> dict:
    """Write the config-4 lane set once (before any rank touches a GPU;
    reused while its DONE.json matches the files on disk)."""
    from mini_parallel_amd.synthetic import write_wgs_dataset
    d, files = c4_layout(args)
    marker = os.path.join(d, "DONE.json")
    try:
        with open(marker) as f:
            m = json.load(f)
        if all(os.path.getsize(p) == m["sizes"][os.path.basename(p)] for p in files):
            return m
    except (OSError, ValueError, KeyError):
        pass
    import shutil
    shutil.rmtree(d, ignore_errors=True)
    t0 = time.perf_counter()
    write_wgs_dataset(d, sample="SYN", lanes=C4_LANES, reads_per_lane=C4_READS_PER_LANE,
                      reads_per_file=args.c4_reads_per_file, genome_bases=C4_GENOME, keep_batches=False,
                      workers=host_cpus()[2], bgzf=True, qual=C4_QUAL, compresslevel=C4_LEVEL, seed=C4_SEED)
    m = {"sizes": {os.path.basename(p): os.path.getsize(p) for p in files},
         "gen_seconds": round(time.perf_counter() - t0, 1)}
    with open(marker + ".tmp", "w") as f:
        json.dump(m, f)
    os.replace(marker + ".tmp", marker)
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


def leg_config4(job, args):
    """configs_extra.config4 -- a bounded BASELINE config 4: the 8 lanes x
    R1/R2 BGZF lane files of ensure_c4_dataset (the full config is 8 x ~50 M
    reads; this one is 16 files x --c4-reads-per-file), sharded by file over
    the ranks (rank r: files r, r + N, ...; strong scaling: the dataset is
    fixed).  Each rank runs the product's --full-wgs driver on its GPU
    (rustseq_mini, WGS_FILE_SHARD=r/N, MSW_DEVICES=local rank: the GPU lane
    reader inflates and parses on the GPU, windows cut from the resident
    genome, score-only kernel, two workers per GPU), as a child process
    started after the fence.  Per-file (score i64, reads, bases) rows are
    all-gathered over RCCL; rank 0 checks every file finished, the read
    count, and file 0's i64 score sum against the oracle."""
    from mini_parallel_amd import dist as mdist
    d, files = c4_layout(args)
    F, R = len(files), args.c4_reads_per_file
    mine = list(range(job.rank, F, job.world))
    rows, stats, err, cells = [], [0.0, 0.0, 0.0, 0.0, 0.0], "", 0
    if job.gpu:
        import tempfile
        cli = os.path.join(ROOT, "mini_parallel_amd", "rustseq_mini")
        wd = tempfile.mkdtemp(prefix=f"msw_c4_r{job.rank}_")
        env = dict(os.environ, WGS_DATA_DIR=d, WGS_SAMPLE_ID="SYN", WGS_LANES=str(C4_LANES),
                   WGS_READS_PER_LANE=str(C4_READS_PER_LANE), GPU_CHUNK_SIZE_READS="65536",
                   WGS_FILE_SHARD=f"{job.rank}/{job.world}", MSW_DEVICES=str(job.local_rank),
                   WGS_RUN_ID=f"bench_c4_r{job.rank}_{os.getpid()}")
        rec_path = os.path.join(wd, "rec.json")
        cmd = [cli, "--full-wgs", "--gpu", "--score-mode", "sw", "--reference", os.path.join(d, "reference.fa"),
               "--window", str(C4_WINDOW), "--checkpoint-dir", wd, "--json", rec_path, "--num-gpus", "1"]
        job.fence()
        t0 = time.perf_counter()
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
        proc = time.perf_counter() - t0
        job.fence()
        if r.returncode != 0:
            err = (r.stdout[-1500:] + r.stderr[-1500:]).strip()
        else:
            with open(rec_path) as f:
                rec = json.load(f)
            with open(os.path.join(wd, f"checkpoint_{rec['run_id']}.json")) as f:
                ck = json.load(f)
            for fr in ck["files"]:
                rows.append([files.index(fr["file_path"]), fr["score"], fr["total_reads"], fr["total_bases"],
                             1 if fr["completed"] else 0])
            stats = [rec["wall_ms"], proc * 1e3, rec["setup_ms"], rec["teardown_ms"], rec["kernel_ms"]]
            cells = int(rec["cells"])
    else:
        job.fence()
        t0 = time.perf_counter()
        for fi in mine:
            rows.append([fi, *_standin_file(files[fi]), 1])
        proc = time.perf_counter() - t0
        job.fence()
        stats = [proc * 1e3, proc * 1e3, 0.0, 0.0, 0.0]
        cells = sum(rw[3] for rw in rows) * C4_WINDOW
    if err:
        print(f"bench.py rank {job.rank}: config-4 leg failed:\n{err}", file=sys.stderr, flush=True)
    mx = job.max(stats + [stats[2] + stats[0]])
    tot = job.sum([cells, 1 if err else 0])
    flat = np.array(rows, np.int64).reshape(-1)
    (g,) = mdist.gather_results(job.tensor(flat))
    if job.rank != 0:
        return None
    g = g.cpu().numpy().reshape(-1, 5)
    if tot[1]:
        raise SystemExit("bench.py: the config-4 leg failed on some rank (see stderr)")
    table = np.zeros((F, 4), np.int64)
    seen = np.zeros(F, np.int64)
    for fi, sc, nr, nb, done in g:
        table[fi] = (sc, nr, nb, done)
        seen[fi] += 1
    reads = int(table[:, 1].sum())
    par = {"files": F, "files_once": bool((seen == 1).all()), "files_done": int(table[:, 3].sum()),
           "reads": reads, "reads_expected": F * R}
    if job.gpu:
        from mini_parallel_amd.synthetic import lane_file_batch
        from oracle import oracle_lib
        b = lane_file_batch(0, R, read_len=150, seed=C4_SEED, genome_bases=C4_GENOME)
        s, _, _, _ = oracle_lib.sw_batch_simd(b.reads, b.read_len, b.wins, b.win_len, threads=host_cpus()[2],
                                              coords=False)
        par.update({"checked_file": os.path.basename(files[0]), "oracle_score": int(s.astype(np.int64).sum()),
                    "gpu_score": int(table[0, 0])})
        par["bit_exact"] = (par["oracle_score"] == par["gpu_score"] and par["files_once"]
                            and par["files_done"] == F and reads == F * R)
    else:
        want = _standin_file(files[0])
        par.update({"standin": True, "file0_ok": bool(tuple(table[0, :3]) == want)})
    wall_ms, proc_ms, setup_ms, tear_ms, kern_ms, setup_wall_ms = mx
    job_cells = int(tot[0])
    return {"workload": f"config4 (bounded): {C4_LANES} lanes x {C4_READS_PER_LANE} BGZF lane files x {R} "
                        f"reads of 150 bp (zlib level {C4_LEVEL}, {C4_QUAL} qualities), {C4_GENOME >> 20} Mbp "
                        f"HBM-resident genome, window {C4_WINDOW}, linear score sums per file; the full config "
                        "is 8 x ~50 M reads",
            "n_ranks": job.world, "scaling": "strong", "files_per_rank": len(mine), "reads": reads,
            "gcups": round(job_cells / (wall_ms * 1e6), 1),
            "reads_per_s": round(reads / (wall_ms * 1e-3)),
            "reads_per_s_incl_setup": round(reads / (setup_wall_ms * 1e-3)),
            "reads_per_s_process": round(reads / (proc_ms * 1e-3)),
            "wall_ms": round(wall_ms, 1), "setup_ms": round(setup_ms, 1), "teardown_ms": round(tear_ms, 1),
            "process_wall_ms": round(proc_ms, 1), "max_kernel_ms": round(kern_ms, 1),
            "timing": "wall_ms = the --full-wgs driver's timed region (workers set up -> last results on the "
                      "host), max over ranks; setup_ms = contexts, genome upload and reader buffers before it; "
                      "process_wall_ms = the rank's child process start to exit (HIP init, setup, teardown)",
            "gather": "per-file (score i64, reads, bases) rows all-gathered over RCCL",
            "parity": par, "dataset_gen_seconds": args._c4_gen_seconds}


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
            if 4 in extras and (args.cpu_standin or visible_gpus() >= world):
                ensure_c4_dataset(args)  # before the ranks start
            return launch_ranks(args, argv)
    rank = int(os.environ.get("RANK", 0))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    gpu = not args.cpu_standin
    args._c4_gen_seconds = None
    if 4 in extras and rank == 0:
        # before anything touches the GPU; the other ranks wait in init_process_group
        args._c4_gen_seconds = ensure_c4_dataset(args).get("gen_seconds")

    import datetime

    import torch  # first: libmsw.so then binds to the same HIP runtime as torch
    import torch.distributed as dist

    if gpu:
        have = int(torch.cuda.device_count())
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        if have < local_world or local_rank >= have:
            print(f"bench.py: rank {rank} needs GPU {local_rank} of {local_world} but only {have} GPU(s) are visible",
                  file=sys.stderr, flush=True)
            return 3
    if world > 1:
        dist.init_process_group("nccl" if gpu else "gloo", init_method="env://",
                                timeout=datetime.timedelta(minutes=30))
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
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
        from mini_parallel_amd import Context
        ctx = Context(local_rank)
        # A dedicated (non-null) stream: the kernels and the timing events share it.
        stream = torch.cuda.Stream(dev)
        torch.cuda.set_stream(stream)
        work = GpuWorkload(ctx, dev, stream, cfg, batch, scoring)
        step = work.step
    else:
        dev = stream = None
        holder = {}

        def step():
            holder["s"] = standin_scores(batch)
    job = Job(rank, world, local_rank, gpu, dev, stream)

    for _ in range(args.warmup):
        step()
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
    job.fence()
    wall_ms = (time.perf_counter() - t0) * 1e3
    kern_ms = ev0.elapsed_time(ev1) if gpu else wall_ms

    wall_ms, kern_ms = job.max([wall_ms, kern_ms])
    # every rank scores its own shard: the job's cells and ranks are sums over ranks
    job_cells, ranks_ran = job.sum([cells, 1])

    # Final score/coordinate gather over RCCL (outside the timed region): the
    # only collective of the path.  Concatenated in rank order = global order.
    if gpu:
        g_score, g_i, g_j = mdist.gather_results(work.score, work.ei, work.ej)
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
                         "traffic_unit": "bytes per launch (rocprofv3 PMC, profiles/pmc_traffic.json)",
                         "traffic_detail": traffic, "alg_bytes_per_launch": alg_bytes,
                         "avg_launch_ms": round(avg_launch_s * 1e3, 4)},
            "valu": dict(valu_block(kind, kernel_gcups), binding=True),
            "cpu_baseline": cpu,
            "parity": parity,
            "configs_extra": extra or None,
            "pcie_inclusive": pcie,
            "cut_windows_roofline": cut,
            "gathered_scores": gathered,
        }
        if not gpu:
            line["standin"] = True
            line["standin_scores"] = g_score.tolist() if g_score.size <= 100_000 else None
        print(json.dumps(line), flush=True)

    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


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
