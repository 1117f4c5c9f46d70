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
(the binding VALU-integer ceiling), ``cpu_baseline`` (oracle restatement on the
host cores, bounded sample, rank 0 at N = 1 only), ``parity``, and at N = 1
``configs_extra`` (configs 3 and 5: kernel GCUPS, VALU fraction, parity
sample), ``pcie_inclusive`` and ``cut_windows_roofline``.
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
    ap.add_argument("--extra-configs", default="3,5",
                    help="N = 1 only: other single-GPU configs timed as extra keys ('' or 'none' = none)")
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


def time_extra_config(ctx, dev, stream, cfg, args):
    """configs_extra: one other single-GPU config timed on its own (kernel
    only, HIP events on the launch stream) with a parity sample."""
    import torch
    from mini_parallel_amd.synthetic import config_shard
    from oracle import oracle_lib
    oracle_lib.build()
    scoring = scoring_of(cfg)
    kind = kind_of(scoring)
    t0 = time.perf_counter()
    batch = config_shard(cfg, 0, DEFAULT_PAIRS[cfg])
    gen_s = time.perf_counter() - t0
    w = GpuWorkload(ctx, dev, stream, cfg, batch, scoring)
    reps = 5 if cfg == 3 else 20
    for _ in range(2):
        w.step()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        w.step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    t = e0.elapsed_time(e1) * 1e-3 / reps
    s, i, j = w.results()
    n = 4096
    _, _, usable = host_cpus()
    cs, ci, cj, _ = oracle_lib.sw_batch_simd(batch.reads[:n], batch.read_len[:n], batch.wins[:n],
                                             batch.win_len[:n], threads=usable, coords=scoring.want_coords,
                                             **_oracle_kw(scoring))
    mism = int((cs != s[:n]).sum())
    if scoring.want_coords:
        mism += int(((ci != i[:n]) | (cj != j[:n])).sum())
    gcups = batch.cells / t / 1e9
    ceiling = 128.0 / CYCLES_PER_ROW_STEP[kind] * SIMDS * CLOCK_HZ / 1e9
    alg = alg_bytes_of(batch, scoring)
    del w
    return {"workload": f"config{cfg}: {batch.n_pairs} pairs, reads {int(batch.read_len.min())}-"
                        f"{int(batch.read_len.max())} bp x windows {int(batch.win_len.min())}-"
                        f"{int(batch.win_len.max())} bp, {kind.replace('_', '+')}, HBM-resident"
                        + (", one length-bucketed planned launch" if cfg == 5 else ""),
            "kernel_gcups": round(gcups, 1), "avg_launch_ms": round(t * 1e3, 4), "launches": reps,
            "valu": {"ceiling_gcups": round(ceiling, 1), "frac": round(gcups / ceiling, 4)},
            "roofline_hbm": {"achieved": round(alg / t / 1e9, 2), "frac": round(alg / t / 1e9 / HBM_PEAK_GBPS, 5),
                             "alg_bytes_per_launch": alg},
            "parity": {"checked_pairs": n, "mismatches": mism, "bit_exact": mism == 0},
            "gen_seconds": round(gen_s, 1)}


# ---------------------------------------------------------------------------
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if args.gpus is not None and args.gpus != world:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
            return 2
    else:
        world = args.gpus or 1
        if world > 1:
            return launch_ranks(args, argv)
    rank = int(os.environ.get("RANK", 0))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    gpu = not args.cpu_standin

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
        dist.init_process_group("nccl" if gpu else "gloo", init_method="env://")
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
        sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
    else:
        dev = None
        holder = {}

        def step():
            holder["s"] = standin_scores(batch)
        sync = lambda: None  # noqa: E731

    for _ in range(args.warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()

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
    sync()
    if world > 1:
        dist.barrier()
    sync()
    wall_ms = (time.perf_counter() - t0) * 1e3
    kern_ms = ev0.elapsed_time(ev1) if gpu else wall_ms

    wall_ms, kern_ms = mdist.max_over_ranks([wall_ms, kern_ms], device=dev)
    # every rank scores its own shard: the job's cells and ranks are sums over ranks
    job_cells, ranks_ran = mdist.sum_over_ranks([cells, 1], device=dev)

    # Final score/coordinate gather over RCCL (outside the timed region): the
    # only collective of the path.  Concatenated in rank order = global order.
    if gpu:
        g_score, g_i, g_j = mdist.gather_results(work.score, work.ei, work.ej)
    else:
        s = torch.from_numpy(holder["s"])
        (g_score,) = mdist.gather_results(s)
        g_i = g_j = None

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
        valu_ceiling = 128.0 / CYCLES_PER_ROW_STEP[kind] * SIMDS * CLOCK_HZ / 1e9
        # PMC bytes exist only for the workload tools/profile_round.sh profiled
        traffic = load_pmc_traffic(f"config{cfg}:{kind}") if (not args.pairs and gpu) else None

        cpu = parity = pcie = cut = None
        extra = {}
        gathered = {"pairs": int(g_score.size), "pairs_expected": n_total,
                    "score_sum": int(g_score.astype(np.int64).sum())}
        if not gpu:
            parity = {"standin": True}
        elif world == 1:
            if args.cpu_seconds > 0:
                cpu, parity = cpu_baseline(args, batch, scoring, g_score, g_i, g_j)
            # PCIe-inclusive rates (never `value`): the same batch from host
            # memory, scores back on the host.
            if not args.no_pcie:
                pcie = pcie_rates(ctx, batch, scoring, cells, g_score)
                cut = cut_roofline(ctx, dev, stream)
            for c in [int(x) for x in args.extra_configs.split(",") if x.strip().isdigit()]:
                if c != cfg:
                    extra[f"config{c}"] = time_extra_config(ctx, dev, stream, c, args)
        elif args.cpu_seconds > 0:
            parity = parity_sample(cfg, scoring, n_total, world, g_score, g_i, g_j)

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
            "valu": {"binding": True, "kernel_gcups": round(kernel_gcups, 1),
                     "ceiling_gcups": round(valu_ceiling, 1),
                     "frac": round(kernel_gcups / valu_ceiling, 4),
                     "cycles_per_packed_row_step": CYCLES_PER_ROW_STEP[kind],
                     "basis": "VALU issue bound of the f16 loop's instruction mix at full "
                              "occupancy, 2.4 GHz peak clock (~2.2 GHz sustained, "
                              "tools/wave_trace.py; DESIGN.md 4)"},
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
