#!/usr/bin/env python3
"""bench.py -- GCUPS of the batched Smith-Waterman scoring path on MI355X.

Workload (BASELINE.json configs[1], "config 2"): 10,000 synthetic 150 bp
reads x 300 bp reference windows, linear gap (+2/-1/-2), score-only, inputs
resident in HBM.  One step = one pass of the hot path (msw_align_batch_device:
the hand-written gfx950 kernel through the C ABI) over the batch.

Multi-GPU: one process per GPU (torch.distributed.run); every rank scores its
own fresh 10k-pair shard (weak scaling, no data-path collective); after the
timed region the scores are gathered to rank 0 over RCCL (the only collective,
as north_star prescribes).  value = cells of all ranks / max-over-ranks time.

Extra fields: ``roofline`` (HBM, as north_star asks; algorithmic bytes per
launch / average launch time from HIP events on the launch stream), ``valu``
(the binding VALU-integer ceiling), ``cpu_baseline`` (the C oracle on the
host cores, bounded sample, rank 0 at N = 1 only), ``parity`` (GPU vs oracle
on that sample; at N > 1 rank 0's first 4096 pairs, untimed) and, at N = 1,
``pcie_inclusive`` / ``cut_windows_roofline``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 5],
                    help="BASELINE config whose batch shape is timed (2 = the metric's)")
    ap.add_argument("--pairs", type=int, default=0, help="override pairs per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target CPU work for the cpu_baseline sample (0 disables)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-pcie", action="store_true", help="skip the host-memory (PCIe) rate")
    return ap.parse_args()


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


def cpu_baseline(args, batch, scoring, gpu_scores, gpu_i, gpu_j):
    """The CPU baseline, timed on this host: the inter-sequence SIMD
    restatement of the oracle (oracle/sw_simd.c, AVX-512BW 32 x int16 lanes /
    AVX2 16, bit-exact with the scalar oracle by tests/test_oracle.py) over a
    bounded sample of the timed pairs sized to ~cpu_seconds, plus the scalar
    oracle on one core for scale.  Parity: GPU vs the SIMD results on the whole
    sample and vs the scalar oracle on its smaller sample."""
    from oracle import oracle_lib
    oracle_lib.build()
    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    kw = dict(match=scoring.match, mismatch=scoring.mismatch, gap_open=scoring.gap_open,
              gap_extend=scoring.gap_extend, affine=scoring.affine)
    coords = scoring.want_coords

    def cells_of(n):
        return int((batch.read_len[:n].astype(np.int64) * batch.win_len[:n]).sum())

    # calibrate on a small sample, then size the sample to ~cpu_seconds
    n0 = min(batch.n_pairs, 256 * threads)
    ts = time.perf_counter()
    oracle_lib.sw_batch_simd(batch.reads[:n0], batch.read_len[:n0], batch.wins[:n0], batch.win_len[:n0],
                             threads=threads, coords=coords, **kw)
    rate = n0 / max(time.perf_counter() - ts, 1e-6)
    ns = int(min(batch.n_pairs, max(n0, rate * args.cpu_seconds)))
    passes = max(1, int(rate * args.cpu_seconds / ns))
    ts = time.perf_counter()
    for _ in range(passes):
        cs, ci, cj, isa = oracle_lib.sw_batch_simd(batch.reads[:ns], batch.read_len[:ns], batch.wins[:ns],
                                                   batch.win_len[:ns], threads=threads, coords=coords, **kw)
    dt = time.perf_counter() - ts
    scells = passes * cells_of(ns)
    # scalar oracle, one core, ~1/5 of the budget
    n1 = max(1, min(ns, int(args.cpu_seconds * 0.2 * 2e8 / max(cells_of(1), 1))))
    ts = time.perf_counter()
    ss, si, sj = oracle_lib.sw_batch(batch.reads[:n1], batch.read_len[:n1], batch.wins[:n1],
                                     batch.win_len[:n1], threads=1, **kw)
    scalar_gcups = cells_of(n1) / max(time.perf_counter() - ts, 1e-9) / 1e9
    cpu = {"value": round(scells / dt / 1e9, 3), "unit": "GCUPS", "cores": threads, "kind": "port",
           "sample": f"{passes} pass(es) over the first {ns} of the {batch.n_pairs} timed pairs "
                     f"({scells} cells, {dt:.1f} s): oracle/sw_simd.c, inter-sequence "
                     f"{'AVX-512BW 32' if isa == 512 else ('AVX2 16' if isa == 256 else 'scalar 1')} "
                     f"x int16 lanes, {threads} threads",
           "cpu_model": oracle_lib.cpu_model(), "isa_bits": isa,
           "scalar_oracle_1core_gcups": round(scalar_gcups, 4)}
    mism = int((cs != gpu_scores[:ns]).sum()) + int((ss != gpu_scores[:n1]).sum())
    if coords:
        mism += int(((ci != gpu_i[:ns]) | (cj != gpu_j[:ns])).sum())
        mism += int(((si != gpu_i[:n1]) | (sj != gpu_j[:n1])).sum())
    parity = {"checked_pairs": ns, "checked_pairs_scalar": n1, "mismatches": mism, "bit_exact": mism == 0}
    return cpu, parity


def parity_sample(batch, scoring, gpu_scores, gpu_i, gpu_j, n=4096):
    """Parity only (N > 1: the CPU baseline is timed at N = 1 alone): rank 0's
    first n pairs against the SIMD restatement, untimed."""
    from oracle import oracle_lib
    oracle_lib.build()
    n = min(n, batch.n_pairs)
    cs, ci, cj, _ = oracle_lib.sw_batch_simd(batch.reads[:n], batch.read_len[:n], batch.wins[:n],
                                             batch.win_len[:n], threads=min(16, os.cpu_count() or 1),
                                             coords=scoring.want_coords, match=scoring.match,
                                             mismatch=scoring.mismatch, gap_open=scoring.gap_open,
                                             gap_extend=scoring.gap_extend, affine=scoring.affine)
    mism = int((cs != gpu_scores[:n]).sum())
    if scoring.want_coords:
        mism += int(((ci != gpu_i[:n]) | (cj != gpu_j[:n])).sum())
    return {"checked_pairs": n, "checked_pairs_scalar": 0, "mismatches": mism, "bit_exact": mism == 0}


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


def main():
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))

    import torch  # first: libmsw.so then binds to the same HIP runtime as torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    from mini_parallel_amd import Context, Scoring
    from mini_parallel_amd.synthetic import config_batch

    cfg = args.config
    scoring = {2: Scoring(), 3: Scoring(gap_open=3, gap_extend=1, affine=True, want_coords=True),
               5: Scoring()}[cfg]
    kind = ("affine" if scoring.affine else "linear") + ("_coords" if scoring.want_coords else "")
    n_pairs = args.pairs or {2: 10_000, 3: 1_000_000, 5: 100_000}[cfg]
    batch = config_batch(cfg, n_pairs=n_pairs, seed_offset=1000 * rank)
    cells = batch.cells

    def to_dev(a, dt=None):
        a = np.ascontiguousarray(a if dt is None else a.view(dt))
        return torch.from_numpy(a).to(dev)

    reads, wins = to_dev(batch.reads), to_dev(batch.wins)
    rlen, wlen = to_dev(batch.read_len, np.int16), to_dev(batch.win_len, np.int16)
    score = torch.zeros(batch.n_pairs, dtype=torch.int32, device=dev)
    ei = torch.zeros(batch.n_pairs, dtype=torch.int16, device=dev)
    ej = torch.zeros(batch.n_pairs, dtype=torch.int16, device=dev)
    max_m, max_n = int(batch.read_len.max()), int(batch.win_len.max())

    ctx = Context(local_rank)
    # A dedicated (non-null) stream: the kernels and the timing events share it.
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    if cfg == 5:
        # Mixed lengths: a length-bucketed plan (msw_plan_create, host-side
        # counting sort of the length arrays + one order upload, made once per
        # batch outside the timed region), then ONE launch per step over all
        # buckets (msw_align_batch_planned).
        step = ctx.prepare_planned_launch(reads.data_ptr(), rlen.data_ptr(), wins.data_ptr(),
                                          wlen.data_ptr(), batch.reads.shape[1], batch.wins.shape[1],
                                          batch.read_len, batch.win_len, score.data_ptr(), scoring,
                                          ei.data_ptr(), ej.data_ptr(), stream.cuda_stream)
    else:
        step = ctx.prepare_device_launch(reads.data_ptr(), rlen.data_ptr(), wins.data_ptr(),
                                         wlen.data_ptr(), batch.reads.shape[1], batch.wins.shape[1],
                                         batch.n_pairs, score.data_ptr(), max_m, max_n, scoring,
                                         ei.data_ptr(), ej.data_ptr(), stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall_ms = (time.perf_counter() - t0) * 1e3
    kern_ms = ev0.elapsed_time(ev1)

    from mini_parallel_amd import dist as mdist
    wall_ms, kern_ms = mdist.max_over_ranks([wall_ms, kern_ms], device=dev)
    # every rank scores its own shard: the job's cells are the sum over ranks
    job_cells = mdist.sum_over_ranks([cells], device=dev)[0]

    # Final score/coordinate gather over RCCL (outside the timed region): the
    # only collective of the path.
    g_score, g_i, g_j = mdist.gather_results(score, ei, ej)
    gathered = {"pairs": int(g_score.numel()),
                "score_sum": int(g_score.to(torch.int64).sum().item())}

    if rank == 0:
        gpu_scores = score.cpu().numpy()
        gpu_i, gpu_j = ei.cpu().numpy(), ej.cpu().numpy()
        value = job_cells * args.steps / (wall_ms * 1e-3) / 1e9
        ms_per_step = wall_ms / args.steps
        avg_launch_s = kern_ms * 1e-3 / args.steps
        alg_bytes = int(batch.read_len.astype(np.int64).sum() + batch.win_len.astype(np.int64).sum()
                        + batch.n_pairs * (8 if scoring.want_coords else 4))
        achieved = alg_bytes / avg_launch_s / 1e9
        kernel_gcups = cells / avg_launch_s / 1e9
        valu_ceiling = 128.0 / CYCLES_PER_ROW_STEP[kind] * SIMDS * CLOCK_HZ / 1e9
        # PMC bytes exist only for the workload tools/profile_round.sh profiled
        traffic = load_pmc_traffic(f"config{cfg}:{kind}") if not args.pairs else None

        cpu = None
        parity = None
        if args.cpu_seconds > 0 and world == 1:
            cpu, parity = cpu_baseline(args, batch, scoring, gpu_scores, gpu_i, gpu_j)
        elif args.cpu_seconds > 0:
            parity = parity_sample(batch, scoring, gpu_scores, gpu_i, gpu_j)

        # PCIe-inclusive rates (never `value`): the same batch from host memory,
        # scores back on the host, best of 3 calls per variant:
        #  pairs_pageable  msw_align_batch, numpy arrays (staged through pinned slabs)
        #  pairs_pinned    msw_align_batch, msw_host_alloc arrays (direct DMA)
        #  genome_*        msw_align_reads: reads + window positions only; the
        #                  windows are cut on the GPU from an HBM-resident genome
        #                  (here: the batch's windows laid end to end, so the
        #                  cells and scores are the same pairs')
        # each with the default chunking and with 4 chunks (copy/kernel overlap).
        pcie = cut = None
        if not args.no_pcie and world == 1:
            pcie = pcie_rates(ctx, batch, scoring, cells, gpu_scores)
            cut = cut_roofline(ctx, dev, stream)

        line = {
            "metric": "GCUPS (billion cell updates/s) on 150bp reads, 1/2/4/8 MI355X; bit-exact scores",
            "value": round(value, 2),
            "unit": "GCUPS",
            "n_gpus": world,
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
            "config": {"workload": f"config{cfg}: {batch.n_pairs} pairs/GPU, reads {int(batch.read_len.min())}-"
                                   f"{max_m} bp x windows {int(batch.win_len.min())}-{max_n} bp, "
                                   f"{kind.replace('_', '+')}, HBM-resident",
                       "pairs_per_gpu": batch.n_pairs, "cells_per_gpu_step": cells,
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
            "pcie_inclusive": pcie,
            "cut_windows_roofline": cut,
            "gathered_scores": gathered,
        }
        print(json.dumps(line), flush=True)

    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
