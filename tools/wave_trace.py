#!/usr/bin/env python3
"""Per-wave placement and timing of one scoring launch (diagnostics).

Runs a config batch through msw_align_batch_device with MSW_WAVE_TRACE set, so
every block records its start/end (100 MHz constant clock), shader-clock
cycles, HW_ID/XCC_ID and which substitution path it took; then summarises the
launch: waves per SIMD, wave durations per layout, effective clock, and the
makespan vs the mean per-SIMD busy time (how much the tail costs).

Usage: python tools/wave_trace.py [--config 2] [--pairs 10000] [--layout auto]
                                   [--affine] [--coords] [--dump file.json]
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LAYOUTS = {0: "pairs", 1: "split", 2: "mixed"}


def decode(path):
    raw = np.fromfile(path, dtype=np.uint64)
    recs, k = [], 0
    while k < raw.size:
        n, lay = int(raw[k]), int(raw[k + 1])
        blk = raw[k + 2:k + 2 + 4 * n].reshape(n, 4)
        recs.append((lay & 0xFF, (lay >> 8) & 0xFF, lay >> 16, blk))
        k += 2 + 4 * n
    return recs


def summarise(blk):
    used = blk[blk[:, 1] != 0]
    t0, t1, info, w3 = (used[:, i].astype(np.int64) for i in range(4))
    cyc = w3 & ((1 << 40) - 1)
    pro_us = (w3 >> 40) / 100.0  # staging before the DP loop
    hw = info & 0xFFFFFFFF
    xcc = (info >> 32) & 0xFF
    fast = (info >> 40) & 1
    split = (info >> 41) & 1
    kr = (info >> 48) & 0xFF
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    base = t0.min()
    dur_us = (t1 - t0) / 100.0  # 100 MHz
    out = {
        "waves": int(used.shape[0]),
        "makespan_us": round((t1.max() - base) / 100.0, 2),
        "last_start_us": round((t0.max() - base) / 100.0, 2),
        "fast_path_frac": round(float(fast.mean()), 4),
        "eff_clock_ghz": round(float((cyc / np.maximum(t1 - t0, 1) * 100e6).mean() / 1e9), 3),
        "simds_used": int(np.unique(key).size),
        "cus_used": int(np.unique(key // 4).size),
        "prologue_us": {"p50": round(float(np.median(pro_us)), 2), "max": round(float(pro_us.max()), 2)},
    }
    for sp in (0, 1):
        m = split == sp
        if m.any():
            d = dur_us[m]
            out["split" if sp else "pairs"] = {
                "waves": int(m.sum()), "kr": int(kr[m][0]),
                "dur_us_min": round(float(d.min()), 2), "dur_us_p50": round(float(np.median(d)), 2),
                "dur_us_max": round(float(d.max()), 2)}
    per = collections.Counter(key.tolist())
    hist = collections.Counter(per.values())
    out["waves_per_simd_hist"] = {int(k): int(v) for k, v in sorted(hist.items())}
    busy = collections.defaultdict(float)
    ends = collections.defaultdict(float)
    for k_, a, b in zip(key.tolist(), t0.tolist(), t1.tolist()):
        busy[k_] = max(busy[k_], (b - base) / 100.0)
    spans = np.array(list(busy.values()))
    out["simd_finish_us"] = {"p10": round(float(np.percentile(spans, 10)), 2),
                             "p50": round(float(np.percentile(spans, 50)), 2),
                             "p90": round(float(np.percentile(spans, 90)), 2),
                             "max": round(float(spans.max()), 2)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=10000)
    ap.add_argument("--layout", default="auto")
    ap.add_argument("--group-lanes", type=int, default=0)
    ap.add_argument("--affine", action="store_true")
    ap.add_argument("--coords", action="store_true")
    ap.add_argument("--dump", default="")
    args = ap.parse_args()

    import torch
    from mini_parallel_amd import Context, Scoring
    from mini_parallel_amd.synthetic import config_batch

    if args.layout != "auto":
        os.environ["MSW_LAYOUT"] = args.layout
    if args.group_lanes:
        os.environ["MSW_GROUP_LANES"] = str(args.group_lanes)
    b = config_batch(args.config, n_pairs=args.pairs)
    dev = torch.device("cuda", 0)
    reads = torch.from_numpy(b.reads).to(dev)
    wins = torch.from_numpy(b.wins).to(dev)
    rl = torch.from_numpy(b.read_len.view(np.int16)).to(dev)
    wl = torch.from_numpy(b.win_len.view(np.int16)).to(dev)
    score = torch.zeros(b.n_pairs, dtype=torch.int32, device=dev)
    ei = torch.zeros(b.n_pairs, dtype=torch.int16, device=dev)
    ej = torch.zeros(b.n_pairs, dtype=torch.int16, device=dev)
    sc = Scoring(gap_open=3 if args.affine else 0, gap_extend=1 if args.affine else 2,
                 affine=args.affine, want_coords=args.coords)
    ctx = Context(0)
    stream = torch.cuda.Stream(dev)
    step = ctx.prepare_device_launch(reads.data_ptr(), rl.data_ptr(), wins.data_ptr(), wl.data_ptr(),
                                     b.reads.shape[1], b.wins.shape[1], b.n_pairs, score.data_ptr(),
                                     int(b.read_len.max()), int(b.win_len.max()), sc,
                                     ei.data_ptr(), ej.data_ptr(), stream.cuda_stream)
    for _ in range(5):
        step()  # warm (untraced)
    torch.cuda.synchronize()
    fd, path = tempfile.mkstemp(suffix=".trace")
    os.close(fd)
    os.environ["MSW_WAVE_TRACE"] = path
    for _ in range(3):
        step()
    os.environ.pop("MSW_WAVE_TRACE")
    recs = decode(path)
    os.unlink(path)
    res = []
    for lay, g, pb, blk in recs:
        s = summarise(blk)
        s.update({"layout": LAYOUTS.get(lay, lay), "group_lanes": g, "pairs_blocks": pb, "pairs": b.n_pairs})
        res.append(s)
        print(json.dumps(s), flush=True)
    if args.dump:
        np.save(args.dump, recs[-1][3])


if __name__ == "__main__":
    main()
