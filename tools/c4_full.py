#!/usr/bin/env python3
"""BASELINE config 4 at its stated size on one GPU.

8 lanes x R1/R2 BGZF lane files x --reads-per-file reads (default 25 M:
400 M 150 bp reads, the config's "8 lanes x ~50 M reads"; the reference's
aligner.rs:214 names 51,858,562 reads per file), binned qualities, zlib level
6, 64 Mbp genome -- the bench's config-4 lane set at full size.  Files are
written in 1 M-read segments by a process pool (bounded memory), then the
product's --full-wgs driver runs over all 16 files on one GPU: the GPU lane
reader (MSW_GPU_INFLATE=1) and the host reader (=0, libdeflate on the host
CPUs), the GPU reader first and last.  Each run's record (wall with and
without setup, setup_ms, teardown_ms, the process wall, kernel time, total
i64 score and reads) goes to --out as one JSON line; a last line states
whether every run reports the same total.

  python3 tools/c4_full.py --out gpurun_out/TAG/config4_full.jsonl
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LANES, RPL, GENOME, WINDOW, LEVEL, QUAL, SEED = 8, 2, 64 << 20, 300, 6, "binned", 1004


def generate(d, reads, segment, workers):
    from multiprocessing import get_context

    from mini_parallel_amd.synthetic import wgs_genome, write_lane_file_segmented
    marker = os.path.join(d, "DONE.json")
    names = ["SYN_L%03d_R%d_001.fastq.gz" % (ln, r) for ln in range(1, LANES + 1) for r in range(1, RPL + 1)]
    try:
        m = json.load(open(marker))
        if all(os.path.getsize(os.path.join(d, n)) == m["sizes"][n] for n in names):
            return m
    except (OSError, ValueError, KeyError):
        pass
    os.makedirs(d, exist_ok=True)
    g = wgs_genome(SEED, GENOME)
    with open(os.path.join(d, "reference.fa"), "w") as f:
        f.write(">synthetic seed=%d\n" % SEED)
        s = g.tobytes().decode()
        f.write("\n".join(s[k:k + 80] for k in range(0, len(s), 80)) + "\n")
    jobs = [(g, os.path.join(d, n), "SYN", k // RPL + 1, k, reads, segment, 150, 2.0, SEED, LEVEL, QUAL)
            for k, n in enumerate(names)]
    t0 = time.perf_counter()
    with get_context("fork").Pool(min(workers, len(jobs))) as pool:
        res = pool.map_async(write_lane_file_segmented, jobs)
        while not res.ready():
            res.wait(30)
            on_disk = sum(os.path.getsize(j[1]) for j in jobs if os.path.exists(j[1]))
            print(f"[c4_full] generating: {on_disk / 1e9:.2f} GB written, {time.perf_counter() - t0:.0f} s",
                  flush=True)
        sizes = res.get()
    m = {"sizes": dict(zip(names, sizes)), "gen_seconds": round(time.perf_counter() - t0, 1),
         "reads_per_file": reads, "segment": segment, "compressed_bytes": int(sum(sizes))}
    json.dump(m, open(marker, "w"))
    return m


def run_cli(d, gpu_inflate, tag, out_dir):
    rec_path = os.path.join(out_dir, f"rec_{tag}.json")
    env = dict(os.environ, WGS_DATA_DIR=d, WGS_SAMPLE_ID="SYN", WGS_LANES=str(LANES),
               WGS_READS_PER_LANE=str(RPL), GPU_CHUNK_SIZE_READS="65536", MSW_GPU_INFLATE=gpu_inflate,
               WGS_RUN_ID=f"c4full_{tag}_{os.getpid()}")
    cmd = [os.path.join(ROOT, "mini_parallel_amd", "rustseq_mini"), "--full-wgs", "--gpu", "--score-mode", "sw",
           "--reference", os.path.join(d, "reference.fa"), "--window", str(WINDOW), "--checkpoint-dir", "/tmp",
           "--json", rec_path]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
    proc_s = time.perf_counter() - t0
    if r.returncode != 0:
        raise SystemExit(f"c4_full: {tag} failed rc={r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
    rec = json.load(open(rec_path))
    keep = ("total_reads", "total_bases", "total_score", "files_processed", "wall_ms", "setup_ms", "teardown_ms",
            "kernel_ms", "gpu_busy_fraction", "gcups", "gcups_end_to_end", "reads_per_second", "gpu_inflate",
            "inflate_bytes_in", "inflate_bytes_out", "host_cpus_usable", "host_threads", "num_gpus")
    row = {k: rec.get(k) for k in keep}
    row.update({"run": tag, "process_wall_s": round(proc_s, 3),
                "reads_per_second_incl_setup": rec["total_reads"] / ((rec["wall_ms"] + rec["setup_ms"]) / 1e3),
                "reads_per_second_process": rec["total_reads"] / proc_s})
    return row


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/tmp/msw_c4_full")
    ap.add_argument("--reads-per-file", type=int, default=25_000_000)
    ap.add_argument("--segment", type=int, default=1_000_000)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    out_dir = os.path.dirname(os.path.abspath(a.out))
    os.makedirs(out_dir, exist_ok=True)
    d = os.path.join(a.dir, f"r{a.reads_per_file}")
    m = generate(d, a.reads_per_file, a.segment, a.workers)
    rows = [{"dataset": d, "files": LANES * RPL, "reads_per_file": a.reads_per_file,
             "reads_total": LANES * RPL * a.reads_per_file, **m, "sizes": None}]
    with open(a.out, "w") as f:
        f.write(json.dumps(rows[0]) + "\n")
    for tag, gi in (("gpu_reader_1", "1"), ("host_reader", "0"), ("gpu_reader_2", "1")):
        row = run_cli(d, gi, tag, out_dir)
        print(f"[c4_full] {tag}: {row['total_reads']} reads, wall {row['wall_ms'] / 1e3:.2f} s "
              f"(+ setup {row['setup_ms'] / 1e3:.2f} s), {row['reads_per_second'] / 1e6:.1f} M reads/s, "
              f"total {row['total_score']}", flush=True)
        rows.append(row)
        with open(a.out, "a") as f:
            f.write(json.dumps(row) + "\n")
    totals = {r["total_score"] for r in rows[1:]}
    summ = {"summary": True, "identical_total": len(totals) == 1,
            "all_reads": all(r["total_reads"] == rows[0]["reads_total"] for r in rows[1:])}
    with open(a.out, "a") as f:
        f.write(json.dumps(summ) + "\n")
    print(f"[c4_full] {summ}", flush=True)
    return 0 if summ["identical_total"] and summ["all_reads"] else 1


if __name__ == "__main__":
    sys.exit(main())
