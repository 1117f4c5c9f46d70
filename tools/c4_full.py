#!/usr/bin/env python3
"""BASELINE config 4 at its stated size on one GPU, every file checked.

The lane set is bench.py's (ensure_c4_dataset): 8 lanes x R1/R2 BGZF lane
files of 25 M 150 bp reads (400 M reads; the reference's aligner.rs:214 names
51,858,562 reads per file), binned qualities, zlib level 6, 64 Mbp genome,
each file the concatenation of 25 segments from a pool of 32 distinct 1 M-read
segments that the oracle scored once when the pool was generated.  The
product's --full-wgs driver then runs over all 16 files on one GPU with the
GPU lane reader (MSW_GPU_INFLATE=1) and the host reader (=0, libdeflate on
the host CPUs), the GPU reader first and last.  Each run's record goes to
--out as one JSON line, with every file's (score i64, reads, bases) compared
with the sums of its segments' oracle results; a last line summarises.

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

import bench  # noqa: E402  (the bench's dataset builder and constants)


def run_cli(d, files, gpu_inflate, tag, out_dir, cli=None):
    rec_path = os.path.join(out_dir, f"rec_{tag}.json")
    env = dict(os.environ, WGS_DATA_DIR=d, WGS_SAMPLE_ID="SYN", WGS_LANES=str(bench.C4_LANES),
               WGS_READS_PER_LANE=str(bench.C4_READS_PER_LANE), GPU_CHUNK_SIZE_READS="65536",
               MSW_GPU_INFLATE=gpu_inflate, WGS_RUN_ID=f"c4full_{tag}_{os.getpid()}")
    cmd = [cli or os.path.join(ROOT, "mini_parallel_amd", "rustseq_mini"), "--full-wgs", "--gpu", "--score-mode", "sw",
           "--reference", os.path.join(d, "reference.fa"), "--window", str(bench.C4_WINDOW),
           "--checkpoint-dir", "/tmp", "--json", rec_path]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
    proc_s = time.perf_counter() - t0
    if r.returncode != 0:
        raise SystemExit(f"c4_full: {tag} failed rc={r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
    rec = json.load(open(rec_path))
    ck = json.load(open(os.path.join("/tmp", f"checkpoint_{rec['run_id']}.json")))
    expect = json.load(open(os.path.join(d, "DONE.json")))["expect"]
    bad = []
    for fr in ck["files"]:
        e = expect[os.path.basename(fr["file_path"])]
        if (fr["score"], fr["total_reads"], fr["total_bases"]) != (e["score"], e["reads"], e["bases"]) \
                or not fr["completed"]:
            bad.append(os.path.basename(fr["file_path"]))
    keep = ("total_reads", "total_bases", "total_score", "files_processed", "wall_ms", "setup_ms", "setup_phases",
            "teardown_ms", "kernel_ms", "gcups", "gcups_end_to_end", "reads_per_second", "gpu_inflate",
            "inflate_bytes_in", "inflate_bytes_out", "host_cpus_usable", "host_threads", "num_gpus")
    row = {k: rec.get(k) for k in keep}
    row.update({"run": tag, "process_wall_s": round(proc_s, 3),
                "reads_per_second_incl_setup": rec["total_reads"] / ((rec["wall_ms"] + rec["setup_ms"]) / 1e3),
                "reads_per_second_process": rec["total_reads"] / proc_s,
                "files_checked": len(ck["files"]), "files_mismatched": bad,
                "bit_exact": not bad and len(ck["files"]) == len(files)})
    return row


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/tmp/msw_bench_c4", help="bench.py's --c4-dir")
    ap.add_argument("--reads-per-file", type=int, default=bench.C4_READS_PER_FILE)
    ap.add_argument("--segment", type=int, default=bench.C4_SEGMENT_READS)
    ap.add_argument("--pool", type=int, default=bench.C4_POOL)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    out_dir = os.path.dirname(os.path.abspath(a.out))
    os.makedirs(out_dir, exist_ok=True)
    args = bench.parse(["--c4-dir", a.dir, "--c4-reads-per-file", str(a.reads_per_file),
                        "--c4-segment-reads", str(a.segment), "--c4-pool", str(a.pool)])
    m = bench.ensure_c4_dataset(args)
    d, files, _ = bench.c4_layout(args)
    head = {"dataset": d, "files": len(files), "reads_per_file": a.reads_per_file,
            "reads_total": len(files) * a.reads_per_file, "segment": a.segment, "pool": a.pool,
            **{k: m.get(k) for k in ("gen_seconds", "assemble_seconds", "bytes", "reused")}}
    with open(a.out, "w") as f:
        f.write(json.dumps(head) + "\n")
    rows = []
    for tag, gi in (("gpu_reader_1", "1"), ("host_reader", "0"), ("gpu_reader_2", "1")):
        row = run_cli(d, files, gi, tag, out_dir)
        print(f"[c4_full] {tag}: {row['total_reads']} reads, wall {row['wall_ms'] / 1e3:.2f} s "
              f"(+ setup {row['setup_ms'] / 1e3:.2f} s), {row['reads_per_second'] / 1e6:.1f} M reads/s, "
              f"total {row['total_score']}, bit_exact {row['bit_exact']}", flush=True)
        rows.append(row)
        with open(a.out, "a") as f:
            f.write(json.dumps(row) + "\n")
    summ = {"summary": True, "all_bit_exact": all(r["bit_exact"] for r in rows),
            "identical_total": len({r["total_score"] for r in rows}) == 1,
            "all_reads": all(r["total_reads"] == head["reads_total"] for r in rows)}
    with open(a.out, "a") as f:
        f.write(json.dumps(summ) + "\n")
    print(f"[c4_full] {summ}", flush=True)
    return 0 if all(summ.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
