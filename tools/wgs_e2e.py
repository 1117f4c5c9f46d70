#!/usr/bin/env python3
"""End-to-end --full-wgs measurement (BASELINE config 4 shape, scaled to one
box): writes a synthetic lane dataset (8 lanes x 2 reads-files of 150 bp
FASTQ.gz reads tagged with their reference window, 64 Mbp genome), then runs
the C++ CLI `rustseq_mini --full-wgs --gpu --score-mode sw` over it: FASTQ.gz
inflate + parse into read slabs (reader threads) -> genome-resident windows
cut on the GPU -> batched SW -> per-file i64 score sums.  One JSON line per
run (the CLI's record + reader count) goes to --out.

  python tools/wgs_e2e.py --reads-per-file 1000000 --readers 4,16 --out gpurun_out/wgs_e2e.jsonl
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/tmp/msw_wgs")
    ap.add_argument("--lanes", type=int, default=8)
    ap.add_argument("--reads-per-lane", type=int, default=2)
    ap.add_argument("--reads-per-file", type=int, default=1_000_000)
    ap.add_argument("--genome-bases", type=int, default=64 << 20)
    ap.add_argument("--readers", default="16")
    ap.add_argument("--host-threads", default="",
                    help="comma list of MSW_HOST_THREADS values to sweep (readers then default to it); "
                         "overrides --readers")
    ap.add_argument("--chunk", type=int, default=65536)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--out", default="gpurun_out/wgs_e2e.jsonl")
    ap.add_argument("--extra-env", default="",
                    help="K=V,K=V added to the CLI's environment; several sets separated by ';' run in turn")
    ap.add_argument("--bgzf", action="store_true", help="write block-gzip (bgzip) lane files")
    ap.add_argument("--qual", default="I", choices=["I", "binned", "illumina"], help="quality strings")
    ap.add_argument("--level", type=int, default=1, help="gzip compression level of the lane files")
    ap.add_argument("--num-gpus", type=int, default=1)
    ap.add_argument("--read-len", type=int, default=150, help="read length (window = --window or 2x)")
    ap.add_argument("--cli", default="", help="CLI binary (A/B against another build)")
    ap.add_argument("--window", type=int, default=300)
    ap.add_argument("--reuse", action="store_true", help="keep an existing dataset in --dir")
    args = ap.parse_args()

    from mini_parallel_amd.synthetic import write_wgs_dataset
    t0 = time.time()
    ref = os.path.join(args.dir, "reference.fa")
    if args.reuse and os.path.exists(ref):
        ds = {"reference": ref, "files": [os.path.join(args.dir, "SYN_L%03d_R%d_001.fastq.gz" % (ln, r))
                                          for ln in range(1, args.lanes + 1)
                                          for r in range(1, args.reads_per_lane + 1)]}
    else:
        ds = write_wgs_dataset(args.dir, lanes=args.lanes, reads_per_lane=args.reads_per_lane,
                               reads_per_file=args.reads_per_file, genome_bases=args.genome_bases,
                               keep_batches=False, workers=args.workers, bgzf=args.bgzf, qual=args.qual,
                               compresslevel=args.level, read_len=args.read_len)
    gen_s = time.time() - t0
    gz_bytes = sum(os.path.getsize(f) for f in ds["files"])
    print(f"dataset: {len(ds['files'])} files, {gz_bytes / 1e6:.0f} MB gz, written in {gen_s:.1f} s", flush=True)
    cli = args.cli or os.path.join(ROOT, "mini_parallel_amd", "rustseq_mini")
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    sweep = ([("threads", int(x)) for x in args.host_threads.split(",")] if args.host_threads
             else [("readers", int(x)) for x in args.readers.split(",")])
    sweep = [(kind, n, ee) for ee in args.extra_env.split(";") for kind, n in sweep]
    for vi, (kind, readers, extra_env) in enumerate(sweep):
        rec = os.path.join(args.dir, f"rec_{kind}_{readers}.json")
        env = dict(os.environ, WGS_DATA_DIR=args.dir, WGS_SAMPLE_ID="SYN", WGS_LANES=str(args.lanes),
                   WGS_READS_PER_LANE=str(args.reads_per_lane), GPU_CHUNK_SIZE_READS=str(args.chunk),
                   WGS_RUN_ID=f"e2e_{kind}_{readers}_v{vi}_{int(time.time() * 1000)}")
        if args.read_len > 256:
            env["MSW_MAX_READ_LEN"] = str(args.read_len + 16)  # room for the synthetic indels
        env["MSW_HOST_THREADS"] = str(readers)  # reader threads = host threads (capped at the file count)
        for kv in filter(None, extra_env.split(",")):
            k, v = kv.split("=", 1)
            env[k] = v
        ts = time.time()
        r = subprocess.run([cli, "--full-wgs", "--gpu", "--score-mode", "sw", "--reference", ds["reference"],
                            "--window", str(args.window), "--checkpoint-dir", args.dir, "--json", rec,
                            "--num-gpus", str(args.num_gpus)],
                           env=env, capture_output=True, text=True, timeout=900)
        wall = time.time() - ts
        if r.stderr:
            sys.stderr.write(r.stderr)
        if r.returncode != 0:
            print(r.stdout[-3000:], r.stderr[-3000:])
            raise SystemExit(f"CLI failed with {r.returncode}")
        d = json.load(open(rec))
        d.update({"sweep": kind, kind: readers, "process_wall_s": round(wall, 3), "gz_bytes": gz_bytes,
                  "chunk_reads": args.chunk, "extra_env": extra_env, "bgzf": args.bgzf, "qual": args.qual,
                  "level": args.level,
                  "dataset": f"{args.lanes} lanes x {args.reads_per_lane} files x {args.reads_per_file} "
                             f"{args.read_len} bp reads, {args.genome_bases} bp genome, window {args.window}"})
        print(json.dumps(d), flush=True)
        with open(args.out, "a") as f:
            f.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
