#!/bin/bash
# Host-pipeline sizing: the config-4-shape --full-wgs run on
# one GPU at several MSW_HOST_THREADS, BGZF lane files (8 lanes x 2 files x N
# reads), plus the single-reader rates (tools/reader_bench.py) that the
# 8-GPU prediction in DESIGN.md 5 extrapolates from.
#   bash tools/e2e_threads.sh OUTDIR READS_PER_FILE THREADS_LIST
set -euo pipefail
OUT=${1:-gpurun_out/e2e}; N=${2:-500000}; T=${3:-4,8,16,32,64}
mkdir -p "$OUT"
timeout -k 10 500 python3 -u tools/wgs_e2e.py --dir /tmp/msw_wgs_r02 --reads-per-file "$N" --bgzf \
    --host-threads "$T" --out "$OUT/threads_sweep.jsonl" --workers 16
timeout -k 10 200 python3 -u tools/reader_bench.py --reads "$N" --threads 1,2,4,8,16 > "$OUT/reader_bench.jsonl" 2>&1 || true
