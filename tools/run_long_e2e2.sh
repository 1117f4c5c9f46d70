#!/bin/bash
# 300 bp reads (window 600) end to end with the GPU lane reader, two runs.
set -euo pipefail
OUT=gpurun_out/long_e2e2
mkdir -p $OUT
export TMPDIR=/tmp
A="--dir /tmp/msw_long_e2e --reads-per-file 1000000 --read-len 300 --window 600 --bgzf --qual binned --level 6 --workers 16 --host-threads 16 --extra-env MSW_GPU_INFLATE=1"
timeout -k 10 600 python3 tools/wgs_e2e.py $A --out $OUT/a.jsonl > $OUT/a.log 2>&1
echo "a $(grep -o '"throughput_reads_per_second": [0-9.]*' $OUT/a.jsonl)"
timeout -k 10 300 python3 tools/wgs_e2e.py $A --reuse --out $OUT/b.jsonl > $OUT/b.log 2>&1
echo "b $(grep -o '"throughput_reads_per_second": [0-9.]*' $OUT/b.jsonl)"
