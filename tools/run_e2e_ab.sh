#!/bin/bash
# Config-4-shape end to end, this tree's CLI against an older build in
# _ab_old/ (same dataset, same box, alternating runs).
set -euo pipefail
OUT=gpurun_out/e2e_ab
mkdir -p $OUT
export TMPDIR=/tmp
D=/tmp/msw_gz_e2e
A="--dir $D --reads-per-file 2000000 --bgzf --qual binned --level 6 --workers 16 --host-threads 16 --extra-env MSW_GPU_INFLATE=1"
timeout -k 10 400 python3 tools/wgs_e2e.py $A --out $OUT/new1.jsonl > $OUT/new1.log 2>&1
for r in old1 new2 old2; do
  case $r in old*) C="--cli _ab_old/rustseq_mini";; *) C="";; esac
  timeout -k 10 200 python3 tools/wgs_e2e.py $A --reuse $C --out $OUT/$r.jsonl > $OUT/$r.log 2>&1
  echo "$r $(grep -o '"throughput_reads_per_second": [0-9.]*' $OUT/$r.jsonl)"
done
