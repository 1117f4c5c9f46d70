#!/bin/bash
# Round 5: GPU-reader workers per GPU (MSW_GFASTQ_WORKERS_PER_GPU) for config 3
# from FASTQ (2 lane files) and config 4 (16), alternating.
#   bash tools/r05_workers.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/c3f_env_ab.py --out "$OUT/c3f_workers.jsonl" --reps 4 \
  --setting w2= --setting w1=MSW_GFASTQ_WORKERS_PER_GPU=1 > "$OUT/c3f_workers.log" 2>&1
timeout -k 10 500 python3 -u tools/c4_env_ab.py --b MSW_GFASTQ_WORKERS_PER_GPU=1 --reps 2 --out "$OUT/c4_workers.jsonl" \
  > "$OUT/c4_workers.log" 2>&1
echo done
