#!/bin/bash
# Round 5 tuning runs on the GPU box: GPU tests, config 3 from FASTQ under
# reader batch / span settings (alternating), and the narrow-group crossover
# by batch size.   bash tools/r05_tune.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_tests.sh "$T"
timeout -k 10 400 python3 -u tools/c3f_env_ab.py --out "$OUT/c3f_ab.jsonl" --reps 3 \
  --setting base= --setting batch262k=MSW_GFASTQ_BATCH=262144 --setting batch131k=MSW_GFASTQ_BATCH=131072 \
  --setting span96=MSW_GFASTQ_SPAN_MB=96 --setting span96_batch131k=MSW_GFASTQ_SPAN_MB=96,MSW_GFASTQ_BATCH=131072 \
  > "$OUT/c3f_ab.log" 2>&1
timeout -k 10 400 python3 -u tools/group_lanes_probe.py --sizes 131072,262144,524288,786432 --settings 9,16 \
  > "$OUT/group_9v16.jsonl" 2> "$OUT/group_9v16.err"
echo done
