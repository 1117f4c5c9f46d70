#!/bin/bash
# Round 5: config 3 from FASTQ by record-batch size (alternating), after the
# narrow-group gate moved (500k-read batches are now past it).
#   bash tools/r05_c3f_batch.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/c3f_env_ab.py --out "$OUT/c3f_batch.jsonl" --reps 4 \
  --setting b262k= --setting b524k=MSW_GFASTQ_BATCH=524288 --setting b393k=MSW_GFASTQ_BATCH=393216 \
  --setting b196k=MSW_GFASTQ_BATCH=196608 > "$OUT/c3f_batch.log" 2>&1
echo done
