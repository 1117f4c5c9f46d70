#!/bin/bash
# Round 5: in-place first spans split: the first P % of members DMA'd and
# inflated from HBM on a second stream (MSW_GZ_SPLIT), config 3 from FASTQ
# alternating against the unsplit in-place span.   bash tools/r05_split.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_gz.py \
  > "$OUT/gz_tests.log" 2>&1
echo "gz tests: $(tail -1 "$OUT/gz_tests.log")"
timeout -k 10 400 python3 -u tools/c3f_env_ab.py --out "$OUT/c3f_split.jsonl" --reps 5 \
  --setting base= --setting s25=MSW_GZ_SPLIT=25 --setting s40=MSW_GZ_SPLIT=40 > "$OUT/c3f_split.log" 2>&1
echo done
