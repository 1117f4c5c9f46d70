#!/bin/bash
# Round 5: first spans inflated in place from pinned host pages.  GPU tests,
# config 3 from FASTQ in place vs uploaded (alternating), config 4 with every
# file's first span in place vs the default, a config-3 kernel trace.
#   bash tools/r05_inplace.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_gz.py \
  > "$OUT/gz_tests.log" 2>&1
echo "gz tests: $(tail -1 "$OUT/gz_tests.log")"
bash tools/gpu_tests.sh "$T"
timeout -k 10 300 python3 -u tools/c3f_env_ab.py --out "$OUT/c3f_ab.jsonl" --reps 4 \
  --setting in_place= --setting upload=MSW_GZ_IN_PLACE_MB=0 > "$OUT/c3f_ab.log" 2>&1
bash tools/c3f_kernel_trace.sh "$T"
timeout -k 10 400 python3 -u tools/c4_env_ab.py --b MSW_GZ_IN_PLACE_MB=100000 --reps 3 --out "$OUT/c4_ab.jsonl" \
  > "$OUT/c4_ab.log" 2>&1
echo done
