#!/bin/bash
# Round 5: a file's last window kept pinned while another reader inflates in
# place, and the reader stream at the greatest priority (MSW_GFASTQ_PRIORITY),
# against the previous build (tools/_ab/unpin_old): config 3 from FASTQ and
# config 4, alternating.   bash tools/r05_unpin3.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
OLD="$PWD/tools/_ab/unpin_old"
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_gz.py \
  tests/test_cli.py > "$OUT/gz_tests.log" 2>&1
echo "gz + cli tests: $(tail -1 "$OUT/gz_tests.log")"
timeout -k 10 400 python3 -u tools/c3f_env_ab.py --out "$OUT/c3f_ab.jsonl" --reps 5 \
  --setting new= --setting prio=MSW_GFASTQ_PRIORITY=1 --setting "old=LD_LIBRARY_PATH=$OLD:${LD_LIBRARY_PATH:-}" \
  > "$OUT/c3f_ab.log" 2>&1
timeout -k 10 400 python3 -u tools/c4_env_ab.py --b "LD_LIBRARY_PATH=$OLD:${LD_LIBRARY_PATH:-}" --reps 2 \
  --out "$OUT/c4_ab_old.jsonl" > "$OUT/c4_ab_old.log" 2>&1
timeout -k 10 400 python3 -u tools/c4_env_ab.py --b MSW_GFASTQ_PRIORITY=1 --reps 2 \
  --out "$OUT/c4_ab_prio.jsonl" > "$OUT/c4_ab_prio.log" 2>&1
echo done
