#!/bin/bash
# Round 5: multi-chunk calls with doubling chunk sizes.  The chunk tests, then
# config 3 host-to-host by chunk size with the ramp on / off (alternating).
#   bash tools/r05_ramp.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "chunk_ramp or config3_affine or memcpy_d2h" > "$OUT/ramp_tests.log" 2>&1
echo "ramp tests: $(tail -1 "$OUT/ramp_tests.log")"
timeout -k 10 400 python3 -u tools/h2h_sweep.py --chunks 32768,65536,131072,262144,524288 --ramp 1,0 --reps 2 \
  > "$OUT/h2h_ramp.jsonl" 2> "$OUT/h2h_ramp.err"
echo done
