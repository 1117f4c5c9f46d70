#!/bin/bash
# Round 5: the reader's window unpin off the critical path (and a file's last
# window kept pinned while another reader inflates in place) against the
# previous build (tools/_ab/unpin_old): config 3 from FASTQ and config 4,
# alternating.   bash tools/r05_unpin2.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
OLD="$PWD/tools/_ab/unpin_old"
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_gz.py \
  tests/test_cli.py > "$OUT/gz_tests.log" 2>&1
echo "gz + cli tests: $(tail -1 "$OUT/gz_tests.log")"
timeout -k 10 400 python3 -u tools/c3f_env_ab.py --out "$OUT/c3f_ab.jsonl" --reps 6 \
  --setting new= --setting "old=LD_LIBRARY_PATH=$OLD:${LD_LIBRARY_PATH:-}" > "$OUT/c3f_ab.log" 2>&1
timeout -k 10 400 python3 -u tools/c4_env_ab.py --b "LD_LIBRARY_PATH=$OLD:${LD_LIBRARY_PATH:-}" --reps 3 \
  --out "$OUT/c4_ab.jsonl" > "$OUT/c4_ab.log" 2>&1
bash tools/c3f_kernel_trace.sh "$T"
echo done
