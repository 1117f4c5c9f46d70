#!/bin/bash
# Round 5: the reader's window unpin moved off the span's critical path.
# gz tests (incl. the in-place page-boundary files), smoke, the GPU suite,
# then config 3 from FASTQ against the previous build (tools/_ab/unpin_old)
# alternating, and a config-3 kernel trace.   bash tools/r05_unpin.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
OLD="$PWD/tools/_ab/unpin_old"
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_gz.py \
  > "$OUT/gz_tests.log" 2>&1
echo "gz tests: $(tail -1 "$OUT/gz_tests.log")"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke: $(tail -1 "$OUT/smoke.log")"
bash tools/gpu_tests.sh "$T"
timeout -k 10 300 python3 -u tools/c3f_env_ab.py --out "$OUT/c3f_ab.jsonl" --reps 4 \
  --setting new= --setting "old=LD_LIBRARY_PATH=$OLD:${LD_LIBRARY_PATH:-}" > "$OUT/c3f_ab.log" 2>&1
bash tools/c3f_kernel_trace.sh "$T"
echo done
