#!/bin/bash
# Round 5 verification on a fresh box: the gz tests first (new in-place edge
# cases), smoke(), then the whole GPU suite.   bash tools/r05_verify.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_gz.py \
  > "$OUT/gz_tests.log" 2>&1
echo "gz tests: $(tail -1 "$OUT/gz_tests.log")"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke: $(tail -1 "$OUT/smoke.log")"
bash tools/gpu_tests.sh "$T"
echo done
