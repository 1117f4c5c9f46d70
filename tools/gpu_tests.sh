#!/bin/bash
# GPU test suite on the box (bash tools/gpu_tests.sh TAG [pytest args...]):
# one pytest process, per-test thread timeouts, log under gpurun_out/TAG.
set -euo pipefail
T=${1:-tests}
shift || true
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread "$@" > "$OUT/gputest.log" 2>&1
echo "gpu tests: $(tail -1 "$OUT/gputest.log")"
