#!/bin/bash
# One GPU-box check of the tree as built here (run from the repo root on the box):
#   bash tools/gpu_check.sh TAG
# GPU test suite, the default bench line, a --gpus 2 refusal check on the
# one-GPU box, and a rocprofv3 kernel-trace summary of the config-2 bench.
set -euo pipefail
T=${1:-check}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/gputest.log" 2>&1
echo "gpu tests ok: $(tail -1 "$OUT/gputest.log")"
timeout -k 10 300 python3 bench.py --detail "$OUT/bench_detail.json" > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench ok"
# fewer GPUs than asked for must fail loudly (rc != 0), never print n_gpus 1
if timeout -k 10 120 python3 bench.py --gpus 2 --steps 2 --warmup 1 > "$OUT/gpus2.out" 2>&1; then
  echo "ERROR: bench.py --gpus 2 succeeded on a one-GPU box"; exit 1
fi
echo "gpus2 refused as expected: $(tail -1 "$OUT/gpus2.out")"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o t --output-format csv -- \
  python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie --extra-configs none --detail "$OUT/prof_detail.json" \
  > "$OUT/prof_c2.log" 2>&1
echo "profile ok"
