#!/bin/bash
# GPU lane reader alone: tools/gfastq_bench.py, then the same under a rocprofv3
# kernel trace (per-kernel times of inflate / CRC / parse / emit, nothing else
# on the GPU).   bash tools/gfastq_prof.sh TAG [reads] [extra bench args]
set -euo pipefail
T=${1:-gfastq}
N=${2:-2000000}
shift 2 || true
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/gfastq_bench.py --reads "$N" "$@" > "$OUT/bench.log" 2>&1
cat "$OUT/bench.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o t --output-format csv -- \
  python3 tools/gfastq_bench.py --reads "$N" --passes 2 "$@" > "$OUT/prof.log" 2>&1
echo "profile done"
