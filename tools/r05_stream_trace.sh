#!/bin/bash
# Round 5: kernel + memory-copy trace of the host-to-host stream of 10k-pair
# calls (tools/stream_probe.py, depth 3): GPU busy vs host-bound.
#   bash tools/r05_stream_trace.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/trace" -o t --output-format csv -- \
  python3 -u tools/stream_probe.py --batches 400 > "$OUT/probe.log" 2>&1
echo done
