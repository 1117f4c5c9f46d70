#!/bin/bash
# config-5 traffic after the window-chunk clamp: FETCH / WRITE per launch + kernel time
set -euo pipefail
OUT=${1:-gpurun_out/tc5}; mkdir -p "$OUT"
B="python3 bench.py --config 5 --steps 20 --warmup 3 --cpu-seconds 0 --no-pcie --extra-configs none"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o t --output-format csv -- $B > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o p --output-format csv -- $B > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o p --output-format csv -- $B > "$OUT/write.log" 2>&1
