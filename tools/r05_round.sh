#!/bin/bash
# Round 5 check on the GPU box: tests, config 3 from FASTQ traced, config 5
# traffic split by buffer, the default bench.   bash tools/r05_round.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_tests.sh "$T"
bash tools/c3f_kernel_trace.sh "$T"
bash tools/traffic_c5_split.sh "$T"
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > "$OUT/bench.out" 2> "$OUT/bench.err"
echo done
