#!/bin/bash
# Long pairs: heaviest-first slots, round-balanced grids, the long launch
# beside the packed ones on the side stream.  Whole GPU suite, long bench.
set -euo pipefail
OUT=gpurun_out/queue3
bash tools/gpu_tests.sh queue3 tests
timeout -k 10 300 python3 tools/long_bench.py > $OUT/long_bench.jsonl 2>$OUT/long_bench.err
echo "bench done"
