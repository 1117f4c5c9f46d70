#!/bin/bash
# Reads of 257..384 bases on the packed kernels (KR 17..24): whole GPU suite,
# the long-pair bench and the 300 bp end to end.
set -euo pipefail
bash tools/gpu_tests.sh wide2 tests
timeout -k 10 300 python3 tools/long_bench.py > gpurun_out/wide2/long_bench.jsonl 2>/dev/null
echo "bench done"
OUT=gpurun_out/wide2
timeout -k 10 600 python3 tools/wgs_e2e.py --dir /tmp/msw_long_e2e --reads-per-file 1000000 --read-len 300 --window 600 \
  --bgzf --qual binned --level 6 --workers 16 --host-threads 16 \
  --extra-env "MSW_GPU_INFLATE=1" --out $OUT/e2e_300bp.jsonl > $OUT/e2e.log 2> $OUT/e2e.err
echo "e2e done"
