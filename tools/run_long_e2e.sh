#!/bin/bash
# Long-read (MiSeq-like 300 bp, window 600) end to end at the config-4 file layout, both readers.
set -euo pipefail
OUT=gpurun_out/long_e2e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/wgs_e2e.py --dir /tmp/msw_long_e2e --reads-per-file 1000000 --read-len 300 --window 600 \
  --bgzf --qual binned --level 6 --workers 16 --host-threads 16 \
  --extra-env "MSW_GPU_INFLATE=1;MSW_GPU_INFLATE=0" --out $OUT/e2e.jsonl > $OUT/e2e.log 2> $OUT/e2e.err
echo done
