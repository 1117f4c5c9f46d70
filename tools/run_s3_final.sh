#!/bin/bash
# Final-state check of the round plus the inflate grid-cap sweep at the config-4 shape.
set -euo pipefail
bash tools/run_final_check.sh s3_check1
D=/tmp/msw_gz_e2e
OUT=gpurun_out/s3_check1/capsweep
mkdir -p $OUT
timeout -k 10 400 python3 tools/wgs_e2e.py --dir $D --reads-per-file 2000000 --bgzf --qual binned --level 6 --reuse \
  --host-threads 16 --extra-env "MSW_GPU_INFLATE=1;MSW_GPU_INFLATE=1,MSW_GZ_WAVES_PER_SIMD=6;MSW_GPU_INFLATE=1,MSW_GZ_WAVES_PER_SIMD=5;MSW_GPU_INFLATE=1,MSW_GZ_WAVES_PER_SIMD=4;MSW_GPU_INFLATE=1,MSW_GZ_WAVES_PER_SIMD=3" \
  --out $OUT/e2e.jsonl > $OUT/e2e.log 2> $OUT/e2e.err
echo "cap sweep done"
