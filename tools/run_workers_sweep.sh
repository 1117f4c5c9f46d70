#!/bin/bash
# Config-4 shape on one GPU: 1 / 2 / 4 CLI workers sharing the device
# (MSW_DEVICES=0,0,...), GPU lane reader.
set -euo pipefail
OUT=gpurun_out/workers
mkdir -p $OUT
export TMPDIR=/tmp
D=/tmp/msw_gz_e2e
A="--dir $D --reads-per-file 2000000 --bgzf --qual binned --level 6 --workers 16 --host-threads 16"
timeout -k 10 400 python3 tools/wgs_e2e.py $A --extra-env "MSW_GPU_INFLATE=1" --out $OUT/w1_a.jsonl > $OUT/gen.log 2>&1
echo "w1_a $(grep -o '"throughput_reads_per_second": [0-9.]*' $OUT/w1_a.jsonl)"
for r in w2_a w4_a w1_b w2_b w4_b; do
  W=${r:1:1}; DEV=$(python3 -c "print(','.join(['0']*$W))")
  MSW_DEVICES=$DEV timeout -k 10 200 python3 tools/wgs_e2e.py $A --reuse --num-gpus $W --extra-env "MSW_GPU_INFLATE=1" \
    --out $OUT/$r.jsonl > $OUT/$r.log 2>&1
  echo "$r $(grep -o '"throughput_reads_per_second": [0-9.]*' $OUT/$r.jsonl)"
done
