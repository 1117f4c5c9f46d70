#!/bin/bash
# GPU reader span (MSW_GFASTQ_SPAN_MB) at the config-4 shape, alternating runs.
set -euo pipefail
OUT=gpurun_out/span
mkdir -p $OUT
export TMPDIR=/tmp
D=/tmp/msw_gz_e2e
A="--dir $D --reads-per-file 2000000 --bgzf --qual binned --level 6 --workers 16 --host-threads 16"
timeout -k 10 400 python3 tools/wgs_e2e.py $A --extra-env "MSW_GPU_INFLATE=1" --out $OUT/s1024_a.jsonl > $OUT/gen.log 2>&1
echo "s1024_a $(grep -o '"throughput_reads_per_second": [0-9.]*' $OUT/s1024_a.jsonl)"
for r in s256_a s512_a s2048_a s1024_b s256_b s512_b s2048_b; do
  S=${r#s}; S=${S%_*}
  timeout -k 10 200 python3 tools/wgs_e2e.py $A --reuse --extra-env "MSW_GPU_INFLATE=1,MSW_GFASTQ_SPAN_MB=$S" \
    --out $OUT/$r.jsonl > $OUT/$r.log 2>&1
  echo "$r $(grep -o '"throughput_reads_per_second": [0-9.]*' $OUT/$r.jsonl)"
done
