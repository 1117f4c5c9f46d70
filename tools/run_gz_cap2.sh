#!/bin/bash
# Inflate grid cap (MSW_GZ_WAVES_PER_SIMD) re-measured at the config-4 shape
# now that the GPU is busy end to end (no host gaps), alternating runs.
set -euo pipefail
OUT=gpurun_out/gzcap2
mkdir -p $OUT
export TMPDIR=/tmp
D=/tmp/msw_gz_e2e
A="--dir $D --reads-per-file 2000000 --bgzf --qual binned --level 6 --workers 16 --host-threads 16"
timeout -k 10 400 python3 tools/wgs_e2e.py $A --extra-env "MSW_GPU_INFLATE=1" --out $OUT/c0_a.jsonl > $OUT/gen.log 2>&1
echo "c0_a $(grep -o '"throughput_reads_per_second": [0-9.]*' $OUT/c0_a.jsonl)"
for r in c6_a c5_a c4_a c0_b c6_b c5_b c4_b; do
  C=${r:1:1}; E="MSW_GPU_INFLATE=1"
  [ "$C" != 0 ] && E="$E,MSW_GZ_WAVES_PER_SIMD=$C"
  timeout -k 10 200 python3 tools/wgs_e2e.py $A --reuse --extra-env "$E" --out $OUT/$r.jsonl > $OUT/$r.log 2>&1
  echo "$r $(grep -o '"throughput_reads_per_second": [0-9.]*' $OUT/$r.jsonl)"
done
