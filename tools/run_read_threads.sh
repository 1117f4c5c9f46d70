#!/bin/bash
# Compressed-read threads of the GPU lane reader (MSW_GZ_READ_THREADS) at the
# config-4 shape, alternating with the pre-change build in _ab_old/.
set -euo pipefail
OUT=gpurun_out/rthreads
mkdir -p $OUT
export TMPDIR=/tmp
D=/tmp/msw_gz_e2e
A="--dir $D --reads-per-file 2000000 --bgzf --qual binned --level 6 --workers 16 --host-threads 16"
timeout -k 10 400 python3 tools/wgs_e2e.py $A --extra-env "MSW_GPU_INFLATE=1" --out $OUT/t4_a.jsonl > $OUT/gen.log 2>&1
for r in old_a t1_a t8_a t4_b old_b t8_b t1_b; do
  C=""; T=${r#t}; T=${T%_*}
  case $r in old*) C="--cli _ab_old/rustseq_mini"; T=4;; esac
  timeout -k 10 200 python3 tools/wgs_e2e.py $A --reuse $C --extra-env "MSW_GPU_INFLATE=1,MSW_GZ_READ_THREADS=$T" \
    --out $OUT/$r.jsonl > $OUT/$r.log 2>&1
  echo "$r $(grep -o '"throughput_reads_per_second": [0-9.]*' $OUT/$r.jsonl)"
done
