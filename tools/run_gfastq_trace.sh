#!/bin/bash
# Config-4-shape end to end with the GPU reader's per-span host trace
# (MSW_GFASTQ_TRACE): where the reader thread spends each span.
set -euo pipefail
OUT=gpurun_out/gtrace
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_tests.sh gtrace tests/test_gpu_gz.py tests/test_cli.py tests/test_fastq.py
timeout -k 10 500 python3 tools/wgs_e2e.py --dir /tmp/msw_gz_e2e --reads-per-file 2000000 --bgzf --qual binned --level 6 \
  --workers 16 --host-threads 16 --extra-env "MSW_GPU_INFLATE=1,MSW_GFASTQ_TRACE=1" --out $OUT/e2e.jsonl > $OUT/e2e.log 2> $OUT/e2e.err
echo "e2e done $(grep -o '"throughput_reads_per_second": [0-9.]*' $OUT/e2e.jsonl)"
