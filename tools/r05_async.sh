#!/bin/bash
# Round 5: one-chunk async uploads on the copy stream.  Genome GPU tests (the
# new async upload-form test among them), the stream A/B against the
# one-stream form, then the default bench.   bash tools/r05_async.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_genome.py \
  > "$OUT/genome_tests.log" 2>&1
echo "genome tests: $(tail -1 "$OUT/genome_tests.log")"
timeout -k 10 200 python3 -u tools/stream_ab.py --setting copy= --setting one=MSW_ASYNC_ONE_STREAM=1 --reps 3 \
  > "$OUT/stream_ab.jsonl" 2> "$OUT/stream_ab.err"
timeout -k 10 600 python3 -u bench.py --detail "$OUT/bench_detail.json" > "$OUT/bench.json" 2> "$OUT/bench.err"
echo done
