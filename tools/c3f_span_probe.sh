#!/bin/bash
# Config 3 from FASTQ (2 lane files x 500k reads) by reader span size, on the box:
#   bash tools/c3f_span_probe.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
for span in 1024 256 128 64 32; do
  for rep in 1 2; do
    MSW_GFASTQ_SPAN_MB=$span timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --pairs 2000 --cpu-seconds 0 \
      --no-pcie --no-h2h --extra-configs 3 --c3-pairs 2000 2>/dev/null | grep '^{' | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())['configs_extra']['config3']['fastq']
print(json.dumps({'span_mb': $span, 'reads_per_s': d['reads_per_s'], 'wall_ms': d['wall_ms'],
                  'kernel_ms': d['max_kernel_ms'], 'bit_exact': d['parity']['bit_exact']}))" >> "$OUT/c3f_span.jsonl"
  done
done
echo done
