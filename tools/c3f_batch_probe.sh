#!/bin/bash
# Config 3 from FASTQ (2 lane files x 500k reads, affine + best cell, every
# record checked) by scoring batch size (MSW_GFASTQ_BATCH: reads per scoring
# launch; smaller batches let a batch's readback and host records overlap the
# next batch's scoring), on the box:  bash tools/c3f_batch_probe.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
for rep in 1 2; do
  for batch in 1048576 262144 131072 65536; do
    MSW_GFASTQ_BATCH=$batch timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --pairs 2000 --cpu-seconds 0 \
      --no-pcie --no-h2h --extra-configs 3 --c3-pairs 2000 2>/dev/null | grep '^{' | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())['configs_extra']['config3']['fastq']
print(json.dumps({'batch': $batch, 'reads_per_s': d['reads_per_s'], 'wall_ms': d['wall_ms'],
                  'kernel_ms': d['max_kernel_ms'], 'bit_exact': d['parity']['bit_exact']}))" >> "$OUT/c3f_batch.jsonl"
  done
done
echo done
