#!/bin/bash
# Config 3 from FASTQ (1 M reads, affine + best cell, every record checked)
# by lane-file layout, on the box:  bash tools/c3f_probe.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
for lanes in 8 2 1; do
  for rep in 1 2; do
    timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --pairs 2000 --cpu-seconds 0 --no-pcie --no-h2h \
      --extra-configs 3 --c3-pairs 2000 --c3-fastq-lanes $lanes 2>/dev/null | grep '^{' | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())['configs_extra']['config3']['fastq']
print(json.dumps({'lanes': $lanes, 'files': 2 * $lanes, 'reads_per_s': d['reads_per_s'], 'wall_ms': d['wall_ms'],
                  'setup_ms': d['setup_ms'], 'kernel_ms': d['max_kernel_ms'], 'bit_exact': d['parity']['bit_exact']}))" >> "$OUT/c3f.jsonl"
  done
done
echo done
