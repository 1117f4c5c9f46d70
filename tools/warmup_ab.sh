#!/bin/bash
# Config-2 headline vs warm-up length and step count (the GPU's clock ramp
# under a 1 ms timed region), on the box:  bash tools/warmup_ab.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
B="python3 bench.py --extra-configs none --no-pcie --cpu-seconds 0"
for rep in 1 2; do
  for v in "20 5" "20 2000" "200 5" "2000 5"; do
    set -- $v
    timeout -k 10 120 $B --steps $1 --warmup $2 2>/dev/null | grep '^{' | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'steps': $1, 'warmup': $2, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'avg_launch_ms': d['roofline']['avg_launch_ms'], 'pipelined': d['pipelined_two_streams']['value']}))" >> "$OUT/warmup_ab.jsonl"
  done
done
echo "warmup A/B done"
