#!/bin/bash
# Round 5 narrow-gate check on the GPU box: GPU tests, the model's choice
# against 16-lane groups by batch size (A/B, alternating), config 3 from
# FASTQ at the new record-mode batch against 128k batches, the default bench
# under a kernel trace.   bash tools/r05_gate.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_tests.sh "$T"
timeout -k 10 400 python3 -u tools/group_lanes_probe.py --sizes 65536,131072,262144,524288,1048576 --settings auto,16 \
  > "$OUT/group_auto_v16.jsonl" 2> "$OUT/group_auto_v16.err"
timeout -k 10 300 python3 -u tools/c3f_env_ab.py --out "$OUT/c3f_ab.jsonl" --reps 3 \
  --setting base= --setting batch131k=MSW_GFASTQ_BATCH=131072 > "$OUT/c3f_ab.log" 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/bench_trace" -o t -- \
  python3 -u bench.py --steps 20 --warmup 5 > "$OUT/bench.out" 2> "$OUT/bench.err"
echo done
