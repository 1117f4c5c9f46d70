#!/bin/bash
# Round 5 host-path check on the GPU box: the GPU test suite, then the
# 10k-pair host-to-host stream with the kernels storing results into the
# mapped host block (default) and with the readback copy (MSW_NO_DIRECT_OUT),
# alternated, then the default bench.  bash tools/r05_host_ab.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_tests.sh "$T"
for k in 1 2; do
  timeout -k 10 200 python3 -u tools/stream_probe.py --trace > "$OUT/stream_direct_$k.jsonl" 2> "$OUT/stream_direct_$k.err"
  MSW_NO_DIRECT_OUT=1 timeout -k 10 200 python3 -u tools/stream_probe.py --trace > "$OUT/stream_copy_$k.jsonl" 2> "$OUT/stream_copy_$k.err"
done
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > "$OUT/bench.out" 2> "$OUT/bench.err"
echo done
