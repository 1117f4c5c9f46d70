#!/bin/bash
# Round-end rehearsal on a fresh box: the GPU suite, smoke(), the driver's
# bench command.   bash tools/r05_final.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_tests.sh "$T"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke: $(tail -1 "$OUT/smoke.log")"
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 --detail "$OUT/bench_detail.json" > "$OUT/bench.json" \
  2> "$OUT/bench.err"
echo done
