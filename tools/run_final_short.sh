#!/bin/bash
# Whole GPU suite, smoke() and the default bench line (no end to end).
set -euo pipefail
T=${1:-final_short}
bash tools/gpu_tests.sh "$T" tests
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1
echo "smoke: $(tail -1 gpurun_out/$T/smoke.log)"
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
echo "bench ok"
