#!/bin/bash
# Whole-tree GPU check (bash tools/run_final_check.sh TAG): the GPU test
# suite, smoke(), the default bench line + rocprof summary (tools/gpu_check.sh
# parts), then the config-4-shape end to end with the GPU lane reader.
set -euo pipefail
T=${1:-final}
bash tools/gpu_tests.sh "$T" tests
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1
echo "smoke: $(tail -1 gpurun_out/$T/smoke.log)"
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof_c2 -o t --output-format csv -- \
  python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie --extra-configs none \
  > gpurun_out/$T/prof_c2.log 2>&1
echo "profile ok"
VARIANTS="MSW_GPU_INFLATE=1" bash tools/gz_e2e.sh $T/e2e 2000000 binned 6
