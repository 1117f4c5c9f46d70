#!/bin/bash
# Collect the round's rocprofv3 evidence for the bench workload (run on the GPU
# box from the repo root):  bash tools/profile_round.sh r01
# One counter group per pass (FETCH_SIZE and WRITE_SIZE cannot share a pass on
# gfx950; see MI355X_MICROARCH.md "rocprofv3 PMC slots").
set -euo pipefail
R=${1:-r01}
OUT=gpurun_out/prof_$R
mkdir -p "$OUT"
BENCH="python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o t --output-format csv -- $BENCH > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o p --output-format csv -- $BENCH > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o p --output-format csv -- $BENCH > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d "$OUT/occ" -o p --output-format csv -- $BENCH > "$OUT/occ.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d "$OUT/inst" -o p --output-format csv -- $BENCH > "$OUT/inst.log" 2>&1
echo "profile $R done"
