#!/bin/bash
# Collect the round's rocprofv3 evidence for the bench workloads (run on the GPU
# box from the repo root):  bash tools/profile_round.sh r01   [CONFIGS="3" for one]
# Per config: one kernel-trace pass (--stats), then one PMC pass per counter
# group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; see
# MI355X_MICROARCH.md "rocprofv3 PMC slots").  The bench runs without the CPU
# baseline and the host-to-host variants, so only the timed launches appear.
set -euo pipefail
R=${1:-r01}
OUT=gpurun_out/prof_$R
mkdir -p "$OUT"
# the commit of the profiled tree (the GPU box has no .git: pass it in)
echo "${MSW_COMMIT:-unknown}" > "$OUT/COMMIT"
export TMPDIR=/tmp
for CFG in ${CONFIGS:-2 3 5}; do  # CONFIGS="3": one config only
  case $CFG in
    2) ARGS="--steps 50 --warmup 5" ;;
    3) ARGS="--steps 5 --warmup 2" ;;
    5) ARGS="--steps 20 --warmup 3" ;;
  esac
  BENCH="python3 bench.py --config $CFG $ARGS --cpu-seconds 0 --no-pcie --extra-configs none"
  D="$OUT/c$CFG"
  mkdir -p "$D"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$D/trace" -o t --output-format csv -- $BENCH > "$D/trace.log" 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$D/fetch" -o p --output-format csv -- $BENCH > "$D/fetch.log" 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$D/write" -o p --output-format csv -- $BENCH > "$D/write.log" 2>&1
  if [ "$CFG" = 2 ]; then
    timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d "$D/occ" -o p --output-format csv -- $BENCH > "$D/occ.log" 2>&1
    timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d "$D/inst" -o p --output-format csv -- $BENCH > "$D/inst.log" 2>&1
  fi
  echo "config $CFG profiled"
done
echo "profile $R done"
