#!/bin/bash
# SQ counters per launch for one lever_probe shape, current build vs variants:
#   bash tools/pmc_ab.sh OUTDIR "PROBE ARGS" VARIANT...
set -euo pipefail
OUT=$1; ARGS=$2; shift 2
mkdir -p "$OUT"
for v in new "$@"; do
  if [ $v = new ]; then unset MSW_LIB_PATH; else export MSW_LIB_PATH=$PWD/tools/_variants/libmsw_$v.so; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY \
      -d "$OUT/$v" -o p --output-format csv -- python3 tools/lever_probe.py --reps 5 --check 0 $ARGS > /dev/null 2>&1
done
