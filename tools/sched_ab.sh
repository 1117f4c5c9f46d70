#!/bin/bash
# A/B of the explicitly scheduled linear f16 loop (MSW_LIN_SCHED) on the GPU box:
#   bash tools/sched_ab.sh OUTDIR   (needs tools/_variants/libmsw_sched0.so)
set -euo pipefail
OUT=${1:-gpurun_out/sched}
mkdir -p "$OUT"
P="python3 tools/lever_probe.py --check 2048"
for v in sched0 new; do
  if [ $v = new ]; then unset MSW_LIB_PATH; else export MSW_LIB_PATH=$PWD/tools/_variants/libmsw_$v.so; fi
  for args in "--pairs 10000" "--pairs 65536" "--pairs 20000" "--read-len 100 --win-len 200 --pairs 40000" "--read-len 250 --win-len 500 --pairs 20000"; do
    timeout -k 10 120 $P --label "$v" $args >> "$OUT/probe.jsonl"
  done
done
unset MSW_LIB_PATH
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_c2" -o k --output-format csv -- $P --label rocprof_c2 --pairs 10000 >> "$OUT/probe.jsonl"
