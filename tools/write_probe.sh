#!/bin/bash
# WRITE_SIZE / FETCH_SIZE per launch and kernel time for a few shapes, current
# build vs tools/_variants/libmsw_$1.so:  bash tools/write_probe.sh VARIANT OUTDIR
set -euo pipefail
V=$1; OUT=${2:-gpurun_out/wprobe}
mkdir -p "$OUT"
for lib in cur $V; do
  if [ $lib = cur ]; then unset MSW_LIB_PATH; else export MSW_LIB_PATH=$PWD/tools/_variants/libmsw_$lib.so; fi
  for shape in "c2:--pairs 10000" "c3:--pairs 10000 --affine --coords"; do
    n=${shape%%:*}; a=${shape#*:}
    timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d "$OUT/${lib}_${n}_w" -o p --output-format csv -- python3 tools/lever_probe.py --reps 5 --check 0 --label ${lib}_$n $a > /dev/null 2>&1
    timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$OUT/${lib}_${n}_f" -o p --output-format csv -- python3 tools/lever_probe.py --reps 5 --check 0 --label ${lib}_$n $a > /dev/null 2>&1
    timeout -k 10 90 python3 tools/lever_probe.py --reps 50 --check 512 --label ${lib}_$n $a >> "$OUT/probe.jsonl"
  done
done
