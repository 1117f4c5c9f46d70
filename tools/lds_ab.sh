#!/bin/bash
# A/B of read staging through LDS (current build) vs byte loads (libmsw_nolds.so)
set -euo pipefail
OUT=${1:-gpurun_out/lds}
mkdir -p "$OUT"
P="python3 tools/lever_probe.py --check 1024"
for v in nolds new; do
  if [ $v = new ]; then unset MSW_LIB_PATH; else export MSW_LIB_PATH=$PWD/tools/_variants/libmsw_$v.so; fi
  for args in "--pairs 10000" "--pairs 65536" "--pairs 10000 --affine --coords" "--read-len 100 --win-len 200 --pairs 40000" "--read-len 250 --win-len 500 --pairs 20000"; do
    timeout -k 10 120 $P --label "$v" $args >> "$OUT/probe.jsonl"
  done
done
