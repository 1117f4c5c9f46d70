#!/bin/bash
# A/B of the explicitly scheduled f16 loops: current build vs variants
#   bash tools/sched_ab.sh OUTDIR VARIANT...   (tools/_variants/libmsw_<v>.so)
set -euo pipefail
OUT=${1:-gpurun_out/sched}; shift
mkdir -p "$OUT"
P="python3 tools/lever_probe.py --check 1024"
for v in new "$@"; do
  if [ $v = new ]; then unset MSW_LIB_PATH; else export MSW_LIB_PATH=$PWD/tools/_variants/libmsw_$v.so; fi
  for args in "--pairs 10000" "--pairs 10000 --coords" "--pairs 10000 --affine" "--pairs 10000 --affine --coords" \
              "--pairs 65536" "--pairs 65536 --coords" "--pairs 65536 --affine" "--pairs 200000 --affine --coords"; do
    timeout -k 10 120 $P --label "$v" $args >> "$OUT/probe.jsonl"
  done
done
