#!/bin/bash
# Wave-level trace (prologue, wave duration, clock) of config-2-shape launches,
# current build vs variants:  bash tools/trace_ab.sh OUT VARIANT...
set -euo pipefail
OUT=${1:-gpurun_out/trace_ab.jsonl}; shift
for v in new "$@"; do
  if [ $v = new ]; then unset MSW_LIB_PATH; else export MSW_LIB_PATH=$PWD/tools/_variants/libmsw_$v.so; fi
  for k in "" "--coords" "--affine --coords" "--affine"; do
    echo "== $v $k" >> "$OUT"
    timeout -k 10 120 python3 tools/wave_trace.py --config 2 --pairs 10000 $k 2>/dev/null | tail -1 >> "$OUT"
  done
done
