#!/bin/bash
# GPU-box A/B of kernel variants (tools/build_variant.sh) over the four scoring
# kinds: bash tools/ab_sweep.sh OUT.log SIZES VARIANT...
set -uo pipefail
OUT=$1; SIZES=$2; shift 2
mkdir -p "$(dirname "$OUT")"
for v in "$@"; do
  export MSW_LIB_PATH=$PWD/tools/_variants/libmsw_$v.so
  for kind in "" "--coords" "--affine" "--affine --coords"; do
    echo "== $v ${kind:-linear}" >> "$OUT"
    timeout -k 10 120 python -u tools/sweep.py --config 2 --sizes "$SIZES" --layouts auto --reps 20 $kind 2>/dev/null >> "$OUT" || exit 1
  done
done
