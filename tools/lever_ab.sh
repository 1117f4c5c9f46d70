#!/bin/bash
# Config-2 lever A/B on the GPU box:  bash tools/lever_ab.sh OUTDIR
#  (a) prologue variants: tools/_variants/libmsw_{pro_base,pro_early,pro_dpp,pro_both}.so
#  (b) best-case proxies of a two-waves-per-SIMD split of config 2 (kernel as is):
#      row split  = 20k pairs of 75 bp reads x 300 bp windows (G = 12 / G = 15)
#      column split = 20k pairs of 150 bp reads x 150 bp windows
# Each point once under rocprofv3 --kernel-trace --stats (its own directory).
set -euo pipefail
OUT=${1:-gpurun_out/lever}
mkdir -p "$OUT"
P="python3 tools/lever_probe.py"
run() {  # name, env..., -- probe args
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o k --output-format csv -- $P --label "$name" "$@" \
      >> "$OUT/probe.jsonl" 2> "$OUT/$name.err"
}
for v in pro_base pro_early pro_dpp pro_both; do
  export MSW_LIB_PATH=$PWD/tools/_variants/libmsw_$v.so
  run "c2_$v" --pairs 10000
  run "c2_65k_$v" --pairs 65536
  run "c3_$v" --pairs 10000 --affine --coords
done
unset MSW_LIB_PATH
run proxy_row_g12 --read-len 75 --pairs 20000 --group-lanes 12 --layout pairs
run proxy_row_g15 --read-len 75 --pairs 20000 --group-lanes 15 --layout pairs
run proxy_col_g12 --win-len 150 --pairs 20000 --group-lanes 12 --layout pairs
run base_20k_g12 --pairs 20000 --group-lanes 12 --layout pairs
echo done
