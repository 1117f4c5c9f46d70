#!/bin/bash
# Round 5: inflate ring size at low member counts (config 3 from FASTQ's
# one-file / two-file launches) and the far-load share of a window
# (MSW_GZ_PROFILE builds).   bash tools/r05_ring.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in gzprof gzprof8; do
  MSW_LIB_PATH="$PWD/tools/_ab/$v/libmsw.so" MSW_GZ_PROFILE=1 MSW_GZ_TIMING=1 timeout -k 10 200 \
    python3 -u tools/inflate_bench.py --members 2534,16384 > "$OUT/prof_$v.out" 2> "$OUT/prof_$v.log"
done
for rep in 1 2 3; do
  for v in ring2 ring4 ring8; do
    LIB="$PWD/tools/_ab/$v/libmsw.so"; [ "$v" = ring2 ] && LIB="$PWD/mini_parallel_amd/libmsw.so"
    MSW_LIB_PATH="$LIB" MSW_GZ_TIMING=1 timeout -k 10 200 python3 -u tools/inflate_bench.py \
      --members 1024,2534,5068,16384 >> "$OUT/infl_$v.out" 2>> "$OUT/infl_$v.log"
  done
done
echo done
