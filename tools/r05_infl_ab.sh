#!/bin/bash
# Round 5: an inflate kernel change against the build of the commit before
# it (tools/_ab/infl_old/libmsw.so: the same tree with the previous
# msw_inflate.hip, tools/build_variant.sh).  GPU gz
# tests, inflate kernel times (MSW_GZ_TIMING), config 3 from FASTQ and
# config 4, old and new alternating.   bash tools/r05_infl_ab.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
OLD="$PWD/tools/_ab/infl_old"
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_gz.py \
  > "$OUT/gz_tests.log" 2>&1
echo "gz tests: $(tail -1 "$OUT/gz_tests.log")"
for rep in 1 2 3; do
  MSW_GZ_TIMING=1 timeout -k 10 200 python3 -u tools/inflate_bench.py --members 2534,5068,16384 \
    >> "$OUT/infl_new.out" 2>> "$OUT/infl_new.log"
  MSW_LIB_PATH="$OLD/libmsw.so" MSW_GZ_TIMING=1 timeout -k 10 200 python3 -u tools/inflate_bench.py \
    --members 2534,5068,16384 >> "$OUT/infl_old.out" 2>> "$OUT/infl_old.log"
done
timeout -k 10 300 python3 -u tools/c3f_env_ab.py --out "$OUT/c3f_ab.jsonl" --reps 3 \
  --setting new= --setting "old=LD_LIBRARY_PATH=$OLD:${LD_LIBRARY_PATH:-}" > "$OUT/c3f_ab.log" 2>&1
timeout -k 10 400 python3 -u tools/c4_env_ab.py --b "LD_LIBRARY_PATH=$OLD:${LD_LIBRARY_PATH:-}" --reps 3 \
  --out "$OUT/c4_ab.jsonl" > "$OUT/c4_ab.log" 2>&1
echo done
