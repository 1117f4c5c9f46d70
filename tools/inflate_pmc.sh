#!/bin/bash
# Where gz_inflate_kernel's wave cycles go (SQ counters, one pass per group,
# each pass its own run of tools/inflate_bench.py), on the box:
#   bash tools/inflate_pmc.sh TAG [MEMBERS]
# -> gpurun_out/TAG/inflate_pmc/: the gfx950 counter list and pass<k>/ CSVs;
# tools/pmc_inflate_summary.py folds them into per-launch sums.
set -euo pipefail
T=${1:?tag}
M=${2:-16384}
OUT=gpurun_out/$T/inflate_pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM"
k=0
for P in "$P1" "$P2"; do
  k=$((k + 1))
  # shellcheck disable=SC2086
  timeout -s KILL 120 rocprofv3 --pmc $P -d "$OUT/pass$k" -o p --output-format csv -- \
    python3 tools/inflate_bench.py --members "$M" > "$OUT/pass$k.log" 2>&1
done
python3 tools/pmc_inflate_summary.py "$OUT" > "$OUT/summary.json"
cat "$OUT/summary.json"
