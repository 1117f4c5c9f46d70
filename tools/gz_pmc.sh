#!/bin/bash
# Instruction mix and HBM traffic of the inflate / CRC kernels (rocprofv3 PMC
# passes over tools/inflate_bench.py, one launch of MEMBERS members), plus a
# kernel-trace summary of the same command.   bash tools/gz_pmc.sh TAG MEMBERS
set -euo pipefail
T=${1:-gzpmc}
M=${2:-16384}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 tools/inflate_bench.py --members $M"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o k --output-format csv -- $B > "$OUT/kt.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d "$OUT/p1" -o p --output-format csv -- $B > "$OUT/p1.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU -d "$OUT/p2" -o p --output-format csv -- $B > "$OUT/p2.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/p3" -o p --output-format csv -- $B > "$OUT/p3.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/p4" -o p --output-format csv -- $B > "$OUT/p4.log" 2>&1
echo pmc done
