#!/bin/bash
# Config 5's HBM reads split by buffer (traffic_over_alg
# 1.33 for sw_multi_kernel), on the box:   bash tools/traffic_c5_split.sh TAG
# Variants (built here beforehand by tools/build_variant.sh):
#   base    mini_parallel_amd/libmsw.so
#   nowin   -DMSW_PROBE_NO_WIN=1                      window loads are constants
#   noread  -DMSW_PROBE_NO_READ=1                     read-byte loads are constants
#   noio    -DMSW_PROBE_NO_WIN=1 -DMSW_PROBE_NO_READ=1  only lengths, slot order, code, arguments
# One FETCH_SIZE pass per variant, the 64 B / 32 B request split of each, and
# WRITE_SIZE of the base build; each pass a short planned config-5 bench run.
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --config 5 --steps 20 --warmup 3 --cpu-seconds 0 --no-pcie --extra-configs none"
for v in base nowin noread noio; do
  lib=$PWD/mini_parallel_amd/libmsw.so
  [ "$v" = base ] || lib=$PWD/tools/_variants/libmsw_$v.so
  MSW_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c5_$v/fetch" -o p --output-format csv \
    -- $B > "$OUT/c5_$v.fetch.log" 2>&1
  MSW_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d "$OUT/c5_$v/req" \
    -o p --output-format csv -- $B > "$OUT/c5_$v.req.log" 2>&1
done
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c5_base/write" -o p --output-format csv \
  -- $B > "$OUT/c5_base.write.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c5_base/trace" -o t --output-format csv \
  -- $B > "$OUT/c5_base.trace.log" 2>&1
echo "config-5 traffic split done"
