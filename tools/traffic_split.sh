#!/bin/bash
# Split the scoring kernels' HBM reads by buffer, on the box:
#   bash tools/traffic_split.sh TAG
# Variants (built here beforehand by tools/build_variant.sh):
#   base    mini_parallel_amd/libmsw.so
#   nowin   -DMSW_PROBE_NO_WIN=1   window loads replaced by constants
#   noread  -DMSW_PROBE_NO_READ=1  read-byte loads replaced by constants
# For configs 2 and 5: one FETCH_SIZE pass per variant, plus WRITE_SIZE and the
# 64 B / 32 B read-request split for the base build.  Each pass is a short bench
# run (no CPU baseline, no host-to-host legs).  tools/traffic_split.py summarises.
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in 2 5; do
  case $cfg in
    2) A="--steps 50 --warmup 5" ;;
    5) A="--steps 20 --warmup 3" ;;
  esac
  B="python3 bench.py --config $cfg $A --cpu-seconds 0 --no-pcie --extra-configs none"
  for v in base nowin noread; do
    lib=$PWD/mini_parallel_amd/libmsw.so
    [ "$v" = base ] || lib=$PWD/tools/_variants/libmsw_$v.so
    MSW_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c${cfg}_$v/fetch" -o p --output-format csv \
      -- $B > "$OUT/c${cfg}_$v.fetch.log" 2>&1
  done
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c${cfg}_base/write" -o p --output-format csv \
    -- $B > "$OUT/c${cfg}_base.write.log" 2>&1
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d "$OUT/c${cfg}_base/req" -o p \
    --output-format csv -- $B > "$OUT/c${cfg}_base.req.log" 2>&1
  echo "config $cfg traffic split done"
done
