#!/bin/bash
# Attribute config 2's non-sequence HBM reads (the "rest"
# after reads and windows), on the box:   bash tools/traffic_rest.sh TAG
# Variants (built here beforehand):
#   base        mini_parallel_amd/libmsw.so
#   noio        tools/build_variant.sh noio -DMSW_PROBE_NO_WIN=1 -DMSW_PROBE_NO_READ=1
#   noio_nolen  tools/build_variant.sh noio_nolen -DMSW_PROBE_NO_WIN=1 -DMSW_PROBE_NO_READ=1 -DMSW_PROBE_CONST_LEN=1
# noio fetches lengths + everything that is not pair data; noio_nolen only the
# latter (code, kernel arguments); one FETCH_SIZE pass each, plus the 64 B /
# 32 B request split of noio_nolen.  Summarised by tools/traffic_split.py rest TAG.
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --config 2 --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie --extra-configs none"
for v in base noio noio_nolen; do
  lib=$PWD/mini_parallel_amd/libmsw.so
  [ "$v" = base ] || lib=$PWD/tools/_variants/libmsw_$v.so
  MSW_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/rest_$v/fetch" -o p --output-format csv \
    -- $B > "$OUT/rest_$v.fetch.log" 2>&1
done
MSW_LIB_PATH=$PWD/tools/_variants/libmsw_noio_nolen.so timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum \
  TCC_EA0_RDREQ_32B_sum -d "$OUT/rest_noio_nolen/req" -o p --output-format csv -- $B > "$OUT/rest_noio_nolen.req.log" 2>&1
echo "traffic rest split done"
