#!/bin/bash
# bash tools/fetch_calib.sh OUTDIR -- FETCH_SIZE of the two load patterns
set -euo pipefail
OUT=${1:-gpurun_out/fcal}; mkdir -p "$OUT"
# built here, on the CPU (the binary is not committed)
[ -x tools/fetch_calib ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/fetch_calib.hip -o tools/fetch_calib
for cfg in "vec16 160 13 12" "bytes 160 13 12" "vec16 256 10 16" "bytes 256 10 16" "bytes 256 5 16" "bytes 256 16 16"; do
  n=$(echo $cfg | tr ' ' '_')
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d "$OUT/$n" -o p --output-format csv -- ./tools/fetch_calib $cfg > "$OUT/$n.log" 2>&1
done
