#!/bin/bash
# A/B builds of the kernel library: tools/build_variant.sh NAME [hipcc -D flags...]
# -> tools/_variants/libmsw_NAME.so (load with MSW_LIB_PATH=...; tools/sweep.py,
# tools/lever_probe.py).  The kernel units compile in parallel.
set -euo pipefail
cd "$(dirname "$0")/../mini_parallel_amd/csrc"
NAME=$1; shift
OUT=../../tools/_variants
mkdir -p "$OUT/o_$NAME"
make -s msw_runtime.o msw_fastq.o msw_gfastq.o >/dev/null
pids=()
for f in msw_kernels.hip msw_launch_*.hip msw_long.hip msw_inflate.hip msw_parse.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include "$@" -c "$f" \
      -o "$OUT/o_$NAME/${f%.hip}.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -lz -lpthread -ldl "$OUT/o_$NAME"/*.o msw_runtime.o msw_fastq.o msw_gfastq.o \
    -o "$OUT/libmsw_$NAME.so"
rm -rf "$OUT/o_$NAME"
