#!/bin/bash
# A/B builds of the kernel library: tools/build_variant.sh NAME [hipcc -D flags...]
# -> tools/_variants/libmsw_NAME.so (load with MSW_LIB_PATH=...; tools/sweep.py)
set -euo pipefail
cd "$(dirname "$0")/../mini_parallel_amd/csrc"
NAME=$1; shift
OUT=../../tools/_variants
mkdir -p "$OUT"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include "$@" -c msw_kernels.hip -o "$OUT/k_$NAME.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -lz -lpthread "$OUT/k_$NAME.o" msw_runtime.o msw_fastq.o -o "$OUT/libmsw_$NAME.so"
rm -f "$OUT/k_$NAME.o"
