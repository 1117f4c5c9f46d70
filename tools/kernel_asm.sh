#!/bin/bash
# ISA of one SW kernel instance, fast (one template instance, not the whole
# instance set): tools/kernel_asm.sh KR AFFINE COORDS SPLIT OUT.s [hipcc -D...]
# e.g. tools/kernel_asm.sh 13 false false false /tmp/k13.s; then
#      python3 tools/loop_mix.py /tmp/k13.s   (instruction mix + s_nop of the DP loops)
set -euo pipefail
KR=$1; AFF=$2; CO=$3; SP=$4; OUT=$5; shift 5
SRC=$(cd "$(dirname "$0")/../mini_parallel_amd/csrc" && pwd)
TMP=$(mktemp --suffix=.hip)
cat > "$TMP" <<EOT

#include "$SRC/msw_device.h"
template __global__ void msw::sw_kernel<$KR, $AFF, $CO, $SP>(msw::SwParams);
EOT
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I"$SRC/../../include" -I"$SRC" --cuda-device-only -S "$TMP" -o "$OUT" "$@" 2>/dev/null
rm -f "$TMP"
