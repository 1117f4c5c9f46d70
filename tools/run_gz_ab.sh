#!/bin/bash
# GPU inflate A/B: gz parity tests on the in-tree build, then inflate
# throughput (16k members) and SALU/VALU/branch counts per variant library.
#   bash tools/run_gz_ab.sh TAG [variant ...]   (variants: tools/_variants/libmsw_NAME.so)
set -euo pipefail
T=${1:-gz_ab}
shift || true
bash tools/gpu_tests.sh "$T" tests/test_gpu_gz.py
export TMPDIR=/tmp
for v in base "$@"; do
  lib=""
  [ "$v" != base ] && lib=tools/_variants/libmsw_$v.so
  MSW_LIB_PATH=$lib MSW_GZ_TIMING=1 timeout -k 10 300 python3 tools/inflate_bench.py --qual binned --level 6 \
    --members 16384 > gpurun_out/$T/inflate_${v}.log 2>&1
  MSW_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_WAVES \
    -d gpurun_out/$T/pmc_$v -o p --output-format csv -- python3 tools/inflate_bench.py --qual binned --level 6 \
    --members 16384 > gpurun_out/$T/pmc_${v}.log 2>&1
  echo "$v: $(grep -h '16384 members' gpurun_out/$T/inflate_${v}.log | tail -1)"
done
