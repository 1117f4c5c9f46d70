#!/bin/bash
# long-pair tests + bench, then the inflate event counters (MSW_GZ_PROFILE build)
set -euo pipefail
bash tools/gpu_tests.sh long4 tests/test_gpu_long.py
timeout -k 10 300 python3 tools/long_bench.py > gpurun_out/long4/long_bench.jsonl 2> gpurun_out/long4/long_bench.err
mkdir -p gpurun_out/gzprof
MSW_GZ_PROFILE=1 MSW_GZ_TIMING=1 MSW_LIB_PATH=tools/_variants/libmsw_gzprof.so timeout -k 10 300 \
  python3 tools/inflate_bench.py --qual binned --level 6 --members 1,16384 > gpurun_out/gzprof/binned_l6.log 2>&1
MSW_GZ_TIMING=1 timeout -k 10 300 python3 tools/inflate_bench.py --qual binned --level 6 --members 16384 \
  > gpurun_out/gzprof/binned_l6_base.log 2>&1
echo done
