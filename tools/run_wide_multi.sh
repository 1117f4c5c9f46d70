#!/bin/bash
# KR 17..24 buckets in one launch: long GPU tests + the mixed 75..384 case,
# wide instance vs one launch per bucket (MSW_NO_WIDE_MULTI).
set -euo pipefail
OUT=gpurun_out/widemulti
bash tools/gpu_tests.sh widemulti tests/test_gpu_long.py tests/test_gpu_parity.py
for v in on off on2 off2; do
  case $v in off*) export MSW_NO_WIDE_MULTI=1;; *) unset MSW_NO_WIDE_MULTI;; esac
  timeout -k 10 300 python3 tools/long_bench.py --only mixed_ > $OUT/long_bench_$v.jsonl 2>$OUT/long_bench_$v.err
  echo "$v done"
done
