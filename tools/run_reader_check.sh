#!/bin/bash
# GPU lane reader check: reader/inflate parity tests + CLI tests, then the
# reader alone under a kernel trace.   bash tools/run_reader_check.sh TAG
set -euo pipefail
T=${1:-reader}
bash tools/gpu_tests.sh "$T" tests/test_gpu_gz.py tests/test_cli.py
bash tools/gfastq_prof.sh "$T" 2000000 --with-pos
