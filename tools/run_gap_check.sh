#!/bin/bash
# Config-4-shape end to end: GPU suite subset, then the e2e run and its kernel
# trace (idle gaps between kernels, tools: python analysis offline).
set -euo pipefail
bash tools/gpu_tests.sh gap2 tests/test_gpu_parity.py tests/test_gpu_genome.py
VARIANTS="MSW_GPU_INFLATE=1" bash tools/gz_e2e.sh gap2/e2e 2000000 binned 6
