#!/bin/bash
# Round 5: device -> pinned host copies as kernels on the caller's stream.
# GPU tests, then config 3 from FASTQ and config 4 with the copies as kernels
# (default) against DMA copies (MSW_D2H_DMA=1), alternating; a config-3
# kernel trace.   bash tools/r05_d2h.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "memcpy_d2h or ctx_prepare" > "$OUT/d2h_tests.log" 2>&1
echo "d2h tests: $(tail -1 "$OUT/d2h_tests.log")"
bash tools/gpu_tests.sh "$T"
timeout -k 10 300 python3 -u tools/c3f_env_ab.py --out "$OUT/c3f_ab.jsonl" --reps 4 \
  --setting kernel_copy= --setting dma=MSW_D2H_DMA=1 > "$OUT/c3f_ab.log" 2>&1
bash tools/c3f_kernel_trace.sh "$T"
timeout -k 10 400 python3 -u tools/c4_env_ab.py --b MSW_D2H_DMA=1 --reps 3 --out "$OUT/c4_ab.jsonl" \
  > "$OUT/c4_ab.log" 2>&1
echo done
