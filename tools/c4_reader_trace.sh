#!/bin/bash
# Config 4 at its stated size through the --full-wgs driver with the reader's
# per-span phase times (MSW_GFASTQ_TRACE) and the CLI's per-batch times
# (MSW_CLI_TRACE) on stderr, then tools/reg_dma_probe on one lane file:
#   bash tools/c4_reader_trace.sh TAG  -> gpurun_out/TAG/c4reader/
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T/c4reader
mkdir -p "$OUT"
export TMPDIR=/tmp
D=$(python3 -c "import sys; sys.path.insert(0, '.'); import bench; a = bench.parse([]); bench.ensure_c4_dataset(a); print(bench.c4_layout(a)[0])")
L=$(python3 -c "import sys; sys.path.insert(0, '.'); import bench; print(bench.C4_LANES, bench.C4_READS_PER_LANE, bench.C4_WINDOW)")
read -r LANES RPL WIN <<< "$L"
W=/tmp/c4reader_$$
mkdir -p "$W"
WGS_DATA_DIR=$D WGS_SAMPLE_ID=SYN WGS_LANES=$LANES WGS_READS_PER_LANE=$RPL GPU_CHUNK_SIZE_READS=65536 \
  MSW_GPU_INFLATE=1 WGS_RUN_ID=c4reader_$$ MSW_GFASTQ_TRACE=1 MSW_CLI_TRACE=1 \
  timeout -k 10 120 mini_parallel_amd/rustseq_mini --full-wgs --gpu --score-mode sw --reference "$D/reference.fa" \
  --window "$WIN" --checkpoint-dir "$W" --json "$OUT/rec.json" > "$OUT/cli.out" 2> "$OUT/cli.err"
rm -rf "$W"
F=$(python3 -c "import sys; sys.path.insert(0, '.'); import bench; a = bench.parse([]); print(bench.c4_layout(a)[1][0])")
timeout -k 10 120 tools/bin/reg_dma_probe "$F" 290 > "$OUT/reg_dma_probe.jsonl" 2>&1
cat "$OUT/reg_dma_probe.jsonl"
