#!/bin/bash
# Kernel trace of BASELINE config 4 at its stated size (bench.py's lane set,
# 400 M reads) through the --full-wgs driver on one GPU, on the box:
#   bash tools/c4_trace.sh TAG
# -> gpurun_out/TAG/trace/*kernel_trace.csv, *kernel_stats.csv + the run record;
# tools/trace_timeline.py summarises busy time and the kernels' shares.
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
D=$(python3 -c "import sys; sys.path.insert(0, '.'); import bench; a = bench.parse([]); m = bench.ensure_c4_dataset(a); print(bench.c4_layout(a)[0])")
export WGS_DATA_DIR=$D WGS_SAMPLE_ID=SYN WGS_LANES=8 WGS_READS_PER_LANE=2 GPU_CHUNK_SIZE_READS=65536 WGS_RUN_ID=c4trace_$$
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o t --output-format csv -- \
  mini_parallel_amd/rustseq_mini --full-wgs --gpu --score-mode sw --reference "$D/reference.fa" --window 300 \
  --checkpoint-dir /tmp --json "$OUT/rec.json" > "$OUT/cli.log" 2>&1
echo "config-4 trace done"
