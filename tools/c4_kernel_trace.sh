#!/bin/bash
# rocprofv3 kernel trace of BASELINE config 4 at its stated size (bench.py's
# 16 lane files x 25 M reads, GPU lane reader, score-only) through the
# --full-wgs driver, on the box:
#   bash tools/c4_kernel_trace.sh TAG
# -> gpurun_out/TAG/c4trace/: kernel_stats.csv (per-kernel totals), the run
# record, split.json (GPU time per kernel family, the busy union and the
# run's wall; tools/trace_split.py), gaps.txt (the largest idle gaps,
# tools/trace_timeline.py) and the per-dispatch trace (kernel_trace.csv.gz).
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T/c4trace
mkdir -p "$OUT"
export TMPDIR=/tmp
D=$(python3 -c "import sys; sys.path.insert(0, '.'); import bench; a = bench.parse([]); bench.ensure_c4_dataset(a); print(bench.c4_layout(a)[0])")
L=$(python3 -c "import sys; sys.path.insert(0, '.'); import bench; print(bench.C4_LANES, bench.C4_READS_PER_LANE, bench.C4_WINDOW)")
read -r LANES RPL WIN <<< "$L"
export WGS_DATA_DIR=$D WGS_SAMPLE_ID=SYN WGS_LANES=$LANES WGS_READS_PER_LANE=$RPL GPU_CHUNK_SIZE_READS=65536
export MSW_GPU_INFLATE=1 WGS_RUN_ID=c4trace_$$
W=/tmp/c4trace_$$
mkdir -p "$W"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$W/prof" -o t --output-format csv -- \
  mini_parallel_amd/rustseq_mini --full-wgs --gpu --score-mode sw --reference "$D/reference.fa" --window "$WIN" \
  --checkpoint-dir "$W" --json "$OUT/rec.json" > "$OUT/cli.log" 2>&1
KT=$(find "$W/prof" -name '*kernel_trace.csv' | head -1)
KS=$(find "$W/prof" -name '*kernel_stats.csv' | head -1)
cp "$KS" "$OUT/kernel_stats.csv"
python3 tools/trace_split.py "$KT" --record "$OUT/rec.json" > "$OUT/split.json"
python3 tools/trace_timeline.py "$KT" --min-ms 1e9 > "$OUT/gaps.txt"
gzip -c "$KT" > "$OUT/kernel_trace.csv.gz"
rm -rf "$W"
cat "$OUT/split.json" "$OUT/gaps.txt"
