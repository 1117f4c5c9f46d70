#!/bin/bash
# rocprofv3 trace of BASELINE config 3 from FASTQ (bench.py's lane set at
# N = 1: one lane's R1/R2 BGZF files of 500k reads, affine + best cell,
# per-read records) through the --full-wgs driver, on the box:
#   bash tools/c3f_kernel_trace.sh TAG [TRACE_FLAGS] [CLI]
# TRACE_FLAGS default "--kernel-trace --stats" ("--hip-trace --kernel-trace
# --memory-copy-trace" for the setup's API calls); CLI default the in-tree
# rustseq_mini.  -> gpurun_out/TAG/c3f/trace<k>/ + run record + reader span
# trace; tools/trace_timeline.py shows where the timed region goes.
set -euo pipefail
T=${1:?tag}
FLAGS=${2:---kernel-trace --stats}
CLI=${3:-mini_parallel_amd/rustseq_mini}
OUT=gpurun_out/$T/c3f
mkdir -p "$OUT"
export TMPDIR=/tmp
D=$(python3 -c "import sys; sys.path.insert(0, '.'); import bench; a = bench.parse([]); bench.ensure_c3f_dataset(a, 1); print(bench.c3f_layout(a, 1)[0])")
export WGS_DATA_DIR=$D WGS_SAMPLE_ID=SYN WGS_LANES=1 WGS_READS_PER_LANE=2 GPU_CHUNK_SIZE_READS=65536
export MSW_GFASTQ_TRACE=1 MSW_CLI_TRACE=1
for k in 1 2; do
  W=$(mktemp -d /tmp/c3ftr_XXXX)
  # shellcheck disable=SC2086
  WGS_RUN_ID=c3ftrace_$$_$k timeout -k 10 120 rocprofv3 $FLAGS -d "$OUT/trace$k" -o t --output-format csv -- \
    "$CLI" --full-wgs --gpu --score-mode sw --reference "$D/reference.fa" --window 300 \
    --gap-model affine --scores-out "$W" --checkpoint-dir "$W" --json "$OUT/rec$k.json" > "$OUT/cli$k.log" 2>&1
  rm -rf "$W"
  sleep 2
done
echo "config-3 FASTQ trace done"
