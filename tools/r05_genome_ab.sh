#!/bin/bash
# Round 5, windows read from the resident genome by the scoring kernels: GPU
# tests, the host-to-host stream, config 4 with and without the cut launch
# (alternating), and a kernel trace of config 3 from FASTQ.
#   bash tools/r05_genome_ab.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_tests.sh "$T"
timeout -k 10 200 python3 -u tools/stream_probe.py --trace > "$OUT/stream_genome.jsonl" 2> "$OUT/stream_genome.err"
MSW_GENOME_CUT=1 timeout -k 10 200 python3 -u tools/stream_probe.py --trace > "$OUT/stream_cut.jsonl" 2> "$OUT/stream_cut.err"
timeout -k 10 400 python3 -u tools/c4_env_ab.py --b MSW_GENOME_CUT=1 --reps 3 --out "$OUT/c4_genome_vs_cut.jsonl"
bash tools/c3f_kernel_trace.sh "$T"
echo done
