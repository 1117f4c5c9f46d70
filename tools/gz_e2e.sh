#!/bin/bash
# End to end at the config-4 shape on one GPU: host lane reader (libdeflate on
# the host CPUs) vs the GPU lane reader (inflate + parse on the GPU), same
# BGZF dataset; then a rocprofv3 kernel trace of the GPU-reader run.
#   bash tools/gz_e2e.sh TAG [reads_per_file] [qual] [level]
set -euo pipefail
T=${1:-gz_e2e}
N=${2:-500000}
Q=${3:-binned}
L=${4:-6}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
D=/tmp/msw_gz_e2e
timeout -k 10 500 python3 tools/wgs_e2e.py --dir $D --reads-per-file "$N" --bgzf --qual "$Q" --level "$L" \
  --workers 16 --host-threads 16 --extra-env "${VARIANTS:-MSW_GPU_INFLATE=0;MSW_GPU_INFLATE=1}" --out "$OUT/e2e.jsonl" \
  > "$OUT/e2e.log" 2>"$OUT/e2e.err"
echo "e2e done"
cp $D/reference.fa /tmp/ref_gz.fa
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o t --output-format csv -- \
  python3 tools/wgs_e2e.py --dir $D --reads-per-file "$N" --bgzf --reuse --host-threads 16 \
  --extra-env "MSW_GPU_INFLATE=1" --out "$OUT/e2e_prof.jsonl" > "$OUT/prof.log" 2>&1
echo "profile done"
