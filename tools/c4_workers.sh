#!/bin/bash
# Config 4 at full size: two GPU-reader workers on the GPU (default) vs four
# and six (MSW_DEVICES=0,0[,0] --num-gpus 2|3: more contexts' worth of workers on GPU 0),
# alternating, on the box:  bash tools/c4_workers.sh TAG
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
D=$(python3 -c "import sys; sys.path.insert(0, '.'); import bench; a = bench.parse([]); m = bench.ensure_c4_dataset(a); print(bench.c4_layout(a)[0])")
export WGS_DATA_DIR=$D WGS_SAMPLE_ID=SYN WGS_LANES=8 WGS_READS_PER_LANE=2 GPU_CHUNK_SIZE_READS=65536
for rep in 1 2 3; do
  for w in 2 4 6; do
    case $w in
      2) DEV="MSW_DEVICES=0"; NG=1 ;;
      4) DEV="MSW_DEVICES=0,0"; NG=2 ;;
      6) DEV="MSW_DEVICES=0,0,0"; NG=3 ;;
    esac
    env $DEV WGS_RUN_ID=w${w}_$rep timeout -k 10 120 mini_parallel_amd/rustseq_mini --full-wgs --gpu --score-mode sw \
      --reference $D/reference.fa --window 300 --checkpoint-dir /tmp --num-gpus $NG --json "$OUT/rec_w${w}_$rep.json" \
      > "$OUT/cli_w${w}_$rep.log" 2>&1
    python3 -c "import json; r = json.load(open('$OUT/rec_w${w}_$rep.json')); print(json.dumps({'workers': $w, 'rep': $rep, 'wall_ms': r['wall_ms'], 'reads_per_s': r['reads_per_second'], 'total_score': r['total_score']}))" >> "$OUT/workers.jsonl"
  done
done
echo done
