#!/bin/bash
# Host feed of the config-4 GPU lane reader, on the box:
#   bash tools/host_feed.sh TAG
# 1. a bench config-4 lane set (16 BGZF files x 2 M reads, segments of 1 M), generated once
# 2. tools/host_feed: page cache -> pinned staging copy rate, S streams x T threads,
#    no GPU work; hipHostRegister of the mmap'ed files as the zero-copy alternative
# 3. the --full-wgs driver on all 16 files and on a 2-file shard (the per-rank
#    share at N = 8); the run records carry the setup phases (setup_phases)
set -euo pipefail
T=${1:?tag}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
D=$(timeout -k 10 600 python3 -c "
import sys; sys.argv=['bench.py']; import bench
a = bench.parse(['--c4-reads-per-file', '2000000'])
print(bench.ensure_c4_dataset(a), file=sys.stderr); print(bench.c4_layout(a)[0])" 2> "$OUT/gen.log")
timeout -k 10 300 ./tools/host_feed "$OUT/host_feed.jsonl" $D/SYN_L00*_R*_001.fastq.gz > "$OUT/host_feed.log" 2>&1
echo "host_feed: $(wc -l < "$OUT/host_feed.jsonl") lines"
for shard in "" 0/8 0/4 0/2; do
  name=all; [ -n "$shard" ] && name=shard_${shard/\//of}
  for rep in 1 2; do
    env WGS_DATA_DIR=$D WGS_SAMPLE_ID=SYN WGS_LANES=8 WGS_READS_PER_LANE=2 GPU_CHUNK_SIZE_READS=65536 \
      WGS_FILE_SHARD=$shard WGS_RUN_ID=hf_${name}_$rep \
      timeout -k 10 300 ./mini_parallel_amd/rustseq_mini --full-wgs --gpu --score-mode sw --reference $D/reference.fa \
      --window 300 --checkpoint-dir /tmp --json "$OUT/rec_${name}_$rep.json" > "$OUT/cli_${name}_$rep.log" 2> "$OUT/cli_${name}_$rep.err"
    echo "$name $rep: $(python3 -c "import json;d=json.load(open('$OUT/rec_${name}_$rep.json'));print(d['total_reads'], round(d['wall_ms'],1), round(d['setup_ms'],1), round(d['teardown_ms'],1), round(d['reads_per_second']/1e6,1))")"
  done
done
