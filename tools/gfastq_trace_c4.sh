set -e
D=$(python3 -c "import sys; sys.path.insert(0, '.'); import bench; a = bench.parse([]); m = bench.ensure_c4_dataset(a); print(bench.c4_layout(a)[0])")
export WGS_DATA_DIR=$D WGS_SAMPLE_ID=SYN WGS_LANES=8 WGS_READS_PER_LANE=2 GPU_CHUNK_SIZE_READS=65536
mkdir -p gpurun_out/r04m
for i in 1 2; do
WGS_RUN_ID=gt_$i MSW_GFASTQ_TRACE=1 timeout -k 10 120 mini_parallel_amd/rustseq_mini --full-wgs --gpu --score-mode sw --reference $D/reference.fa --window 300 --checkpoint-dir /tmp --json gpurun_out/r04m/rec_$i.json > gpurun_out/r04m/cli_$i.log 2> gpurun_out/r04m/trace_$i.log
done
