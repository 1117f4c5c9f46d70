#!/bin/bash
# Round-6 probe job on the box:  bash tools/r06_probe.sh TAG
# GPU lane reader tests, config 3 from FASTQ (two-group first spans vs the
# one-launch build), config 4 A/B, the host-to-host stream probes, default bench.
set -euo pipefail
export TMPDIR=/tmp
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gz.py tests/test_cli.py > $O/gputest_gz.log 2>&1
echo "gz tests: $(tail -1 $O/gputest_gz.log)"
timeout -k 10 300 python3 -u tools/c3f_env_ab.py --out $O/c3f_split_ab.jsonl --setting split= --setting nosplit=CLI=tools/bin/nosplit/rustseq_mini --reps 4 --sleep 1 > $O/c3f.log 2>&1
echo c3f ok
timeout -k 10 900 python3 -u tools/c4_env_ab.py --cli-b tools/bin/nosplit/rustseq_mini --reps 2 --out $O/c4_split_ab.jsonl > $O/c4.log 2>&1
echo c4 ok
timeout -k 10 120 python3 -u tools/stream_probe.py > $O/stream_probe.jsonl 2> $O/stream_probe.err
timeout -k 10 120 python3 -u tools/wait_probe.py > $O/wait_probe.json 2> $O/wait_probe.err
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/st -o st -- python3 -u tools/stream_probe.py --batches 200 > $O/stream_traced.jsonl 2> $O/stream_traced.err
echo stream ok
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err
echo done
