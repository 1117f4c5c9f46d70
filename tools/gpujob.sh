#!/bin/bash
# One parametrised GPU job (replaces the round-1/2 tools/run_*.sh wrappers):
#   bash tools/gpujob.sh TAG STEP [STEP ...]
# Steps run in order, each under its own time limit; the first failure ends
# the job (set -e), so nothing runs on the GPU after a fault or a kill.
#   tests[=PYTEST_PATHS]   pytest -m gpu (default: tests), log gpurun_out/TAG/gputest.log
#   smoke                  __graft_entry__.smoke()
#   bench[=ARGS]           python3 bench.py ARGS > gpurun_out/TAG/bench.json
#   prof                   rocprofv3 --kernel-trace --stats of the config-2 bench (gpurun_out/TAG/prof_c2)
#   e2e[=ENVSETS]          tools/wgs_e2e.py over the config-4-shape BGZF set (16 x 2 M reads, binned, level 6);
#                          ENVSETS as wgs_e2e.py --extra-env (default MSW_GPU_INFLATE=1)
#   longbench              tools/long_bench.py
#   sys                    df / free / CPU quota of the box (disk and memory for the full-size config-4 set)
#   c4full[=READS]         tools/c4_full.py: BASELINE config 4 at full size (16 files x READS, default 25 M)
#   ab=VARIANT             bench configs 2 / 3 / 5 (kernel-only), in-tree build vs tools/_variants/libmsw_VARIANT.so,
#                          alternating, 3 rounds -> gpurun_out/TAG/ab_VARIANT.jsonl
#   gzab=VARIANT           GPU inflate, in-tree build vs tools/_variants/libmsw_VARIANT.so, alternating, 3 rounds:
#                          tools/inflate_bench.py at 16384 members (fastq, binned, level 6), MSW_GZ_TIMING kernel times
#   traffic                tools/traffic_split.sh (FETCH_SIZE of the probe builds, configs 2 and 5)
#   hostfeed               tools/host_feed.sh (config-4 host feed: copy rates, CLI runs with setup traced)
#   c3fab=SETTINGS         tools/c3f_env_ab.py, SETTINGS = ';'-separated NAME=VAR=VAL,... (CLI=path: another
#                          build), 4 alternating rounds, 1 s idle between runs -> c3f_ab.jsonl
#   c3ftrace[=CLI]         tools/c3f_kernel_trace.sh (kernel trace of config 3 from FASTQ; CLI: another build)
#   c4ab=CLI               tools/c4_env_ab.py, the in-tree CLI against another build, 2 rounds -> c4_ab.jsonl
#   c4trace                tools/c4_kernel_trace.sh (kernel trace of config 4 at full size, GPU time per kernel family)
#   stream                 tools/stream_probe.py + tools/wait_probe.py (10k-pair host-to-host stream), and the
#                          same probe under a kernel + memory-copy trace (stream_trace/)
# Example: gpurun --timeout 1200 -- bash tools/gpujob.sh r03a tests smoke bench prof
set -euo pipefail
T=${1:?tag}
shift
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  name=${step%%=*}
  arg=""
  [[ "$step" == *=* ]] && arg=${step#*=}
  case "$name" in
    tests)
      # shellcheck disable=SC2086
      bash tools/gpu_tests.sh "$T" ${arg:-tests} ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      echo "smoke: $(tail -1 "$OUT/smoke.log")" ;;
    bench)
      # shellcheck disable=SC2086
      timeout -k 10 600 python3 bench.py $arg > "$OUT/bench.json" 2> "$OUT/bench.err"
      echo "bench: $(head -c 300 "$OUT/bench.json")" ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o t --output-format csv -- \
        python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie --extra-configs none \
        > "$OUT/prof_c2.log" 2>&1
      echo "prof ok" ;;
    e2e)
      timeout -k 10 900 python3 tools/wgs_e2e.py --dir /tmp/msw_gz_e2e --reads-per-file 2000000 --bgzf \
        --qual binned --level 6 --workers 16 --host-threads 16 --extra-env "${arg:-MSW_GPU_INFLATE=1}" \
        --out "$OUT/e2e.jsonl" > "$OUT/e2e.log" 2> "$OUT/e2e.err"
      echo "e2e: $(grep -o '"throughput_reads_per_second": [0-9.]*' "$OUT/e2e.jsonl" | tr '\n' ' ')" ;;
    longbench)
      timeout -k 10 300 python3 tools/long_bench.py > "$OUT/long_bench.jsonl" 2> "$OUT/long_bench.err"
      echo "longbench ok" ;;
    sys)
      { df -h /tmp /dev/shm; free -g; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true; } > "$OUT/sys.txt" 2>&1
      cat "$OUT/sys.txt" ;;
    c4full)
      timeout -k 10 1100 python3 tools/c4_full.py --reads-per-file "${arg:-25000000}" \
        --out "$OUT/config4_full.jsonl" > "$OUT/c4full.log" 2>&1
      tail -5 "$OUT/c4full.log" ;;
    ab)
      for rep in 1 2 3; do
        for lib in "" "$PWD/tools/_variants/libmsw_$arg.so"; do
          for cfg in 2 3 5; do
            MSW_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --config $cfg --steps 50 --warmup 5 --cpu-seconds 0 \
              --no-pcie --extra-configs none > "$OUT/ab_tmp.json" 2>> "$OUT/ab.err"
            python3 -c "import json,sys; d=json.load(open('$OUT/ab_tmp.json')); print(json.dumps({'lib': '${lib:-in-tree}', 'config': $cfg, 'rep': $rep, 'value': d['value'], 'avg_launch_ms': d['roofline']['avg_launch_ms'], 'bit_exact': (d.get('parity') or {}).get('bit_exact')}))" >> "$OUT/ab_$arg.jsonl"
          done
        done
      done
      cat "$OUT/ab_$arg.jsonl" ;;
    gzab)
      for rep in 1 2 3; do
        for lib in "" "$PWD/tools/_variants/libmsw_$arg.so"; do
          echo "== lib ${lib:-in-tree} rep $rep" >> "$OUT/gzab_$arg.log"
          MSW_LIB_PATH=$lib MSW_GZ_TIMING=1 timeout -k 10 300 python3 tools/inflate_bench.py --members 16384 \
            >> "$OUT/gzab_$arg.log" 2>&1
        done
      done
      grep -E "==|members|inflate" "$OUT/gzab_$arg.log" | tail -40 ;;
    traffic)
      bash tools/traffic_split.sh "$T/traffic" ;;
    hostfeed)
      bash tools/host_feed.sh "$T/hostfeed" ;;
    c3fab)
      sets=()
      IFS=';' read -ra parts <<< "$arg"
      for p in "${parts[@]}"; do sets+=(--setting "$p"); done
      timeout -k 10 400 python3 -u tools/c3f_env_ab.py --out "$OUT/c3f_ab.jsonl" "${sets[@]}" --reps 4 --sleep 1 \
        > "$OUT/c3f_ab.log" 2>&1
      echo "c3fab ok" ;;
    c3ftrace)
      bash tools/c3f_kernel_trace.sh "$T/trace_${arg//\//_}" "--kernel-trace --stats" "${arg:-mini_parallel_amd/rustseq_mini}" ;;
    c4ab)
      timeout -k 10 900 python3 -u tools/c4_env_ab.py --cli-b "$arg" --reps 2 --out "$OUT/c4_ab.jsonl" > "$OUT/c4_ab.log" 2>&1
      echo "c4ab ok" ;;
    c4trace)
      bash tools/c4_kernel_trace.sh "$T" ;;
    stream)
      timeout -k 10 120 python3 -u tools/stream_probe.py > "$OUT/stream_probe.jsonl" 2> "$OUT/stream_probe.err"
      timeout -k 10 120 python3 -u tools/wait_probe.py > "$OUT/wait_probe.json" 2> "$OUT/wait_probe.err"
      timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/stream_trace" -o st \
        -- python3 -u tools/stream_probe.py --batches 200 > "$OUT/stream_traced.jsonl" 2> "$OUT/stream_traced.err"
      cat "$OUT/stream_probe.jsonl" ;;
    *)
      echo "unknown step $name" >&2; exit 2 ;;
  esac
done
