#!/bin/bash
# Group width at large batches: config-2 shape, 1M pairs, auto vs forced G.
set -euo pipefail
OUT=gpurun_out/gsweep
mkdir -p $OUT
export TMPDIR=/tmp
for g in ${GS:-auto 10 12 15 16}; do
  if [ $g = auto ]; then unset MSW_GROUP_LANES MSW_LAYOUT; else export MSW_LAYOUT=pairs MSW_GROUP_LANES=$g; fi
  timeout -k 10 300 python3 bench.py --pairs 1000000 --steps 10 --warmup 2 --cpu-seconds 0 --no-pcie \
    --extra-configs none > $OUT/g_$g.json 2> $OUT/g_$g.err
  python3 -c "import json;d=json.load(open('$OUT/g_$g.json'));print('$g', d['value'], d['ms_per_step'], d['parity']['bit_exact'] if d.get('parity') else None)"
done
