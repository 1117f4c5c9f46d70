set -e
mkdir -p gpurun_out/r03z
for rep in 1 2; do
 for lib in "" "$PWD/tools/_variants/libmsw_cs1.so"; do
  echo "== ${lib:-in-tree} rep $rep" >> gpurun_out/r03z/h2h.jsonl
  MSW_LIB_PATH=$lib timeout -k 10 200 python3 tools/h2h_sweep.py --chunks 65536,131072 >> gpurun_out/r03z/h2h.jsonl 2>>gpurun_out/r03z/h2h.err
 done
done
