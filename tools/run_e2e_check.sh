set -euo pipefail
mkdir -p gpurun_out/e2e_nocoords
timeout -k 10 300 python3 -u -m pytest tests/test_cli.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e2e_nocoords/test_cli.log 2>&1
echo "cli tests: $(tail -1 gpurun_out/e2e_nocoords/test_cli.log)"
VARIANTS="MSW_GPU_INFLATE=1;MSW_GPU_INFLATE=0" bash tools/gz_e2e.sh e2e_nocoords 2000000 binned 6
