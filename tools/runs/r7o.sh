#!/bin/bash
# letterbox pair kernel with exact-gather fast path (columns and rows with weights (1, 0)): exactness tests, rocprof, headline x2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r7o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_plates.py tests/test_gpu_configs.py tests/test_gpu_parity_fp32.py -k "letterbox or paired or configs or c3 or c2 or c5 or parity" > gpurun_out/r7o/tests.txt 2>&1 || { tail -40 gpurun_out/r7o/tests.txt; exit 1; }
tail -2 gpurun_out/r7o/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r7o/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing > gpurun_out/r7o/bench.json 2> gpurun_out/r7o/bench.err || { tail -5 gpurun_out/r7o/bench.err; exit 1; }
grep -h "letterbox" $(find gpurun_out/r7o/prof -name 'run_kernel_stats.csv') | cut -c1-200
for round in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing > gpurun_out/r7o/ab.json 2> gpurun_out/r7o/ab.err || { tail -5 gpurun_out/r7o/ab.err; exit 1; }
  echo "[new] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r7o/ab.json)"
done
