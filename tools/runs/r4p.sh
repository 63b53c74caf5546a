#!/bin/bash
# plates-only rocprof kernel trace (fp32 plan) and the per-launch plate view
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
T=${PROF_TAG:-prof_plates}
mkdir -p gpurun_out/$T
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T -o run --output-format csv -- python3 bench.py --faces 0 --steps 5 --warmup 2 --no-cpu-baseline --compare "" --host-pipeline 0 --no-timing "$@" > gpurun_out/$T/bench.log 2>&1 || { tail -20 gpurun_out/$T/bench.log; exit 1; }
K=$(find gpurun_out/$T -name 'run_kernel_trace.csv' | head -1)
python tools/plate_layers.py "$K" > gpurun_out/$T/plates.txt 2>&1
cat gpurun_out/$T/plates.txt
grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/bench.log
