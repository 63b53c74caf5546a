#!/bin/bash
# rocprofv3 kernel trace + stats of the headline bench (PROF_TAG names the output dir;
# BARGS the bench arguments), then the per-kernel summary and the per-layer fp32 view.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
T=${PROF_TAG:-prof}
mkdir -p gpurun_out/$T
BARGS=${BARGS:-"--steps 5 --warmup 2 --no-cpu-baseline --compare '' --host-pipeline 0 --no-timing"}
eval timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$T -o run --output-format csv -- python3 bench.py $BARGS > gpurun_out/$T/bench.log 2>&1 || { tail -20 gpurun_out/$T/bench.log; exit 1; }
S=$(find gpurun_out/$T -name 'run_kernel_stats.csv' | head -1)
K=$(find gpurun_out/$T -name 'run_kernel_trace.csv' | head -1)
python tools/prof_summary.py "$S" gpurun_out/$T/summary.md > /dev/null 2>&1 || true
python tools/fp32_layers.py "$K" ${PROF_B:-64} ${PROF_BLOCK:-1} > gpurun_out/$T/layers.txt 2>&1 || true
tail -3 gpurun_out/$T/layers.txt
