#!/bin/bash
# rocprofv3 kernel trace + stats of the headline command WITH its instrumented pass (face_groups=1,
# one launch per layer over the batch), so the summary's last-launch average checks roofline.per_launch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
T=r6prof
mkdir -p gpurun_out/$T
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$T -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --compare '' --host-pipeline 0 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
S=$(find gpurun_out/$T -name 'run_kernel_stats.csv' | head -1)
K=$(find gpurun_out/$T -name 'run_kernel_trace.csv' | head -1)
tail -1 gpurun_out/$T/bench.json > gpurun_out/$T/line.json
python tools/prof_summary.py "$S" gpurun_out/$T/summary.md gpurun_out/$T/line.json > /dev/null 2>&1 || true
python tools/fp32_layers.py "$K" 64 1 > gpurun_out/$T/layers.txt 2>&1 || true
tail -12 gpurun_out/$T/summary.md
tail -3 gpurun_out/$T/layers.txt
